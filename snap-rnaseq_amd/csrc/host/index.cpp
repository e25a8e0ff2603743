// index.cpp -- seed index: CPU builder with the reference's lookup semantics and table sizing,
// loader/saver of the reference on-disk format, a flat shared-memory form for multi-rank
// jobs (build once per node, map in every rank), host lookupSeed.
//
// Lookup semantics that every consumer (oracle, HIP kernels) relies on:
//   lookupSeed(seed) -> for each direction the list of genome offsets whose
//   seedLen bases equal the seed (FORWARD) or its reverse complement (RC),
//   singletons as one hit, larger sets in DESCENDING order
//   (GenomeIndex.cpp:971-1086, 546-619).
#include "internal.h"

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <thread>
#include <unistd.h>

namespace snapgpu {

Index::~Index() {
    delete genome;
    if (mapBase) munmap(mapBase, mapLen);
}

const uint32_t *lookupSlot(const Index &idx, uint32_t table, uint32_t key, uint32_t *nProbes) {
    // SNAPHashTable::Lookup, HashTable.h:74-105.
    const uint64_t size = idx.tableSize[table];
    const uint32_t *t = idx.slots.data() + 3 * idx.tableBase[table];
    uint64_t i = hashKey(key) % size;
    if (t[3 * i] == key && t[3 * i + 1] != kInvalidLocation) return t + 3 * i + 1;
    uint64_t probes = 0;
    for (;;) {
        probes++;
        if (probes > size + kQuadraticChainingDepth) { if (nProbes) *nProbes += (uint32_t)probes; return nullptr; }
        if (probes < kQuadraticChainingDepth) i = (i + probes * probes) % size;
        else i = (i + 1) % size;
        if (t[3 * i] == key || t[3 * i + 1] == kInvalidLocation) break;
    }
    if (nProbes) *nProbes += (uint32_t)probes;
    if (t[3 * i + 1] == kInvalidLocation) return nullptr;
    return t + 3 * i + 1;
}

// Seed encoding of Seed::Seed (Seed.h:38-51): first base in the highest bits.
static inline bool encodeSeed(const char *b, uint32_t L, int64_t *bases, int64_t *rc) {
    uint64_t f = 0, r = 0;
    for (uint32_t i = 0; i < L; i++) {
        int v = baseValue(b[i]);
        if (v > 3) return false;
        f |= (uint64_t)v << ((L - i - 1) * 2);
        r |= (uint64_t)(v ^ 3) << (i * 2);
    }
    *bases = (int64_t)f;
    *rc = (int64_t)r;
    return true;
}

}  // namespace snapgpu

using namespace snapgpu;

namespace {

unsigned hwThreads(int n) {
    if (n > 0) return (unsigned)n;
    return snapgpu::hostThreadBudget();   // threads.cpp: affinity, cgroup quota, ranks of the node
}

// f(thread, begin, end) over [0, n) in nThreads static slices
template <class F>
void parallelFor(unsigned nThreads, uint64_t n, F &&f) {
    std::vector<std::thread> ts;
    for (unsigned t = 0; t < nThreads; t++) {
        uint64_t b = n * t / nThreads, e = n * (t + 1) / nThreads;
        ts.emplace_back([=, &f] { f(t, b, e); });
    }
    for (auto &th : ts) th.join();
}

// f(item) over [0, n) with dynamic scheduling (hash tables differ in size by 10x and more)
template <class F>
void parallelEach(unsigned nThreads, uint64_t n, F &&f) {
    std::atomic<uint64_t> next{0};
    std::vector<std::thread> ts;
    for (unsigned t = 0; t < nThreads; t++)
        ts.emplace_back([&] {
            for (uint64_t i; (i = next++) < n;) f(i);
        });
    for (auto &th : ts) th.join();
}

// Every valid seed position of [beg, end) in genome order, as (position, canonical seed,
// seed > its RC): a rolling 2-bit encoding (Seed.h:38-51, isBiggerThanItsReverseComplement
// Seed.h:89-91) instead of re-encoding seedLen bases per position.
template <class F>
void forEachSeed(const char *b, uint32_t L, uint64_t beg, uint64_t end, F &&f) {
    const uint64_t mask = L == 32 ? ~0ull : ((1ull << (2 * L)) - 1);
    uint64_t fw = 0, rc = 0;
    uint32_t run = 0;
    // prime with the first L-1 bases of the first seed
    for (uint64_t p = beg; p < end + L - 1; p++) {
        const int v = baseValue(b[p]);
        if (v > 3) { run = 0; fw = rc = 0; continue; }
        fw = ((fw << 2) | (uint64_t)v) & mask;
        rc = (rc >> 2) | ((uint64_t)(v ^ 3) << (2 * (L - 1)));
        if (++run >= L) {
            const uint64_t start = p + 1 - L;
            if (start >= beg) f(start, fw > rc ? rc : fw, fw > rc);
        }
    }
}

}  // namespace

extern "C" {

// GenomeIndex::BuildIndexToDirectory (GenomeIndex.cpp:348-720) with the table sizing of
// allocateHashTables (GenomeIndex.cpp:294-346) under an exact bias table (ComputeBiasTable,
// GenomeIndex.cpp:1109-1243, as its exact-count mode computes it): table i gets
// (nBases * (1 + slack) / nTables) * bias_i slots, bias_i = (distinct_i / distinct) *
// (validSeeds / nBases) * nTables, at least 100 -- so the load factor and probe chains are the
// reference's.  Records go straight to their final places: per-table counts, a scatter of
// (key, position), a per-table sort, then tables and overflow runs written in place.
snapgpu_index_t *snapgpu_index_build_ex(snapgpu_genome_t *genome, int seedLen, int nThreadsArg, double slack) {
    if (!genome || seedLen < 16 || seedLen > 31) { setError("index_build: seedLen must be 16..31"); delete genome; return nullptr; }
    if (!(slack > 0)) slack = 0.3;   // GenomeIndex.cpp:208 default
    auto *idx = new snapgpu_index_t();
    idx->genome = genome;
    idx->seedLen = (uint32_t)seedLen;
    idx->nTables = 1u << ((seedLen - 16) * 2);
    const uint32_t L = (uint32_t)seedLen, nT = idx->nTables;
    const uint32_t nBases = genome->nBases;
    const char *b = genome->bases();
    if (nBases > 0xfffffff0u) { setError("genome too big"); delete idx; return nullptr; }
    // Positions indexed: [0, nBases - seedLen - 1), the last builder chunk's end in
    // GenomeIndex.cpp:433-437.
    const uint64_t nPos = nBases > L + 1 ? (uint64_t)nBases - L - 1 : 0;
    const unsigned nThreads = hwThreads(nThreadsArg);

    // Slices on 64-position bounds: the side bitmap below is written without atomics.
    std::vector<uint64_t> sb(nThreads + 1);
    for (unsigned t = 0; t <= nThreads; t++) sb[t] = t == nThreads ? nPos : ((nPos * t / nThreads) & ~63ull);
    // Pass 1: per-thread per-table counts of valid seeds; IUPAC scan.
    std::vector<std::vector<uint64_t>> counts(nThreads, std::vector<uint64_t>(nT, 0));
    std::atomic<bool> iupac{false};
    parallelFor(nThreads, nThreads, [&](unsigned, uint64_t t0, uint64_t t1) {
        for (uint64_t t = t0; t < t1; t++) {
            auto &c = counts[t];
            forEachSeed(b, L, sb[t], sb[t + 1], [&](uint64_t, uint64_t canon, bool) { c[(uint32_t)(canon >> 32)]++; });
            for (uint64_t p = sb[t]; p < sb[t + 1]; p++) {
                const char ch = b[p];
                if (ch != 'A' && ch != 'C' && ch != 'G' && ch != 'T' && ch != 'n') { iupac = true; break; }
            }
        }
    });
    for (uint64_t p = nPos; p < nBases; p++) {
        const char ch = b[p];
        if (ch != 'A' && ch != 'C' && ch != 'G' && ch != 'T' && ch != 'n') iupac = true;
    }
    idx->hasIupac = iupac;
    std::vector<uint64_t> recStart(nT + 1, 0);
    std::vector<std::vector<uint64_t>> cursor(nThreads, std::vector<uint64_t>(nT));
    for (uint32_t tb = 0; tb < nT; tb++) {
        uint64_t s = recStart[tb];
        for (unsigned t = 0; t < nThreads; t++) { cursor[t][tb] = s; s += counts[t][tb]; }
        recStart[tb + 1] = s;
    }
    const uint64_t validSeeds = recStart[nT];
    // Pass 2: scatter key << 32 | position by table; the side (value1 = the seed itself,
    // value2 = its RC, GenomeIndex.cpp:1444-1447) goes to a bitmap by position.
    std::unique_ptr<uint64_t[]> recs(new uint64_t[validSeeds ? validSeeds : 1]);
    std::unique_ptr<uint64_t[]> side(new uint64_t[nPos / 64 + 2]);
    memset(side.get(), 0, (nPos / 64 + 2) * 8);
    {
        uint64_t *R = recs.get(), *S = side.get();
        parallelFor(nThreads, nThreads, [&](unsigned, uint64_t t0, uint64_t t1) {
            for (uint64_t t = t0; t < t1; t++) {
                auto &cur = cursor[t];
                forEachSeed(b, L, sb[t], sb[t + 1], [&](uint64_t p, uint64_t canon, bool isRc) {
                    R[cur[(uint32_t)(canon >> 32)]++] = ((canon & 0xffffffffull) << 32) | p;
                    if (isRc) S[p >> 6] |= 1ull << (p & 63);
                });
            }
        });
    }
    // Pass 3: per table, sort by (key, position); count distinct keys and overflow words.
    std::vector<uint64_t> distinct(nT, 0), ovfWords(nT, 0);
    parallelEach(nThreads, nT, [&](uint64_t tb) {
        uint64_t *r0 = recs.get() + recStart[tb], *r1 = recs.get() + recStart[tb + 1];
        std::sort(r0, r1);
        const uint64_t *S = side.get();
        uint64_t d = 0, ow = 0;
        for (uint64_t *q = r0; q < r1;) {
            uint64_t *e = q;
            uint64_t n1 = 0;
            while (e < r1 && (*e >> 32) == (*q >> 32)) {
                const uint64_t p = *e & 0xffffffffull;
                n1 += (S[p >> 6] >> (p & 63)) & 1;
                e++;
            }
            const uint64_t n0 = (uint64_t)(e - q) - n1;
            if (n0 > 1) ow += 1 + n0;
            if (n1 > 1) ow += 1 + n1;
            d++;
            q = e;
        }
        distinct[tb] = d;
        ovfWords[tb] = ow;
    });
    uint64_t distinctTotal = 0;
    for (uint32_t tb = 0; tb < nT; tb++) distinctTotal += distinct[tb];
    // allocateHashTables sizing (see above)
    idx->tableSize.assign(nT, 0);
    idx->tableUsed.assign(nT, 0);
    idx->tableBase.assign(nT, 0);
    std::vector<uint64_t> ovfBase(nT + 1, 0);
    const uint64_t avgSize = (uint64_t)((double)nBases * (slack + 1.0) / nT);
    uint64_t totalSlots = 0;
    for (uint32_t tb = 0; tb < nT; tb++) {
        const double bias = distinctTotal ? ((double)distinct[tb] / (double)distinctTotal) *
                                                ((double)validSeeds / (double)nBases) * nT : 0.0;
        uint64_t size = (uint64_t)(unsigned)((double)avgSize * bias);
        if (size < 100) size = 100;
        if (size < distinct[tb] + 1) size = distinct[tb] + 1;   // Lookup needs an empty slot to stop
        idx->tableSize[tb] = size;
        idx->tableUsed[tb] = distinct[tb];
        idx->tableBase[tb] = totalSlots;
        totalSlots += size;
        ovfBase[tb + 1] = ovfBase[tb] + ovfWords[tb];
    }
    const uint64_t totalOverflow = ovfBase[nT];
    if ((uint64_t)nBases + totalOverflow > 0xfffffff0ull) { setError("overflow table namespace exhausted"); delete idx; return nullptr; }
    idx->slots.allocate(3 * totalSlots);
    idx->overflow.allocate(totalOverflow);
    // Pass 4: each table in place -- empty slots (HashTable.cpp:72-75), overflow runs
    // [count, hits descending] (GenomeIndex.cpp:546-619), keys at the first free slot of
    // Lookup's probe sequence.
    parallelEach(nThreads, nT, [&](uint64_t tb) {
        const uint64_t size = idx->tableSize[tb];
        uint32_t *slots = idx->slots.mut() + 3 * idx->tableBase[tb];
        for (uint64_t i = 0; i < size; i++) { slots[3 * i] = 0; slots[3 * i + 1] = kInvalidLocation; slots[3 * i + 2] = 0; }
        uint32_t *ovf = idx->overflow.mut();
        uint64_t op = ovfBase[tb];
        const uint64_t *S = side.get();
        const uint64_t *r0 = recs.get() + recStart[tb], *r1 = recs.get() + recStart[tb + 1];
        for (const uint64_t *q = r0; q < r1;) {
            const uint32_t key = (uint32_t)(*q >> 32);
            const uint64_t *e = q;
            uint64_t n[2] = {0, 0};
            uint32_t single[2] = {0, 0};
            while (e < r1 && (uint32_t)(*e >> 32) == key) {
                const uint64_t p = *e & 0xffffffffull;
                const int s = (int)((S[p >> 6] >> (p & 63)) & 1);
                n[s]++;
                single[s] = (uint32_t)p;
                e++;
            }
            uint32_t v[2];
            for (int s = 0; s < 2; s++) {
                if (n[s] == 0) v[s] = kUnusedSide;
                else if (n[s] == 1) v[s] = single[s];
                else {
                    v[s] = nBases + (uint32_t)op;
                    ovf[op++] = (uint32_t)n[s];
                    for (const uint64_t *x = e; x-- > q;) {   // descending positions
                        const uint64_t p = *x & 0xffffffffull;
                        if ((int)((S[p >> 6] >> (p & 63)) & 1) == s) ovf[op++] = (uint32_t)p;
                    }
                }
            }
            uint64_t i = hashKey(key) % size;
            if (slots[3 * i + 1] != kInvalidLocation) {
                uint64_t probes = 0;
                for (;;) {
                    probes++;
                    if (probes < kQuadraticChainingDepth) i = (i + probes * probes) % size;
                    else i = (i + 1) % size;
                    if (slots[3 * i + 1] == kInvalidLocation) break;
                }
            }
            slots[3 * i] = key; slots[3 * i + 1] = v[0]; slots[3 * i + 2] = v[1];
            q = e;
        }
    });
    return idx;
}

snapgpu_index_t *snapgpu_index_build(snapgpu_genome_t *genome, int seedLen, int nThreads) {
    return snapgpu_index_build_ex(genome, seedLen, nThreads, 0.3);
}

static bool readAll(FILE *f, void *dst, size_t n) { return fread(dst, 1, n, f) == n; }

snapgpu_index_t *snapgpu_index_load(const char *dir) {
    // GenomeIndex::loadFromDirectory (GenomeIndex.cpp:844-963).
    std::string d(dir);
    FILE *f = fopen((d + "/GenomeIndex").c_str(), "r");
    if (!f) { setError("cannot open " + d + "/GenomeIndex"); return nullptr; }
    unsigned major, minor, nTables, ovfSize, seedLen, padding;
    int n = fscanf(f, "%u %u %u %u %u %u", &major, &minor, &nTables, &ovfSize, &seedLen, &padding);
    fclose(f);
    if (n != 6 || seedLen == 0 || nTables == 0) { setError("GenomeIndex: bad header"); return nullptr; }
    auto *idx = new snapgpu_index_t();
    idx->seedLen = seedLen;
    idx->nTables = nTables;
    idx->overflow.allocate(ovfSize);
    f = fopen((d + "/OverflowTable").c_str(), "rb");
    if (!f || !readAll(f, idx->overflow.mut(), (size_t)ovfSize * 4)) { if (f) fclose(f); setError("OverflowTable read failed"); delete idx; return nullptr; }
    fclose(f);
    // GenomeIndexHash: per table {u32 magic, size_t size, size_t used, size x 12 B}
    // (HashTable.cpp:104-150, 180-215): headers first, then one allocation for all slots
    f = fopen((d + "/GenomeIndexHash").c_str(), "rb");
    if (!f) { setError("cannot open GenomeIndexHash"); delete idx; return nullptr; }
    idx->tableBase.resize(nTables); idx->tableSize.resize(nTables); idx->tableUsed.resize(nTables);
    uint64_t total = 0;
    std::vector<long> dataPos(nTables);
    for (unsigned t = 0; t < nTables; t++) {
        uint32_t magic; uint64_t size, used;
        if (!readAll(f, &magic, 4) || !readAll(f, &size, 8) || !readAll(f, &used, 8) || magic != kHashMagic || size == 0) {
            fclose(f); setError("GenomeIndexHash: bad table header"); delete idx; return nullptr;
        }
        idx->tableBase[t] = total; idx->tableSize[t] = size; idx->tableUsed[t] = used;
        dataPos[t] = ftell(f);
        if (fseek(f, (long)(size * 12), SEEK_CUR) != 0) { fclose(f); setError("GenomeIndexHash: short file"); delete idx; return nullptr; }
        total += size;
    }
    idx->slots.allocate(3 * total);
    for (unsigned t = 0; t < nTables; t++) {
        if (fseek(f, dataPos[t], SEEK_SET) != 0 ||
            !readAll(f, idx->slots.mut() + 3 * idx->tableBase[t], idx->tableSize[t] * 12)) {
            fclose(f); setError("GenomeIndexHash: short read"); delete idx; return nullptr;
        }
    }
    fclose(f);
    // Genome::loadFromFile (Genome.cpp:160-261).
    f = fopen((d + "/Genome").c_str(), "rb");
    if (!f) { setError("cannot open Genome"); delete idx; return nullptr; }
    unsigned nBases, nPieces;
    if (fscanf(f, "%u %u", &nBases, &nPieces) != 2) { fclose(f); setError("Genome: bad header"); delete idx; return nullptr; }
    fgetc(f);   // '\n'
    auto *g = new snapgpu_genome_t();
    g->chromosomePadding = padding;
    char line[512];
    for (unsigned i = 0; i < nPieces; i++) {
        if (!fgets(line, sizeof(line), f)) { fclose(f); delete g; setError("Genome: piece line"); delete idx; return nullptr; }
        char *sp = strchr(line, ' ');
        std::string name;
        if (sp) { name = sp + 1; if (!name.empty() && name.back() == '\n') name.pop_back(); *sp = 0; }
        g->pieceOffsets.push_back((uint32_t)strtoul(line, nullptr, 10));
        g->pieceNames.push_back(name);
    }
    g->buf.assign(kGenomeGuard, 'n');
    g->buf.resize(kGenomeGuard + (size_t)nBases);
    if (!readAll(f, g->buf.data() + kGenomeGuard, nBases)) { fclose(f); delete g; setError("Genome: short read"); delete idx; return nullptr; }
    fclose(f);
    g->nBases = nBases;
    g->finish();
    idx->genome = g;
    for (uint32_t p = 0; p < nBases; p++) {
        char c = g->bases()[p];
        if (c != 'A' && c != 'C' && c != 'G' && c != 'T' && c != 'n') { idx->hasIupac = true; break; }
    }
    return idx;
}

int snapgpu_index_save(const snapgpu_index_t *idx, const char *dir) {
    std::string d(dir);
    std::string cmd = "mkdir -p '" + d + "'";
    if (system(cmd.c_str()) != 0) { setError("mkdir failed"); return SNAPGPU_EIO; }
    FILE *f = fopen((d + "/GenomeIndex").c_str(), "w");
    if (!f) return SNAPGPU_EIO;
    fprintf(f, "%d %d %d %d %d %d", 1, 0, (int)idx->nTables, (int)idx->overflow.size(), (int)idx->seedLen,
            (int)idx->genome->chromosomePadding);
    fclose(f);
    f = fopen((d + "/OverflowTable").c_str(), "wb");
    if (!f) return SNAPGPU_EIO;
    fwrite(idx->overflow.data(), 4, idx->overflow.size(), f);
    fclose(f);
    f = fopen((d + "/GenomeIndexHash").c_str(), "wb");
    if (!f) return SNAPGPU_EIO;
    for (uint32_t t = 0; t < idx->nTables; t++) {
        uint64_t size = idx->tableSize[t], used = idx->tableUsed[t];
        fwrite(&kHashMagic, 4, 1, f);
        fwrite(&size, 8, 1, f);
        fwrite(&used, 8, 1, f);
        fwrite(idx->slots.data() + 3 * idx->tableBase[t], 12, size, f);
    }
    fclose(f);
    f = fopen((d + "/Genome").c_str(), "wb");
    if (!f) return SNAPGPU_EIO;
    const Genome *g = idx->genome;
    fprintf(f, "%d %d\n", (int)g->nBases, (int)g->pieceOffsets.size());
    for (size_t i = 0; i < g->pieceOffsets.size(); i++) {
        std::string name = g->pieceNames[i];
        for (auto &c : name) if (c == ' ') c = '_';
        fprintf(f, "%d %s\n", (int)g->pieceOffsets[i], name.c_str());
    }
    fwrite(g->bases(), 1, g->nBases, f);
    int ok = ferror(f) == 0;
    fclose(f);
    return ok ? SNAPGPU_OK : SNAPGPU_EIO;
}

// ----------------------------------------------------------- shared (flat) form
// One file, every section 4 KiB-aligned, so a rank can map it and use the tables in place:
// header | tableBase | tableSize | tableUsed | pieceOffsets | piece names (NUL-separated) |
// genome buffer (guard + bases + guard) | slots | overflow.
namespace {
struct SharedHeader {
    char magic[8];            // "SNAPGPU\1"
    uint32_t seedLen, nTables, nBases, padding, nPieces, hasIupac;
    uint64_t slotWords, ovfWords, genomeBytes, namesBytes;
    uint64_t off[8];          // tableBase, tableSize, tableUsed, pieces, names, genome, slots, overflow
    uint64_t total;
};
const char kSharedMagic[8] = {'S', 'N', 'A', 'P', 'G', 'P', 'U', 1};
uint64_t align4k(uint64_t x) { return (x + 4095) & ~4095ull; }
}  // namespace

int snapgpu_index_share(const snapgpu_index_t *idx, const char *path) {
    if (!idx || !path) return SNAPGPU_EINVAL;
    const Genome *g = idx->genome;
    std::string names;
    for (auto &s : g->pieceNames) { names += s; names += '\0'; }
    SharedHeader h{};
    memcpy(h.magic, kSharedMagic, 8);
    h.seedLen = idx->seedLen; h.nTables = idx->nTables; h.nBases = g->nBases; h.padding = g->chromosomePadding;
    h.nPieces = (uint32_t)g->pieceOffsets.size(); h.hasIupac = idx->hasIupac;
    h.slotWords = idx->slots.size(); h.ovfWords = idx->overflow.size();
    h.genomeBytes = (uint64_t)g->nBases + 2 * kGenomeGuard; h.namesBytes = names.size();
    const uint64_t sz[8] = {8ull * h.nTables, 8ull * h.nTables, 8ull * h.nTables, 4ull * h.nPieces, h.namesBytes,
                            h.genomeBytes, 4 * h.slotWords, 4 * h.ovfWords};
    uint64_t o = align4k(sizeof(SharedHeader));
    for (int i = 0; i < 8; i++) { h.off[i] = o; o = align4k(o + sz[i]); }
    h.total = o;
    const std::string tmp = std::string(path) + ".tmp";
    FILE *f = fopen(tmp.c_str(), "wb");
    if (!f) { setError(std::string("cannot write ") + tmp); return SNAPGPU_EIO; }
    const void *src[8] = {idx->tableBase.data(), idx->tableSize.data(), idx->tableUsed.data(), g->pieceOffsets.data(),
                          names.data(), g->bases() - kGenomeGuard, idx->slots.data(), idx->overflow.data()};
    bool ok = fwrite(&h, sizeof(h), 1, f) == 1;
    for (int i = 0; i < 8 && ok; i++) {
        ok = fseek(f, (long)h.off[i], SEEK_SET) == 0 && (sz[i] == 0 || fwrite(src[i], 1, sz[i], f) == sz[i]);
    }
    ok = ok && ftruncate(fileno(f), (off_t)h.total) == 0;
    ok = (fclose(f) == 0) && ok;
    if (!ok || rename(tmp.c_str(), path) != 0) { unlink(tmp.c_str()); setError("index_share: write failed"); return SNAPGPU_EIO; }
    return SNAPGPU_OK;
}

snapgpu_index_t *snapgpu_index_attach(const char *path) {
    const int fd = open(path, O_RDONLY);
    if (fd < 0) { setError(std::string("cannot open ") + path); return nullptr; }
    struct stat st;
    if (fstat(fd, &st) != 0 || (uint64_t)st.st_size < sizeof(SharedHeader)) { close(fd); setError("index_attach: short file"); return nullptr; }
    void *base = mmap(nullptr, (size_t)st.st_size, PROT_READ, MAP_SHARED, fd, 0);
    close(fd);
    if (base == MAP_FAILED) { setError("index_attach: mmap failed"); return nullptr; }
    const auto *h = (const SharedHeader *)base;
    if (memcmp(h->magic, kSharedMagic, 8) != 0 || h->total != (uint64_t)st.st_size) {
        munmap(base, (size_t)st.st_size);
        setError("index_attach: not a shared index file");
        return nullptr;
    }
    const char *B = (const char *)base;
    auto *idx = new snapgpu_index_t();
    idx->mapBase = base;
    idx->mapLen = (uint64_t)st.st_size;
    idx->seedLen = h->seedLen;
    idx->nTables = h->nTables;
    idx->hasIupac = h->hasIupac != 0;
    const uint64_t *tb = (const uint64_t *)(B + h->off[0]), *ts = (const uint64_t *)(B + h->off[1]),
                   *tu = (const uint64_t *)(B + h->off[2]);
    idx->tableBase.assign(tb, tb + h->nTables);
    idx->tableSize.assign(ts, ts + h->nTables);
    idx->tableUsed.assign(tu, tu + h->nTables);
    auto *g = new snapgpu_genome_t();
    g->nBases = h->nBases;
    g->chromosomePadding = h->padding;
    const uint32_t *po = (const uint32_t *)(B + h->off[3]);
    g->pieceOffsets.assign(po, po + h->nPieces);
    const char *nm = B + h->off[4];
    for (uint32_t i = 0; i < h->nPieces; i++) { g->pieceNames.emplace_back(nm); nm += g->pieceNames.back().size() + 1; }
    g->ext = B + h->off[5];
    idx->genome = g;
    idx->slots.view((const uint32_t *)(B + h->off[6]), h->slotWords);
    idx->overflow.view((const uint32_t *)(B + h->off[7]), h->ovfWords);
    return idx;
}

void snapgpu_index_free(snapgpu_index_t *idx) { delete idx; }

int snapgpu_index_get_info(const snapgpu_index_t *idx, snapgpu_index_info_t *info) {
    if (!idx || !info) return SNAPGPU_EINVAL;
    memset(info, 0, sizeof(*info));
    info->nBases = idx->genome->nBases;
    info->seedLen = idx->seedLen;
    info->nHashTables = idx->nTables;
    info->chromosomePadding = idx->genome->chromosomePadding;
    info->overflowTableSize = idx->overflow.size();
    for (uint32_t t = 0; t < idx->nTables; t++) { info->totalHashSlots += idx->tableSize[t]; info->totalUsedSlots += idx->tableUsed[t]; }
    info->nPieces = (int32_t)idx->genome->pieceOffsets.size();
    info->hasIupac = idx->hasIupac;
    return SNAPGPU_OK;
}

int snapgpu_index_get_view(const snapgpu_index_t *idx, snapgpu_index_view_t *v) {
    if (!idx || !v) return SNAPGPU_EINVAL;
    memset(v, 0, sizeof(*v));
    v->slots = idx->slots.data();
    v->tableBase = idx->tableBase.data();
    v->tableSize = idx->tableSize.data();
    v->overflow = idx->overflow.data();
    v->genome = idx->genome->bases();
    v->pieceOffsets = idx->genome->pieceOffsets.data();
    v->nBases = idx->genome->nBases;
    v->seedLen = idx->seedLen;
    v->nHashTables = idx->nTables;
    v->chromosomePadding = idx->genome->chromosomePadding;
    v->nPieces = (int32_t)idx->genome->pieceOffsets.size();
    v->overflowTableSize = idx->overflow.size();
    return SNAPGPU_OK;
}

const snapgpu_genome_t *snapgpu_index_genome(const snapgpu_index_t *idx) {
    return idx ? static_cast<const snapgpu_genome_t *>(idx->genome) : nullptr;   // always allocated as one
}

int snapgpu_index_lookup(const snapgpu_index_t *idx, const char *seedBases, uint32_t nHits[2],
                         uint32_t *hitsFwd, uint32_t *hitsRc, uint32_t cap) {
    // GenomeIndex::lookupSeed + fillInLookedUpResults (GenomeIndex.cpp:971-1086),
    // unconstrained [0, 0xffffffff] window.
    int64_t f, r;
    nHits[0] = nHits[1] = 0;
    if (!encodeSeed(seedBases, idx->seedLen, &f, &r)) return SNAPGPU_EINVAL;
    bool comp = f > r;
    int64_t canon = comp ? r : f;
    uint32_t table = (uint32_t)((uint64_t)canon >> 32);
    if (table >= idx->nTables) return SNAPGPU_EINVAL;
    const uint32_t *e = lookupSlot(*idx, table, (uint32_t)canon, nullptr);
    if (!e) return SNAPGPU_OK;
    const uint32_t nBases = idx->genome->nBases;
    auto fill = [&](uint32_t v, uint32_t *n, uint32_t *out) {
        if (v < nBases) { *n = 1; if (cap) out[0] = v; }
        else if (v == kUnusedSide) *n = 0;
        else {
            uint32_t off = v - nBases;
            *n = idx->overflow[off];
            for (uint32_t i = 0; i < *n && i < cap; i++) out[i] = idx->overflow[off + 1 + i];
        }
    };
    fill(comp ? e[1] : e[0], &nHits[0], hitsFwd);
    if (f == r) {   // palindrome: RC hits are the forward hits (GenomeIndex.cpp:1003-1006)
        nHits[1] = nHits[0];
        for (uint32_t i = 0; i < nHits[0] && i < cap; i++) hitsRc[i] = hitsFwd[i];
    } else {
        fill(comp ? e[0] : e[1], &nHits[1], hitsRc);
    }
    return SNAPGPU_OK;
}

}  // extern "C"
