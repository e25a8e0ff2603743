// index.cpp -- seed index: CPU builder with the reference's lookup semantics,
// loader/saver of the reference on-disk format, host lookupSeed.
//
// Lookup semantics that every consumer (oracle, HIP kernels) relies on:
//   lookupSeed(seed) -> for each direction the list of genome offsets whose
//   seedLen bases equal the seed (FORWARD) or its reverse complement (RC),
//   singletons as one hit, larger sets in DESCENDING order
//   (GenomeIndex.cpp:971-1086, 546-619).
#include "internal.h"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <thread>

namespace snapgpu {

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

struct Rec { uint32_t low, pos; };

unsigned hwThreads(int n) {
    if (n > 0) return (unsigned)n;
    unsigned h = std::thread::hardware_concurrency();
    return h ? h : 4;
}

template <class F>
void parallelFor(unsigned nThreads, uint64_t n, F &&f) {
    std::vector<std::thread> ts;
    for (unsigned t = 0; t < nThreads; t++) {
        uint64_t b = n * t / nThreads, e = n * (t + 1) / nThreads;
        ts.emplace_back([=, &f] { f(t, b, e); });
    }
    for (auto &th : ts) th.join();
}

}  // namespace

extern "C" {

snapgpu_index_t *snapgpu_index_build(snapgpu_genome_t *genome, int seedLen, int nThreadsArg) {
    if (!genome || seedLen < 16 || seedLen > 31) { setError("index_build: seedLen must be 16..31"); delete genome; return nullptr; }
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

    // Pass 1: per-thread per-table counts of valid seeds.
    std::vector<std::vector<uint64_t>> counts(nThreads, std::vector<uint64_t>(nT, 0));
    parallelFor(nThreads, nPos, [&](unsigned t, uint64_t beg, uint64_t end) {
        auto &c = counts[t];
        for (uint64_t p = beg; p < end; p++) {
            int64_t f, r;
            if (!encodeSeed(b + p, L, &f, &r)) continue;
            int64_t canon = f > r ? r : f;   // isBiggerThanItsReverseComplement (Seed.h:89-91)
            c[(uint32_t)((uint64_t)canon >> 32)]++;
        }
    });
    std::vector<uint64_t> tableStart(nT + 1, 0);
    std::vector<std::vector<uint64_t>> cursor(nThreads, std::vector<uint64_t>(nT));
    for (uint32_t tb = 0; tb < nT; tb++) {
        uint64_t s = tableStart[tb];
        for (unsigned t = 0; t < nThreads; t++) { cursor[t][tb] = s; s += counts[t][tb]; }
        tableStart[tb + 1] = s;
    }
    std::vector<Rec> recs(tableStart[nT]);
    // Pass 2: scatter (low bases, position) by table.
    parallelFor(nThreads, nPos, [&](unsigned t, uint64_t beg, uint64_t end) {
        auto &cur = cursor[t];
        for (uint64_t p = beg; p < end; p++) {
            int64_t f, r;
            if (!encodeSeed(b + p, L, &f, &r)) continue;
            uint64_t canon = (uint64_t)(f > r ? r : f);
            recs[cur[(uint32_t)(canon >> 32)]++] = Rec{(uint32_t)canon, (uint32_t)p};
        }
    });
    // Pass 3: per table, sort by (key, position), build the closed hash table and a
    // table-local overflow run list.
    idx->tableSize.assign(nT, 0);
    idx->tableUsed.assign(nT, 0);
    std::vector<std::vector<uint32_t>> localSlots(nT), localOverflow(nT);
    parallelFor(nThreads, nT, [&](unsigned, uint64_t tb0, uint64_t tb1) {
        for (uint64_t tb = tb0; tb < tb1; tb++) {
            Rec *r0 = recs.data() + tableStart[tb], *r1 = recs.data() + tableStart[tb + 1];
            std::sort(r0, r1, [](const Rec &x, const Rec &y) { return x.low != y.low ? x.low < y.low : x.pos < y.pos; });
            uint64_t distinct = 0;
            for (Rec *q = r0; q < r1; q++) if (q == r0 || q->low != q[-1].low) distinct++;
            uint64_t size = distinct * 2 + 1;
            if (size < 101) size = 101;
            idx->tableSize[tb] = size;
            idx->tableUsed[tb] = distinct;
            auto &slots = localSlots[tb];
            slots.assign(3 * size, 0);
            for (uint64_t i = 0; i < size; i++) slots[3 * i + 1] = kInvalidLocation;   // HashTable.cpp:72-75
            auto &ovf = localOverflow[tb];
            std::vector<uint32_t> side[2];
            for (Rec *q = r0; q < r1;) {
                Rec *e = q;
                side[0].clear(); side[1].clear();
                while (e < r1 && e->low == q->low) {
                    int64_t f = 0, r = 0;
                    encodeSeed(b + e->pos, L, &f, &r);
                    side[f > r ? 1 : 0].push_back(e->pos);   // value1: seed itself, value2: its RC
                    e++;
                }
                uint32_t v[2];
                for (int s = 0; s < 2; s++) {
                    if (side[s].empty()) v[s] = kUnusedSide;
                    else if (side[s].size() == 1) v[s] = side[s][0];
                    else {
                        v[s] = nBases + (uint32_t)ovf.size();   // fixed up below with the table's base
                        ovf.push_back((uint32_t)side[s].size());
                        for (auto it = side[s].rbegin(); it != side[s].rend(); ++it) ovf.push_back(*it);
                    }
                }
                // Insert at the first free slot of Lookup's probe sequence.
                uint32_t key = q->low;
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
        }
    });
    // Assemble: concatenate tables and overflow runs.
    idx->tableBase.assign(nT, 0);
    uint64_t totalSlots = 0, totalOverflow = 0;
    std::vector<uint64_t> ovfBase(nT);
    for (uint32_t tb = 0; tb < nT; tb++) {
        idx->tableBase[tb] = totalSlots;
        totalSlots += idx->tableSize[tb];
        ovfBase[tb] = totalOverflow;
        totalOverflow += localOverflow[tb].size();
    }
    if ((uint64_t)nBases + totalOverflow > 0xfffffff0ull) { setError("overflow table namespace exhausted"); delete idx; return nullptr; }
    idx->slots.resize(3 * totalSlots);
    idx->overflow.resize(totalOverflow);
    parallelFor(nThreads, nT, [&](unsigned, uint64_t tb0, uint64_t tb1) {
        for (uint64_t tb = tb0; tb < tb1; tb++) {
            auto &s = localSlots[tb];
            for (uint64_t i = 0; i < idx->tableSize[tb]; i++) {
                for (int k = 1; k <= 2; k++) {
                    uint32_t v = s[3 * i + k];
                    if (s[3 * i + 1] != kInvalidLocation && v != kUnusedSide && v >= nBases) s[3 * i + k] = v + (uint32_t)ovfBase[tb];
                }
            }
            memcpy(idx->slots.data() + 3 * idx->tableBase[tb], s.data(), s.size() * 4);
            if (!localOverflow[tb].empty())
                memcpy(idx->overflow.data() + ovfBase[tb], localOverflow[tb].data(), localOverflow[tb].size() * 4);
            std::vector<uint32_t>().swap(s);
        }
    });
    for (uint32_t p = 0; p < nBases; p++) {
        char c = b[p];
        if (c != 'A' && c != 'C' && c != 'G' && c != 'T' && c != 'n') { idx->hasIupac = true; break; }
    }
    return idx;
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
    if (n != 6 || seedLen == 0) { setError("GenomeIndex: bad header"); return nullptr; }
    auto *idx = new snapgpu_index_t();
    idx->seedLen = seedLen;
    idx->nTables = nTables;
    idx->overflow.resize(ovfSize);
    f = fopen((d + "/OverflowTable").c_str(), "rb");
    if (!f || !readAll(f, idx->overflow.data(), (size_t)ovfSize * 4)) { if (f) fclose(f); setError("OverflowTable read failed"); delete idx; return nullptr; }
    fclose(f);
    f = fopen((d + "/GenomeIndexHash").c_str(), "rb");
    if (!f) { setError("cannot open GenomeIndexHash"); delete idx; return nullptr; }
    idx->tableBase.resize(nTables); idx->tableSize.resize(nTables); idx->tableUsed.resize(nTables);
    uint64_t total = 0;
    for (unsigned t = 0; t < nTables; t++) {
        uint32_t magic; uint64_t size, used;
        if (!readAll(f, &magic, 4) || !readAll(f, &size, 8) || !readAll(f, &used, 8) || magic != kHashMagic || size == 0) {
            fclose(f); setError("GenomeIndexHash: bad table header"); delete idx; return nullptr;
        }
        idx->tableBase[t] = total; idx->tableSize[t] = size; idx->tableUsed[t] = used;
        idx->slots.resize(3 * (total + size));
        if (!readAll(f, idx->slots.data() + 3 * total, size * 12)) { fclose(f); setError("GenomeIndexHash: short read"); delete idx; return nullptr; }
        total += size;
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
