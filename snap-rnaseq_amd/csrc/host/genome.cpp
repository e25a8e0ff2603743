// genome.cpp -- whole-genome byte string with contig padding (reference semantics of
// SNAPLib/Genome.{h,cpp} and SNAPLib/FASTA.cpp), plus a deterministic synthetic
// genome generator standing in for GRCh38 data that is not available offline.
#include "internal.h"

#include <cctype>
#include <cstdio>
#include <cstring>
#include <mutex>

namespace snapgpu {

static thread_local std::string g_lastError;
void setError(const std::string &msg) { g_lastError = msg; }

void Genome::reserve(uint64_t n) { buf.reserve(n + 2 * kGenomeGuard); }

void Genome::startPiece(const std::string &name) {
    // Genome::startPiece (Genome.cpp:80-108): the piece begins at the current end.
    pieceOffsets.push_back(nBases);
    pieceNames.push_back(name);
}

void Genome::append(const char *data, size_t len) {
    if (buf.empty()) buf.assign(kGenomeGuard, 'n');
    buf.insert(buf.end(), data, data + len);
    nBases += (uint32_t)len;
}

void Genome::appendPadding() {
    std::string pad(chromosomePadding, 'n');
    append(pad.data(), pad.size());
}

void Genome::finish() {
    if (buf.empty()) buf.assign(kGenomeGuard, 'n');
    buf.insert(buf.end(), kGenomeGuard, 'n');
}

Rng::Rng(uint64_t seed) {
    uint64_t x = seed;
    for (int i = 0; i < 4; i++) {   // splitmix64
        x += 0x9e3779b97f4a7c15ull;
        uint64_t z = x;
        z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
        z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
        s[i] = z ^ (z >> 31);
    }
}

static inline uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }

uint64_t Rng::next() {
    const uint64_t result = rotl(s[1] * 5, 7) * 9;
    const uint64_t t = s[1] << 17;
    s[2] ^= s[0]; s[3] ^= s[1]; s[1] ^= s[2]; s[0] ^= s[3];
    s[2] ^= t;
    s[3] = rotl(s[3], 45);
    return result;
}

}  // namespace snapgpu

using namespace snapgpu;

extern "C" {

const char *snapgpu_last_error(void) { return g_lastError.c_str(); }
int snapgpu_abi_version(void) { return SNAPGPU_ABI_VERSION; }

snapgpu_genome_t *snapgpu_genome_from_fasta(const char *path, uint32_t chromosomePadding) {
    // Restates ReadFASTAGenome (FASTA.cpp:31-130), including its 4096-byte fgets
    // line buffer, the name cut at the first blank/tab, upper-casing and N -> 'n'.
    FILE *f = fopen(path, "r");
    if (!f) { setError(std::string("cannot open FASTA ") + path); return nullptr; }
    auto *g = new snapgpu_genome_t();
    g->chromosomePadding = chromosomePadding;
    fseek(f, 0, SEEK_END);
    long size = ftell(f);
    fseek(f, 0, SEEK_SET);
    g->reserve((uint64_t)size + 64ull * chromosomePadding);
    char line[4096];
    while (fgets(line, sizeof(line), f)) {
        if (line[0] == '>') {
            g->appendPadding();
            char *space = strchr(line, ' ');
            char *tab = strchr(line, '\t');
            char *end = space ? (tab ? (space < tab ? space : tab) : space) : tab;
            if (!end) end = line + strlen(line) - 1;
            *end = '\0';
            g->startPiece(line + 1);
        } else {
            char *nl = strchr(line, '\n');
            if (nl) *nl = 0;
            size_t len = strlen(line);
            for (size_t i = 0; i < len; i++) {
                line[i] = (char)toupper((unsigned char)line[i]);
                if (line[i] == 'N') line[i] = 'n';
            }
            g->append(line, len);
        }
    }
    fclose(f);
    g->appendPadding();
    g->finish();
    return g;
}

snapgpu_genome_t *snapgpu_genome_synthetic(const snapgpu_synth_genome_params_t *p) {
    if (!p || p->totalBases == 0 || p->nContigs == 0) { setError("bad synthetic genome params"); return nullptr; }
    Rng rng(p->seed);
    static const char kBases[4] = {'A', 'C', 'G', 'T'};
    // Repeat families: consensus length in {300, 1000, 6000}, copy weight in
    // [2, 1000] with a heavy tail (u^4) -- a stand-in for the copy-number power law
    // of human interspersed repeats.  No libm: results are bit-identical everywhere.
    struct Family { std::string seq; uint64_t weight; };
    std::vector<Family> fam(p->nRepeatFamilies);
    uint64_t totalWeight = 0;
    double meanFamLen = 0;
    for (auto &f : fam) {
        double u = rng.uniform();
        size_t len = u < 0.5 ? 300 : (u < 0.85 ? 1000 : 6000);
        f.seq.resize(len);
        for (auto &c : f.seq) c = kBases[rng.next() >> 62];
        double w = rng.uniform();
        f.weight = 2 + (uint64_t)(998.0 * w * w * w * w);
        totalWeight += f.weight;
        meanFamLen += (double)f.weight * (double)len;
    }
    if (totalWeight) meanFamLen /= (double)totalWeight;
    const double meanBackground = 800.0;
    double meanCopy = meanFamLen * 0.75;        // copies are random fragments >= half the consensus
    double frac = p->nRepeatFamilies ? p->repeatFraction : 0.0;
    double pRepeat = frac <= 0 ? 0.0 : frac * meanBackground / (meanCopy * (1 - frac) + frac * meanBackground);

    auto *g = new snapgpu_genome_t();
    g->chromosomePadding = p->chromosomePadding;
    g->reserve(p->totalBases + (uint64_t)(p->nContigs + 1) * p->chromosomePadding);
    std::vector<uint64_t> contigLen(p->nContigs);
    uint64_t remaining = p->totalBases;
    for (uint32_t c = 0; c < p->nContigs; c++) {
        if (c + 1 == p->nContigs) { contigLen[c] = remaining; break; }
        uint64_t base = p->totalBases / p->nContigs;
        uint64_t len = base - base / 5 + rng.below(base / 5 * 2 + 1);
        if (len > remaining) len = remaining;
        contigLen[c] = len;
        remaining -= len;
    }
    std::string contig, copy;
    for (uint32_t c = 0; c < p->nContigs; c++) {
        contig.clear();
        contig.reserve(contigLen[c] + 8192);
        while (contig.size() < contigLen[c]) {
            double u = rng.uniform();
            if (p->nRunFraction > 0 && u < p->nRunFraction / 500.0) {
                size_t n = 10 + rng.below(1990);
                contig.append(n, 'N');
            } else if (rng.uniform() < pRepeat && !fam.empty()) {
                uint64_t r = rng.below(totalWeight);
                size_t fi = 0;
                while (r >= fam[fi].weight) { r -= fam[fi].weight; fi++; }
                const std::string &cons = fam[fi].seq;
                size_t flen = cons.size() / 2 + rng.below(cons.size() / 2 + 1);
                size_t start = rng.below(cons.size() - flen + 1);
                double div = p->maxDivergence * rng.uniform();
                copy.clear();
                for (size_t i = start; i < start + flen; i++) {
                    double v = rng.uniform();
                    if (v < div * 0.9) {
                        char b;
                        do { b = kBases[rng.next() >> 62]; } while (b == cons[i]);
                        copy.push_back(b);
                    } else if (v < div * 0.95) {
                        // deletion
                    } else if (v < div) {
                        copy.push_back(cons[i]);
                        copy.push_back(kBases[rng.next() >> 62]);
                    } else {
                        copy.push_back(cons[i]);
                    }
                }
                if (rng.next() >> 63) {   // reverse-complement copy
                    std::string rc(copy.rbegin(), copy.rend());
                    for (auto &ch : rc) ch = ch == 'A' ? 'T' : ch == 'C' ? 'G' : ch == 'G' ? 'C' : 'A';
                    copy.swap(rc);
                }
                contig += copy;
            } else {
                size_t n = 1 + rng.below((uint64_t)(2 * meanBackground));
                for (size_t i = 0; i < n; i++) contig.push_back(kBases[rng.next() >> 62]);
            }
        }
        contig.resize(contigLen[c]);
        for (auto &ch : contig) if (ch == 'N') ch = 'n';   // FASTA.cpp:112-116
        g->appendPadding();
        g->startPiece("chr" + std::to_string(c + 1));
        g->append(contig.data(), contig.size());
    }
    g->appendPadding();
    g->finish();
    return g;
}

int snapgpu_genome_write_fasta(const snapgpu_genome_t *g, const char *path) {
    FILE *f = fopen(path, "w");
    if (!f) { setError(std::string("cannot write ") + path); return SNAPGPU_EIO; }
    for (size_t i = 0; i < g->pieceOffsets.size(); i++) {
        uint32_t start = g->pieceOffsets[i];
        uint32_t end = i + 1 < g->pieceOffsets.size() ? g->pieceOffsets[i + 1] - g->chromosomePadding
                                                      : g->nBases - g->chromosomePadding;
        fprintf(f, ">%s\n", g->pieceNames[i].c_str());
        const char *b = g->bases();
        for (uint32_t p = start; p < end; p += 80) {
            uint32_t n = end - p < 80 ? end - p : 80;
            std::string line(b + p, b + p + n);
            for (auto &ch : line) if (ch == 'n') ch = 'N';
            fputs(line.c_str(), f);
            fputc('\n', f);
        }
    }
    int ok = ferror(f) == 0;
    fclose(f);
    return ok ? SNAPGPU_OK : SNAPGPU_EIO;
}

void snapgpu_genome_free(snapgpu_genome_t *g) { delete g; }
uint32_t snapgpu_genome_nbases(const snapgpu_genome_t *g) { return g ? g->nBases : 0; }
const char *snapgpu_genome_bases(const snapgpu_genome_t *g) { return g ? g->bases() : nullptr; }
int snapgpu_genome_npieces(const snapgpu_genome_t *g) { return g ? (int)g->pieceOffsets.size() : 0; }
uint32_t snapgpu_genome_piece_offset(const snapgpu_genome_t *g, int i) { return g->pieceOffsets.at(i); }
const char *snapgpu_genome_piece_name(const snapgpu_genome_t *g, int i) { return g->pieceNames.at(i).c_str(); }

}  // extern "C"
