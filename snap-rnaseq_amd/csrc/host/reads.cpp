// reads.cpp -- read batches: wgsim-like simulator, FASTQ in/out, caller arrays.
#include "internal.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

using namespace snapgpu;

namespace {

snapgpu_reads_t *allocReads(uint64_t n, uint64_t totalBytes, bool truth, bool zero = true) {
    auto *r = new snapgpu_reads_t();
    r->n = n;
    r->totalBytes = totalBytes;
    bool pb = false, pq = false;
    r->bases = (char *)hostAlloc(totalBytes + 64, &pb, zero);
    r->quals = (char *)hostAlloc(totalBytes + 64, &pq, zero);
    r->hostFlags = (pb ? 1u : 0u) | (pq ? 2u : 0u);
    r->offsets = new uint64_t[n + 1]();
    r->lengths = new uint32_t[n + 1]();
    r->truthLocation = truth ? new uint32_t[n + 1]() : nullptr;
    r->truthDirection = truth ? new uint8_t[n + 1]() : nullptr;
    return r;
}

inline char complement(char c) {
    switch (c) { case 'A': return 'T'; case 'C': return 'G'; case 'G': return 'C'; case 'T': return 'A'; default: return 'N'; }
}

}  // namespace

extern "C" {

snapgpu_reads_t *snapgpu_reads_synthetic(const snapgpu_genome_t *g, const snapgpu_synth_reads_params_t *p) {
    if (!g || !p || p->readLength == 0 || g->pieceOffsets.empty()) { setError("bad read params"); return nullptr; }
    const uint32_t L = p->readLength;
    snapgpu_reads_t *r = allocReads(p->nReads, p->nReads * (uint64_t)L, true);
    Rng rng(p->seed);
    static const char kBases[4] = {'A', 'C', 'G', 'T'};
    // contig extents
    std::vector<uint64_t> cStart, cLen, cum;
    uint64_t total = 0;
    for (size_t i = 0; i < g->pieceOffsets.size(); i++) {
        uint64_t s = g->pieceOffsets[i];
        uint64_t e = i + 1 < g->pieceOffsets.size() ? g->pieceOffsets[i + 1] - g->chromosomePadding : g->nBases - g->chromosomePadding;
        cStart.push_back(s); cLen.push_back(e - s);
        total += e - s > 2 * L + 64 ? e - s : 0;
        cum.push_back(total);
    }
    if (total == 0) { setError("contigs too short"); snapgpu_reads_free(r); return nullptr; }
    const char *gb = g->bases();
    std::string frag;
    for (uint64_t i = 0; i < p->nReads; i++) {
        char *out = r->bases + i * L;
        r->offsets[i] = i * L;
        r->lengths[i] = L;
        memset(r->quals + i * L, (int)p->qualityChar, L);
        if (p->randomReadFraction > 0 && rng.uniform() < p->randomReadFraction) {
            for (uint32_t j = 0; j < L; j++) out[j] = kBases[rng.next() >> 62];
            r->truthLocation[i] = kInvalidLocation;
            continue;
        }
        for (int attempt = 0;; attempt++) {
            uint64_t x = rng.below(total);
            size_t c = 0;
            while (cum[c] <= x) c++;
            uint64_t start = cStart[c] + rng.below(cLen[c] - L - 48);
            // haplotype walk with mutations (wgsim: substitution / indel with extension)
            frag.clear();
            uint64_t pos = start;
            while (frag.size() < L) {
                char base = gb[pos];
                if (base == 'n') base = 'N';
                double u = rng.uniform();
                if (u < p->mutationRate) {
                    if (rng.uniform() < p->indelFraction) {
                        uint32_t len = 1;
                        while (rng.uniform() < p->indelExtend && len < 10) len++;
                        if (rng.next() >> 63) { pos += len; continue; }        // deletion
                        frag.push_back(base);
                        for (uint32_t k = 0; k < len && frag.size() < L; k++) frag.push_back(kBases[rng.next() >> 62]);
                        pos++;
                        continue;
                    }
                    char nb;
                    do { nb = kBases[rng.next() >> 62]; } while (nb == base);
                    frag.push_back(nb);
                } else {
                    frag.push_back(base);
                }
                pos++;
            }
            frag.resize(L);
            uint32_t nN = 0;
            for (char ch : frag) nN += ch == 'N';
            if (nN > L / 20 && attempt < 16) continue;   // wgsim -A 0.05: discard ambiguous reads
            bool rc = rng.next() >> 63;
            if (rc) {
                std::string t(frag.rbegin(), frag.rend());
                for (auto &ch : t) ch = complement(ch);
                frag.swap(t);
            }
            for (uint32_t j = 0; j < L; j++) {
                char ch = frag[j];
                if (ch != 'N' && rng.uniform() < p->baseErrorRate) {
                    char nb;
                    do { nb = kBases[rng.next() >> 62]; } while (nb == ch);
                    ch = nb;
                }
                out[j] = ch;
            }
            r->truthLocation[i] = (uint32_t)start;
            r->truthDirection[i] = rc ? 1 : 0;
            break;
        }
    }
    return r;
}

// wgsim-like pairs: a fragment of length insert ~ N(insertMean, insertSd) (Irwin-Hall, no libm)
// walked through the mutated haplotype; read 0 = the fragment's first L bases, read 1 = the
// reverse complement of its last L, the whole fragment from either strand; base errors per read.
// Truth: fragment start and the strand of read 0.
int snapgpu_reads_synthetic_pairs(const snapgpu_genome_t *g, const snapgpu_synth_reads_params_t *p, uint32_t insertMean,
                                  uint32_t insertSd, snapgpu_reads_t **reads0, snapgpu_reads_t **reads1) {
    if (!g || !p || !reads0 || !reads1 || p->readLength == 0 || g->pieceOffsets.empty() || insertMean < p->readLength) {
        setError("bad pair params");
        return SNAPGPU_EINVAL;
    }
    const uint32_t L = p->readLength;
    const uint64_t n = p->nReads;
    snapgpu_reads_t *R[2] = {allocReads(n, n * (uint64_t)L, true), allocReads(n, n * (uint64_t)L, true)};
    Rng rng(p->seed);
    static const char kBases[4] = {'A', 'C', 'G', 'T'};
    const uint32_t maxIns = insertMean + 6 * insertSd + 1;
    std::vector<uint64_t> cStart, cLen, cum;
    uint64_t total = 0;
    for (size_t i = 0; i < g->pieceOffsets.size(); i++) {
        uint64_t st = g->pieceOffsets[i];
        uint64_t e = i + 1 < g->pieceOffsets.size() ? g->pieceOffsets[i + 1] - g->chromosomePadding : g->nBases - g->chromosomePadding;
        cStart.push_back(st); cLen.push_back(e - st);
        total += e - st > 2ull * maxIns + 64 ? e - st : 0;
        cum.push_back(total);
    }
    if (total == 0) { setError("contigs too short"); snapgpu_reads_free(R[0]); snapgpu_reads_free(R[1]); return SNAPGPU_EINVAL; }
    const char *gb = g->bases();
    std::string frag, t;
    for (uint64_t i = 0; i < n; i++) {
        for (int k = 0; k < 2; k++) {
            R[k]->offsets[i] = i * L;
            R[k]->lengths[i] = L;
            memset(R[k]->quals + i * L, (int)p->qualityChar, L);
        }
        double z = 0;
        for (int j = 0; j < 12; j++) z += rng.uniform();
        int64_t ins = (int64_t)insertMean + (int64_t)((z - 6.0) * (double)insertSd);
        if (ins < (int64_t)L) ins = L;
        if (ins > (int64_t)maxIns) ins = maxIns;
        for (int attempt = 0;; attempt++) {
            uint64_t x = rng.below(total);
            size_t c = 0;
            while (cum[c] <= x) c++;
            const uint64_t start = cStart[c] + rng.below(cLen[c] - maxIns - 48);
            frag.clear();
            uint64_t pos = start;
            while (frag.size() < (size_t)ins) {
                char base = gb[pos];
                if (base == 'n') base = 'N';
                const double u = rng.uniform();
                if (u < p->mutationRate) {
                    if (rng.uniform() < p->indelFraction) {
                        uint32_t len = 1;
                        while (rng.uniform() < p->indelExtend && len < 10) len++;
                        if (rng.next() >> 63) { pos += len; continue; }
                        frag.push_back(base);
                        for (uint32_t k = 0; k < len && frag.size() < (size_t)ins; k++) frag.push_back(kBases[rng.next() >> 62]);
                        pos++;
                        continue;
                    }
                    char nb;
                    do { nb = kBases[rng.next() >> 62]; } while (nb == base);
                    frag.push_back(nb);
                } else frag.push_back(base);
                pos++;
            }
            frag.resize((size_t)ins);
            uint32_t nN = 0;
            for (char ch : frag) nN += ch == 'N';
            if (nN > (uint32_t)ins / 20 && attempt < 16) continue;
            const bool rc = rng.next() >> 63;
            if (rc) {
                t.assign(frag.rbegin(), frag.rend());
                for (auto &ch : t) ch = complement(ch);
                frag.swap(t);
            }
            std::string m[2];
            m[0] = frag.substr(0, L);
            t.assign(frag.rbegin(), frag.rbegin() + L);
            for (auto &ch : t) ch = complement(ch);
            m[1] = t;
            for (int k = 0; k < 2; k++) {
                char *out = R[k]->bases + i * L;
                for (uint32_t j = 0; j < L; j++) {
                    char ch = m[k][j];
                    if (ch != 'N' && rng.uniform() < p->baseErrorRate) {
                        char nb;
                        do { nb = kBases[rng.next() >> 62]; } while (nb == ch);
                        ch = nb;
                    }
                    out[j] = ch;
                }
                R[k]->truthLocation[i] = (uint32_t)start;
                R[k]->truthDirection[i] = (uint8_t)(rc ^ (k == 1));
            }
            break;
        }
    }
    *reads0 = R[0];
    *reads1 = R[1];
    return SNAPGPU_OK;
}

snapgpu_reads_t *snapgpu_reads_from_arrays(uint64_t n, const char *bases, const char *quals,
                                           const uint64_t *offsets, const uint32_t *lengths) {
    uint64_t total = 0;
    for (uint64_t i = 0; i < n; i++) total += lengths[i];
    snapgpu_reads_t *r = allocReads(n, total, false);
    uint64_t o = 0;
    for (uint64_t i = 0; i < n; i++) {
        memcpy(r->bases + o, bases + offsets[i], lengths[i]);
        memcpy(r->quals + o, quals + offsets[i], lengths[i]);
        r->offsets[i] = o;
        r->lengths[i] = lengths[i];
        o += lengths[i];
    }
    return r;
}

}  // extern "C"

namespace snapgpu {

// reads[offsets[i] .. + lengths[i]) of the parent's buffers, without copying them: the view shares
// the parent's bases, qualities and byte size (the kernels' uploads and the +64 slack past the last
// read are the parent's), owns only its offsets and lengths, and must not outlive the parent.
// A small subset (under a quarter of the parent's bytes: the chimeric fallback ends, a few
// thousand reads of a 500k-pair batch) is packed into its own buffers instead, since the aligner
// uploads a view's whole parent (measured: +3.8 ms per 500k-pair paired batch as a view).
snapgpu_reads_t *readsView(const snapgpu_reads_t *parent, uint64_t n, const uint64_t *offsets, const uint32_t *lengths) {
    uint64_t useful = 0;
    for (uint64_t i = 0; i < n; i++) useful += lengths[i];
    if (4 * useful < parent->totalBytes) return snapgpu_reads_from_arrays(n, parent->bases, parent->quals, offsets, lengths);
    auto *r = new snapgpu_reads_t();
    r->n = n;
    r->totalBytes = parent->totalBytes;
    r->bases = parent->bases;
    r->quals = parent->quals;
    r->hostFlags = (parent->hostFlags & 3u) | kReadsView;
    r->offsets = new uint64_t[n + 1]();
    r->lengths = new uint32_t[n + 1]();
    if (n) {
        memcpy(r->offsets, offsets, n * 8);
        memcpy(r->lengths, lengths, n * 4);
    }
    return r;
}

}  // namespace snapgpu

extern "C" {

snapgpu_reads_t *snapgpu_reads_from_fastq(const char *path) {
    // FASTQReader::getNextRead (FASTQ.cpp:196-253): 4-line records, id = header line without
    // '@' (trailing CR/LF removed), bases, '+' line, qualities (a quality line shorter than the
    // bases leaves NUL bytes: SAM's %.*s then ends early, as the reference's would).  A trailing
    // partial record is ignored.  The file is mapped and parsed in parallel (this rank's host thread
    // budget): the newline positions per byte range, then per record its lengths, prefix sums,
    // and the copies into the batch -- 1M 100-bp reads: 306 ms with one thread and per-line strings.
    const int fd = open(path, O_RDONLY);
    if (fd < 0) { setError(std::string("cannot open ") + path); return nullptr; }
    struct stat sb;
    if (fstat(fd, &sb) != 0) { close(fd); setError(std::string("cannot stat ") + path); return nullptr; }
    const uint64_t size = (uint64_t)sb.st_size;
    const char *base = nullptr;
    if (size) {
        void *m = mmap(nullptr, size, PROT_READ, MAP_PRIVATE, fd, 0);
        if (m == MAP_FAILED) { close(fd); setError(std::string("cannot map ") + path); return nullptr; }
        base = (const char *)m;
    }
    close(fd);
    struct Unmap {
        const char *p; uint64_t n;
        ~Unmap() { if (p) munmap(const_cast<char *>(p), n); }
    } unmap{base, size};
    const unsigned nt = size < (8u << 20) ? 1u : hostThreads(16);
    auto parallel = [&](uint64_t n, auto &&fn) {
        if (nt == 1 || n < 4096) { fn(0u, (uint64_t)0, n); return; }
        std::vector<std::thread> th;
        for (unsigned t = 0; t < nt; t++) th.emplace_back([&, t] { fn(t, n * t / nt, n * (t + 1) / nt); });
        for (auto &x : th) x.join();
    };
    // newline positions, per byte range, then concatenated in file order
    std::vector<std::vector<uint64_t>> part(nt);
    parallel(size, [&](unsigned t, uint64_t b, uint64_t e) {
        auto &v = part[t];
        v.reserve((e - b) / 48 + 16);
        for (const char *p = base + b, *end = base + e; p < end;) {
            const char *q = (const char *)memchr(p, '\n', end - p);
            if (!q) break;
            v.push_back((uint64_t)(q - base));
            p = q + 1;
        }
    });
    std::vector<uint64_t> nl;
    {
        uint64_t tot = 0;
        for (auto &v : part) tot += v.size();
        nl.reserve(tot + 1);
        for (auto &v : part) { nl.insert(nl.end(), v.begin(), v.end()); std::vector<uint64_t>().swap(v); }
    }
    const uint64_t nLines = nl.size() + ((nl.empty() ? size : size - nl.back() - 1) > 0 ? 1 : 0);
    if (nLines > nl.size()) nl.push_back(size);   // the last line, without its newline
    const uint64_t n = nLines / 4;
    // line i: [start, end), cut at its first NUL byte (the C-string reading of FASTQReader's lines: a
    // reader never hands the aligner a NUL inside a read) and without its trailing CR/LF bytes
    auto line = [&](uint64_t i, uint64_t &b, uint64_t &e) {
        b = i ? nl[i - 1] + 1 : 0;
        e = nl[i];
        if (const char *z = (const char *)memchr(base + b, 0, e - b)) e = (uint64_t)(z - base);
        while (e > b && (base[e - 1] == '\r' || base[e - 1] == '\n')) e--;
    };
    std::vector<uint32_t> blen(n + 1, 0), qlen(n + 1, 0), ilen(n + 1, 0);
    std::vector<uint64_t> badAt(nt, n);
    parallel(n, [&](unsigned t, uint64_t a, uint64_t z) {
        for (uint64_t r = a; r < z; r++) {
            uint64_t b, e;
            line(4 * r, b, e);
            if (e == b || base[b] != '@') { badAt[t] = std::min(badAt[t], r); break; }
            ilen[r] = (uint32_t)(e - b - 1);
            line(4 * r + 1, b, e);
            blen[r] = (uint32_t)(e - b);
            line(4 * r + 3, b, e);
            qlen[r] = (uint32_t)(e - b);
        }
    });
    if (*std::min_element(badAt.begin(), badAt.end()) < n) {
        setError(std::string("FASTQ record without '@' header in ") + path);
        return nullptr;
    }
    uint64_t total = 0, idTotal = 0;
    for (uint64_t r = 0; r < n; r++) { total += blen[r]; idTotal += ilen[r]; }
    snapgpu_reads_t *rd = allocReads(n, total, false, /*zero=*/false);
    rd->ids = new char[idTotal + 1]();
    rd->idOffsets = new uint64_t[n + 1]();
    rd->idLengths = new uint32_t[n + 1]();
    for (uint64_t r = 0, o = 0, io = 0; r < n; r++) {
        rd->offsets[r] = o;
        rd->lengths[r] = blen[r];
        o += blen[r];
        rd->idOffsets[r] = io;
        rd->idLengths[r] = ilen[r];
        io += ilen[r];
    }
    parallel(n, [&](unsigned, uint64_t a, uint64_t z) {
        for (uint64_t r = a; r < z; r++) {
            uint64_t b, e;
            line(4 * r, b, e);
            memcpy(rd->ids + rd->idOffsets[r], base + b + 1, ilen[r]);
            line(4 * r + 1, b, e);
            memcpy(rd->bases + rd->offsets[r], base + b, blen[r]);
            line(4 * r + 3, b, e);
            const uint32_t nq = std::min(qlen[r], blen[r]);
            memcpy(rd->quals + rd->offsets[r], base + b, nq);
            if (nq < blen[r]) memset(rd->quals + rd->offsets[r] + nq, 0, blen[r] - nq);
        }
    });
    memset(rd->bases + total, 0, 64);   // the batch's zero slack
    memset(rd->quals + total, 0, 64);
    return rd;
}

int snapgpu_reads_write_fastq(const snapgpu_reads_t *r, const char *path) {
    FILE *f = fopen(path, "w");
    if (!f) { setError(std::string("cannot write ") + path); return SNAPGPU_EIO; }
    for (uint64_t i = 0; i < r->n; i++) {
        if (r->ids) {
            fputc('@', f);
            fwrite(r->ids + r->idOffsets[i], 1, r->idLengths[i], f);
        } else {
            fprintf(f, "@read%llu", (unsigned long long)i);
            if (r->truthLocation) fprintf(f, "_%u_%u", r->truthLocation[i], (unsigned)r->truthDirection[i]);
        }
        fputc('\n', f);
        fwrite(r->bases + r->offsets[i], 1, r->lengths[i], f);
        fputs("\n+\n", f);
        fwrite(r->quals + r->offsets[i], 1, r->lengths[i], f);
        fputc('\n', f);
    }
    int ok = ferror(f) == 0;
    fclose(f);
    return ok ? SNAPGPU_OK : SNAPGPU_EIO;
}

void snapgpu_reads_free(snapgpu_reads_t *r) {
    if (!r) return;
    if (!(r->hostFlags & kReadsView)) {   // a view's bases and qualities belong to its parent
        hostFree(r->bases, r->hostFlags & 1u);
        hostFree(r->quals, r->hostFlags & 2u);
    }
    delete[] r->offsets; delete[] r->lengths;
    delete[] r->truthLocation; delete[] r->truthDirection;
    delete[] r->frontClipped; delete[] r->unclippedLength;
    delete[] r->ids; delete[] r->idOffsets; delete[] r->idLengths;
    delete r;
}

}  // extern "C"
