// charseeds.hip -- gfx950 BaseAligner::CharacterizeSeeds (SNAPLib/BaseAligner.cpp:206-508), the
// seed census the RNA paired product path takes of reads it could not align
// as a pair: AlignmentFilter::UnalignedRead (AlignmentFilter.cpp:742-933) and FindPartialMatches
// (:957-1037) run it through the "partial aligner" of PairedAligner.cpp:518-527 (maxHits 300,
// 12 seeds) and look only at its two maps genome location -> set of seed offsets.
//
// The reference walks the seeds of AlignRead's order (used bits, +seedLen steps, the wrap
// table), looks each one up, and inserts every hit of a direction that is not popular into a
// std::map<unsigned, std::set<unsigned>>.  Here one wave owns a read:
//   * the seed walk is wave-uniform scalar code (as align_kernel's), the 2-bit encoding one base
//     per lane, the lookup one bucket line (bucket_table.h) on lanes 0-3, the next on 4-7;
//   * the hits of an applied direction are appended one per lane as 42-bit keys
//     dir << 41 | location << 9 | seedOffset into an LDS array (at most (numSeeds + 1) * maxHits
//     <= 4096 keys: the loop tests the applied count once per seed, a seed applies <= 2 sides);
//   * a bitonic sort of that array in LDS gives the maps' iteration order (map before mapRC,
//     locations ascending, each set ascending); a segmented scan turns equal (dir, location)
//     runs into one record {location, min = *set.begin(), max = *set.rbegin(), count}.
// Records are appended to an HBM pool at an atomically reserved offset; the host copies back
// only the used prefix.  Work: ~12 lookups and <= 3,900 keys per read, so the kernel is bound by
// the lookups' dependent probe chains (as seed_lookup_kernel) plus the LDS sort.
#include <hip/hip_runtime.h>

#include <cstring>
#include <string>
#include <vector>

#include "align_device.h"
#include "bucket_table.h"
#include "internal.h"

int snapgpu_internal_index_args(const snapgpu_aligner_t *a, sgk::KArgs *A, int *device);
int snapgpu_internal_devbuf(snapgpu_aligner_t *a, int slot, uint64_t bytes, void **p);   // grow-only, the aligner's
hipStream_t snapgpu_internal_stream(snapgpu_aligner_t *a);

namespace sgk {
namespace cs {

constexpr int KEYCAP = 4096;   // LDS keys per wave (32 KB)

struct Run {                   // = snapgpu_seed_run_t
    uint32_t location;
    uint16_t minOffset, maxOffset, count;
    uint8_t direction, reserved;
};
static_assert(sizeof(Run) == 12, "snapgpu_seed_run_t layout");

struct ReadRec {               // per read: where its runs went
    uint32_t start;            // index into the pool
    uint32_t nRuns;
    uint32_t nForward;
    uint32_t flags;            // SNAPGPU_FLAG_READ_TOO_LONG / SNAPGPU_FLAG_TOO_MANY_NS / SNAPGPU_FLAG_CS_*
};

struct CArgs {
    KArgs X;                   // index + DevTables (the aligner's upload)
    const char *bases;
    const uint64_t *offsets;
    const uint32_t *lengths;
    const uint32_t *readList;  // reads of this launch (indices into offsets/lengths)
    uint32_t nReads;
    uint32_t maxHits, maxK, maxSeeds, maxReadSize, explore;
    uint32_t *counter;         // [0] read queue, [1] pool fill
    Run *pool;
    uint64_t poolCap;
    ReadRec *rec;              // [nReads], in readList order
};

constexpr uint32_t FLAG_POOL_FULL = 0x100;   // host retries (never with the host's sizing)
constexpr uint32_t FLAG_GUARD = 0x200;       // seed-loop guard tripped (cannot happen; fails the call)

struct Lds {
    uint64_t keys[KEYCAP];
    char fwd[512 + 64];
    uint64_t used[9];
};

__global__ __launch_bounds__(64) void charseeds_kernel(CArgs C) {
    __shared__ Lds S;
    const KArgs &A = C.X;
    const uint32_t seedLen = A.seedLen;
    for (;;) {
        const int lane = lane_id();
        uint32_t qi = 0;
        if (lane == 0) qi = atomicAdd(C.counter, 1u);
        qi = uni((uint32_t)readlane((int)qi, 0));
        if (qi >= C.nReads) break;
        const uint32_t r = C.readList ? uni(C.readList[qi]) : qi;
        const uint32_t n = uni(C.lengths[r]);
        const uint64_t off = uni64(C.offsets[r]);
        uint32_t flags = 0, nKeys = 0;
        bool run = true;
        if (n > C.maxReadSize || n > 512) { flags |= SNAPGPU_FLAG_READ_TOO_LONG; run = false; }   // :272-275 soft_exit
        else if (n < seedLen) run = false;                                                          // :277-282
        if (run) {
            // Read::init upper-casing; countOfNs (:289-306)
            uint32_t nN = 0;
            for (int i = lane; i < 512 + 64; i += WAVE) {
                uint32_t c = 0;
                if (i < (int)n) {
                    c = (uint8_t)C.bases[off + i];
                    if (c >= 'a' && c <= 'z') c -= 0x20;
                }
                S.fwd[i] = (char)c;
                nN += __popcll(ballot(i < (int)n && c == 'N'));
            }
            if (lane < 9) S.used[lane] = 0;
            wave_sync();
            if (nN > C.maxK) { flags |= SNAPGPU_FLAG_TOO_MANY_NS; run = false; }   // :303-306
        }
        if (run) {
            const uint32_t nPossible = n - seedLen + 1;
            uint32_t next = 0, wrapCount = 0, applied[2] = {0, 0};
            const uint32_t guardMax = (nPossible + 2) * (seedLen + 2) + C.maxSeeds + 4;
            for (uint32_t guard = 0; applied[0] + applied[1] < C.maxSeeds; guard++) {   // :336
                const int lane = lane_id();
                if (guard > guardMax) { flags |= FLAG_GUARD; break; }
                if (next >= nPossible) {   // :341-358
                    wrapCount++;
                    if (wrapCount >= seedLen) break;
                    next = A.tab->wrap[wrapCount];
                }
                while (next < nPossible && ((uni64(S.used[next >> 6]) >> (next & 63)) & 1)) next++;   // :360-365
                if (next >= nPossible) continue;
                {
                    const uint64_t w = uni64(S.used[next >> 6]) | (1ull << (next & 63));
                    wave_sync();
                    if (lane == 0) S.used[next >> 6] = w;
                    wave_sync();
                }
                // Seed::DoesTextRepresentASeed (:375-377: skipped without the +seedLen step) + Seed::Seed
                const int v = lane < (int)seedLen ? base_value((uint8_t)S.fwd[next + lane]) : 0;
                if (ballot(lane < (int)seedLen && v > 3)) continue;
                const uint64_t f = uni64(or_reduce64(lane < (int)seedLen ? (uint64_t)v << ((seedLen - lane - 1) * 2) : 0));
                const uint64_t rcv = uni64(or_reduce64(lane < (int)seedLen ? (uint64_t)(v ^ 3) << (lane * 2) : 0));
                // GenomeIndex::lookupSeed (GenomeIndex.cpp:971-1011) + SNAPHashTable::Lookup (HashTable.h:74-105)
                const bool comp = (int64_t)f > (int64_t)rcv, pal = f == rcv;
                const uint64_t canon = comp ? rcv : f;
                const uint32_t table = (uint32_t)(canon >> 32), key = (uint32_t)canon;
                // SNAPHashTable::Lookup answered by the bucket image (bucket_table.h)
                uint32_t v1 = 0, v2 = 0, aux = 0, lines = 0;
                const bool found = bucket_lookup_wave(A, table, key, lane, v1, v2, aux, lines);
                // fillInLookedUpResults (GenomeIndex.cpp:1013-1086), unwindowed (minSeedLoc 0, maxSeedLoc ~0: :384-386)
                uint32_t nH[2] = {0, 0}, sg[2] = {0, 0};
                const uint32_t *ls[2] = {nullptr, nullptr};
                if (found) {
                    const uint32_t vs[2] = {comp ? v2 : v1, comp ? v1 : v2};
                    const uint32_t cs[2] = {comp ? (aux >> 15) & BK_CSAT : aux & BK_CSAT, comp ? aux & BK_CSAT : (aux >> 15) & BK_CSAT};
                    for (int sd = 0; sd < 2; sd++) {
                        if (sd == 1 && pal) { nH[1] = nH[0]; sg[1] = sg[0]; ls[1] = ls[0]; break; }
                        const uint32_t vv = vs[sd];
                        if (vv < A.nBases) { nH[sd] = 1; sg[sd] = vv; }
                        else if (vv != UNUSED_SIDE) {
                            const uint32_t o = vv - A.nBases;
                            nH[sd] = uni(bucket_count(A, cs[sd], vv));
                            ls[sd] = A.overflow + o + 1;
                        }
                    }
                }
                // :393-497: every hit of a side that is not popular, into map / mapRC
                for (uint32_t dir = 0; dir < 2; dir++) {
                    const uint32_t nh = nH[dir];
                    if (nh > C.maxHits && !C.explore) continue;   // popular: pretend we never looked
                    const uint32_t lim = nh < C.maxHits ? nh : C.maxHits;
                    const uint32_t offset = dir == 0 ? next : n - seedLen - next;   // :420-434
                    for (uint32_t b = 0; b < lim; b += WAVE) {
                        const uint32_t i = b + lane;
                        uint32_t hit = 0;
                        if (i < lim) hit = ls[dir] ? ls[dir][i] : sg[dir];
                        const bool keep = i < lim && hit >= offset;   // :456-460 (the window is [0, ~0])
                        const uint64_t mk = ballot(keep);
                        const uint32_t before = __popcll(mk & ((1ull << lane) - 1));
                        if (keep && nKeys + before < (uint32_t)KEYCAP)
                            S.keys[nKeys + before] = ((uint64_t)dir << 41) | ((uint64_t)(hit - offset) << 9) | next;
                        nKeys += __popcll(mk);
                    }
                    applied[dir]++;   // :494
                }
                next += seedLen;   // :504
            }
            if (nKeys > (uint32_t)KEYCAP) { flags |= FLAG_GUARD; nKeys = 0; }
        }
        wave_sync();
        // bitonic sort of keys[0, P), P = next power of two >= nKeys (padding sorts last)
        uint32_t P = 64;
        while (P < nKeys) P <<= 1;
        if (nKeys > 1) {
            for (uint32_t i = nKeys + lane; i < P; i += WAVE) S.keys[i] = ~0ull;
            wave_sync();
            for (uint32_t k = 2; k <= P; k <<= 1)
                for (uint32_t j = k >> 1; j > 0; j >>= 1) {
                    for (uint32_t t = lane; t < P / 2; t += WAVE) {
                        const uint32_t i = 2 * t - (t & (j - 1));   // lower index of the pair
                        const uint32_t l = i + j;
                        const uint64_t a = S.keys[i], b = S.keys[l];
                        const bool up = (i & k) == 0;
                        if ((a > b) == up) { S.keys[i] = b; S.keys[l] = a; }
                    }
                    wave_sync();
                }
        }
        // runs of equal (dir, location): count, reserve pool space, write
        uint32_t nRuns = 0, nFwd = 0;
        for (uint32_t b = 0; b < nKeys; b += WAVE) {
            const uint32_t i = b + lane;
            const uint64_t kk = i < nKeys ? S.keys[i] : 0;
            const bool st = i < nKeys && (i == 0 || (S.keys[i - 1] >> 9) != (kk >> 9));
            nRuns += __popcll(ballot(st));
            nFwd += __popcll(ballot(st && (kk >> 41) == 0));
        }
        uint32_t base = 0;
        if (lane == 0 && nRuns) base = atomicAdd(C.counter + 1, nRuns);
        base = uni((uint32_t)readlane((int)base, 0));
        if ((uint64_t)base + nRuns > C.poolCap) { flags |= FLAG_POOL_FULL; nRuns = nFwd = 0; }
        if (nRuns) {
            uint32_t runIdx = 0, carry = 0;   // carry: key index where the current run started
            for (uint32_t b = 0; b < nKeys; b += WAVE) {
                const uint32_t i = b + lane;
                const uint64_t kk = i < nKeys ? S.keys[i] : ~0ull;
                const bool st = i < nKeys && (i == 0 || (S.keys[i - 1] >> 9) != (kk >> 9));
                const bool en = i < nKeys && (i + 1 == nKeys || (S.keys[i + 1] >> 9) != (kk >> 9));
                // segmented max-scan of run starts: the start index of this key's run
                uint32_t s = st ? i : carry;
#pragma unroll
                for (int o = 1; o < WAVE; o <<= 1) {
                    const uint32_t y = (uint32_t)shfl_idx((int)s, lane >= o ? lane - o : lane);
                    if (lane >= o && y > s) s = y;
                }
                const uint64_t sm = ballot(st);
                const uint32_t j = runIdx + __popcll(sm & ((1ull << lane) - 1)) - (st ? 0u : 1u);
                if (en) {
                    Run o;
                    o.location = (uint32_t)(kk >> 9);
                    o.minOffset = (uint16_t)(S.keys[s] & 511);
                    o.maxOffset = (uint16_t)(kk & 511);
                    o.count = (uint16_t)(i - s + 1);
                    o.direction = (uint8_t)(kk >> 41);
                    o.reserved = 0;
                    C.pool[(uint64_t)base + j] = o;
                }
                runIdx += __popcll(sm);
                carry = uni((uint32_t)readlane((int)s, WAVE - 1));
            }
        }
        if (lane == 0) {
            ReadRec o;
            o.start = base; o.nRuns = nRuns; o.nForward = nFwd; o.flags = flags;
            C.rec[qi] = o;
        }
        wave_sync();
    }
}

}  // namespace cs
}  // namespace sgk

using namespace sgk;
using namespace sgk::cs;

namespace {
#define CCHK(x)                                                                         \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            snapgpu::setError(std::string(#x) + ": " + hipGetErrorString(e_));          \
            rc = SNAPGPU_EDEVICE;                                                       \
            goto done;                                                                  \
        }                                                                               \
    } while (0)
}  // namespace

extern "C" {

void snapgpu_charseeds_params_default(snapgpu_charseeds_params_t *p) {
    if (!p) return;
    memset(p, 0, sizeof(*p));
    p->maxHits = 300;        // PairedAligner.cpp:520
    p->maxK = 15;            // the paired CLI's maxDist (AlignerOptions.cpp:73-77)
    p->numSeeds = 12;        // PairedAligner.cpp:523
    p->maxReadSize = 500;    // MAX_READ_LENGTH
    p->explorePopularSeeds = 0;
}

void snapgpu_seed_runs_free(snapgpu_seed_runs_t *r) {
    if (!r) return;
    delete[] r->start;
    delete[] r->nForward;
    delete[] r->flags;
    delete[] r->runs;
    delete r;
}

snapgpu_seed_runs_t *snapgpu_characterize_seeds(snapgpu_aligner_t *a, const snapgpu_reads_t *reads,
                                                const uint64_t *readList, uint64_t nList,
                                                const snapgpu_charseeds_params_t *p) {
    if (!a || !reads || !p) { snapgpu::setError("characterize_seeds: null argument"); return nullptr; }
    if (p->numSeeds == 0 || (uint64_t)(p->numSeeds + 1) * p->maxHits > (uint64_t)KEYCAP || p->maxReadSize > 512) {
        snapgpu::setError("characterize_seeds: needs numSeeds >= 1, (numSeeds + 1) * maxHits <= 4096 and "
                          "maxReadSize <= 512 (the partial aligner: 12 seeds, maxHits 300, 500)");
        return nullptr;
    }
    const uint64_t n = readList ? nList : reads->n;
    if (readList)
        for (uint64_t i = 0; i < n; i++)
            if (readList[i] >= reads->n) { snapgpu::setError("characterize_seeds: read index out of range"); return nullptr; }
    KArgs X;
    int device = 0, rc = snapgpu_internal_index_args(a, &X, &device);
    if (rc) { snapgpu::setError("characterize_seeds: aligner unusable"); return nullptr; }
    auto *out = new snapgpu_seed_runs_t();
    out->n = n;
    out->start = new uint64_t[n + 1]();
    out->nForward = new uint32_t[n + 1]();
    out->flags = new uint32_t[n + 1]();
    std::vector<std::vector<Run>> parts;
    std::vector<ReadRec> recs;
    std::vector<uint32_t> counts(n + 1, 0);
    hipStream_t s = nullptr;
    char *dB = nullptr;
    uint64_t *dO = nullptr;
    uint32_t *dL = nullptr, *dList = nullptr, *dCnt = nullptr;
    Run *dPool = nullptr;
    ReadRec *dRec = nullptr;
    // device buffers: the aligner's grow-only scratch slots (a hipMalloc / hipFree per call, the
    // pool up to 3 GB, cost more than the kernel and hipFree waits for the whole device)
    auto buf = [&](int slot, uint64_t bytes, auto *&ptr) -> hipError_t {
        void *v = nullptr;
        if (snapgpu_internal_devbuf(a, slot, bytes, &v)) return hipErrorOutOfMemory;
        ptr = reinterpret_cast<std::remove_reference_t<decltype(ptr)>>(v);
        return hipSuccess;
    };
    const uint64_t perRead = (uint64_t)(p->numSeeds + 1) * p->maxHits;
    const uint64_t CH = 65536;   // reads per launch: pool <= 65536 * 3900 * 12 B = 3 GB
    uint64_t total = 0;
    int grid = 0;
    rc = SNAPGPU_OK;
    CCHK(hipSetDevice(device));
    s = snapgpu_internal_stream(a);
    {
        int ncu = 0;
        CCHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device));
        grid = ncu * 4;   // 33 KB LDS per wave: 4 waves per CU
    }
    CCHK(buf(0, reads->totalBytes + 1024, dB));
    CCHK(hipMemsetAsync(dB + reads->totalBytes, 0, 1024, s));
    CCHK(hipMemcpyAsync(dB, reads->bases, reads->totalBytes, hipMemcpyHostToDevice, s));
    CCHK(buf(1, reads->n * 8 + 8, dO));
    CCHK(buf(2, reads->n * 4 + 4, dL));
    CCHK(hipMemcpyAsync(dO, reads->offsets, reads->n * 8, hipMemcpyHostToDevice, s));
    CCHK(hipMemcpyAsync(dL, reads->lengths, reads->n * 4, hipMemcpyHostToDevice, s));
    CCHK(buf(3, 16, dCnt));
    CCHK(buf(4, CH * 4, dList));
    CCHK(buf(5, CH * sizeof(ReadRec), dRec));
    CCHK(buf(6, std::min(CH, n ? n : 1) * perRead * sizeof(Run), dPool));
    recs.resize(CH);
    for (uint64_t c0 = 0; c0 < n; c0 += CH) {
        const uint64_t m = std::min(CH, n - c0);
        std::vector<uint32_t> list(m);
        for (uint64_t i = 0; i < m; i++) list[i] = (uint32_t)(readList ? readList[c0 + i] : c0 + i);
        CCHK(hipMemcpyAsync(dList, list.data(), m * 4, hipMemcpyHostToDevice, s));
        CCHK(hipMemsetAsync(dCnt, 0, 16, s));
        CArgs C;
        memset(&C, 0, sizeof(C));
        C.X = X;
        C.bases = dB; C.offsets = dO; C.lengths = dL; C.readList = dList; C.nReads = (uint32_t)m;
        C.maxHits = p->maxHits; C.maxK = p->maxK; C.maxSeeds = p->numSeeds; C.maxReadSize = p->maxReadSize;
        C.explore = p->explorePopularSeeds;
        C.counter = dCnt; C.pool = dPool; C.poolCap = m * perRead; C.rec = dRec;
        const int g = (int)std::min<uint64_t>((uint64_t)grid, m);
        hipLaunchKernelGGL(charseeds_kernel, dim3(g), dim3(64), 0, s, C);
        CCHK(hipGetLastError());
        uint32_t cnt[4] = {0, 0, 0, 0};
        CCHK(hipMemcpyAsync(cnt, dCnt, 16, hipMemcpyDeviceToHost, s));
        CCHK(hipMemcpyAsync(recs.data(), dRec, m * sizeof(ReadRec), hipMemcpyDeviceToHost, s));
        CCHK(hipStreamSynchronize(s));
        parts.emplace_back(std::min<uint64_t>(cnt[1], m * perRead));
        if (!parts.back().empty())
            CCHK(hipMemcpyAsync(parts.back().data(), dPool, parts.back().size() * sizeof(Run), hipMemcpyDeviceToHost, s));
        CCHK(hipStreamSynchronize(s));
        {
            // this part's runs in read order (the pool holds them in completion order)
            std::vector<Run> &pt = parts.back();
            std::vector<Run> ordered;
            ordered.reserve(pt.size());
            for (uint64_t i = 0; i < m; i++) {
                const ReadRec &q = recs[i];
                if ((q.flags & (FLAG_POOL_FULL | FLAG_GUARD)) || (uint64_t)q.start + q.nRuns > pt.size()) {
                    snapgpu::setError("characterize_seeds: internal capacity exceeded");
                    rc = SNAPGPU_EDEVICE;
                    goto done;
                }
                out->flags[c0 + i] = q.flags;
                out->nForward[c0 + i] = q.nForward;
                counts[c0 + i] = q.nRuns;
                ordered.insert(ordered.end(), pt.begin() + q.start, pt.begin() + q.start + q.nRuns);
            }
            pt.swap(ordered);
            total += pt.size();
        }
    }
    // final layout: runs in read order, start[i] = first run of read i
    out->nRuns = total;
    out->runs = new snapgpu_seed_run_t[total + 1];
    {
        uint64_t at = 0;
        for (auto &pt : parts) {
            if (!pt.empty()) memcpy(out->runs + at, pt.data(), pt.size() * sizeof(Run));
            at += pt.size();
        }
        at = 0;
        for (uint64_t i = 0; i < n; i++) { out->start[i] = at; at += counts[i]; }
        out->start[n] = at;
    }
done:
    if (rc && s) (void)hipStreamSynchronize(s);   // nothing of this call left in flight on the scratch
    if (rc) { snapgpu_seed_runs_free(out); return nullptr; }
    return out;
}

}  // extern "C"
