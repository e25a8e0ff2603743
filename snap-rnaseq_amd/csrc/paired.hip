// paired.hip -- gfx950 paired-end aligner: IntersectingPairedEndAligner::align
// (SNAPLib/IntersectingPairedEndAligner.cpp:142-753) for a batch of read pairs, one wave per pair,
// and ChimericPairedEndAligner::align (ChimericPairedEndAligner.cpp:56-126) on the host around it,
// whose single-end fallback is the GPU BaseAligner of aligner.hip.
//
// Per pair the wave runs the reference's three phases with its control flow kept sequential and
// each step's inner work spread over the lanes:
//   1. seeds: the seed offsets depend only on the read's bases, so they are chosen first (scalar
//      SeedSequencer walk); the lookups then run one lane per seed; the hit sets
//      (HashTableHitSet, :844-899) are assembled in the reference's order afterwards, because
//      where a disjoint hit set begins depends on which lookups were recorded.
//   2. intersection (:357-511): the walk over both ends' hit sets is sequential; every hit-set
//      step (first hit, binary search per lookup, next lower hit, best possible score) is one lane
//      per lookup plus a wave reduction; mate candidates, scoring candidates and merge anchors live
//      in a per-wave HBM pool.
//   3. scoring (:516-718): candidates in best-possible-score order; scoreLocation (:755-841) is
//      the byte-compare Landau-Vishkin of align_device.h (one lane per diagonal).
// Pass 1 takes pairs of reads <= 128 bases with pools sized for ordinary pairs; pairs with a longer
// read, or whose pools overflow, are deferred to pass 1b (reads <= 256 on 256-bit planes, the same
// pools), then to pass 2 (reads <= 512 and IUPAC cases, byte compares, the same pool sizes on the
// full grid); pass 2's pool overflows go to pass 3 (pools of the reference's size on a small grid:
// 22 MB per wave at the paired defaults).  A pair that exceeds the reference's own pool is
// flagged: the reference exits there (soft_exit, :436-439, :482-485, :634-637).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "align_device.h"
#include "bucket_table.h"
#include "order_long.h"
#include "internal.h"

int snapgpu_internal_index_args(const snapgpu_aligner_t *a, sgk::KArgs *A, int *device);
void snapgpu_internal_fill_tables(sgk::DevTables *t, uint32_t seedLen);
bool snapgpu_internal_aligner_failed(const snapgpu_aligner_t *a);

namespace sgk {
namespace pe {

constexpr int LCAP = 32;                    // lookups per hit set (MAX_MAX_SEEDS = 30, IntersectingPairedEndAligner.h:93)
constexpr uint32_t UNSCORED = 0xfffffffeu;  // ScoringMateCandidate::score before scoring (-2)
constexpr int MAX_LISTS = 64;               // scoringCandidates[maxK + extraSearchDepth + 1]

struct PArgs {
    KArgs X;                                // index, genome, tables (aligner.hip's upload)
    const char *bases[2], *quals[2];
    const uint64_t *offsets[2];
    const uint32_t *lengths[2];
    uint32_t nPairs;                        // pairs in this launch (pairList entries in pass 2)
    const uint32_t *pairList;               // pass 2: pair indices; pass 1: nullptr (identity)
    uint32_t *deferList, *deferCount;       // pass 1 -> pass 2
    snapgpu_pair_result_t *out;
    uint32_t *counter;                      // work queue
    uint32_t maxK, extra, maxSeedsCmd, minSpacing, maxSpacing, maxBigHits, maxReadSize;
    double seedCoverage;
    char *pool;                             // per block: candidates, mates[2], anchors
    uint64_t poolStride;
    uint32_t candCap, mateCap, anchorCap;   // this pass's pool capacities
    uint32_t refPool;                       // the reference's scoringCandidatePoolSize (:128)
    uint32_t maxLen;                        // reads this pass takes (128 or 512)
    uint32_t deferred;                      // the pairs of this pass were deferred (passes 1b, 2, 3)
    uint32_t passId;                        // snapgpu_pair_result_t::writtenBy of this launch's records
};

struct Lookup {                             // HashTableLookup (IntersectingPairedEndAligner.h:101-134);
    uint32_t at;                            // overflow index of hits[0], or the singleton value
    uint32_t nHits;                         // the cursor lives in registers during the walk (LaneLk)
    uint16_t seedOffset;
    uint8_t set, single;
};
static_assert(sizeof(Lookup) == 12, "Lookup layout");
struct HitSet {                             // HashTableHitSet (IntersectingPairedEndAligner.h:139-194)
    Lookup lk[LCAP];
    uint32_t exhausted[LCAP];               // DisjointHitSet::countOfExhaustedHits
    int32_t curSet;
    uint32_t nLookups, lastReturned, pad;
};
struct Mate {                               // ScoringMateCandidate (:401-423)
    double prob;
    uint32_t loc, bestPossible, score, scoreLimit, seedOffset;
    int32_t genomeOffset;
};
struct Cand {                               // ScoringCandidate (:425-447), indices for pointers
    int32_t next, anchor;
    uint32_t mateIndex, loc, setPair, seedOffset, bestPossible, pad;
};
struct Anchor {                             // MergeAnchor (:364-393)
    double prob;
    uint32_t moreLoc, fewerLoc;
    int32_t pairScore, pad;
};
static_assert(sizeof(Mate) == 32 && sizeof(Cand) == 32 && sizeof(Anchor) == 24, "pool layout");

template <int MAXLEN>
struct PLds {
    static constexpr int NB = MAXLEN / 64;
    static constexpr int PW = MAXLEN <= 256 ? NB : 2;   // read bit-plane words (<128>, <256>)
    char rd[2][2][MAXLEN + 64];             // [read][direction] bases, upper-cased, zero slack
    char rq[2][2][MAXLEN + 64];             // qualities in the same coordinates
    uint32_t win[MAXLEN <= 256 ? 1 : (MAXLEN + 192) / 4];   // <512>: genome window of scoreLocation
    // phases 1-2 (seeds, hit sets) and phase 3 (scoring) never overlap: their scratch shares LDS
    union {
        struct {
            HitSet hs[2][2];                // [read][direction]
            uint32_t look[2][LCAP][6];      // per read, seed, direction: nHits | single << 31, at, trimmed
        } walk;
        struct {
            uint16_t rows[MAX_K][WAVE];     // lv_wave row history
            int16_t btAct[MAX_K + 1], btMatched[MAX_K + 1];
        } lv;
    } u;
    uint32_t miss[LCAP];                    // DisjointHitSet::missCount scratch
    uint32_t sel[2][LCAP];                  // chosen seed offsets per read (bit 31: a wrap preceded it)
    uint64_t validBits[NB], usedBits[NB];
    uint64_t rpl[2][2][3][PW];              // <128>/<256>: read bit planes [read][dir]{hi, lo, notACGT} x NB words
    int32_t lists[MAX_LISTS];
};

__device__ __forceinline__ bool is_within(uint32_t a, uint32_t b, uint32_t d) {   // Util.h:538-541
    return (a <= b && a + d >= b) || (a >= b && a <= b + d);
}
__device__ __forceinline__ uint32_t loc_distance(uint32_t a, uint32_t b) { return a > b ? a - b : b - a; }

__device__ __forceinline__ uint32_t hit_at(const PArgs &P, const Lookup &l, uint32_t i) {
    return l.single ? l.at : P.X.overflow[l.at + i];
}

// --------------------------------------------------------------- hit sets
// The intersection walks two hit sets at a time (the fewer-hits and the more-hits end of one set
// pair).  Lane i keeps lookup i of each in registers: its cursor (currentHitForIntersection) and
// the hits at cur - 1, cur and cur + 1, so computeBestPossibleScoreForCurrentHit needs no load and
// getNextLowerHit's advance uses the prefetched next hit (the load for the one after it is issued
// then and only waited for at the next advance).  Ties between lookups go to the lowest index,
// as the reference's in-order scans with strict comparisons do.
struct LaneLk {
    uint32_t cur, nHits, so, set, at, single;
    uint32_t curV, prevV, nextV;   // hits[cur], hits[cur - 1], hits[cur + 1] (when they exist)
    bool on;                       // lane < nLookups
};
struct Walk {                      // one hit set being walked: per-lane lookups + uniform state
    LaneLk l;
    uint32_t last;                 // mostRecentLocationReturned
    uint32_t nLookups;
    int32_t curSet;
    const uint32_t *exhausted;     // LDS: DisjointHitSet::countOfExhaustedHits
};

__device__ __forceinline__ uint32_t lk_hit(const PArgs &P, const LaneLk &l, uint32_t i) {
    return l.single ? l.at : P.X.overflow[l.at + i];
}

__device__ __forceinline__ void walk_init(const PArgs &P, const HitSet &h, Walk &w) {
    const int lane = lane_id();
    w.nLookups = h.nLookups;
    w.curSet = h.curSet;
    w.exhausted = h.exhausted;
    w.last = 0;
    LaneLk &l = w.l;
    l.on = (uint32_t)lane < w.nLookups;
    const Lookup k = h.lk[l.on ? lane : 0];
    l.cur = 0; l.nHits = l.on ? k.nHits : 0; l.so = k.seedOffset; l.set = k.set; l.at = k.at; l.single = k.single;
    l.curV = l.nHits > 0 ? lk_hit(P, l, 0) : 0u;
    l.nextV = l.nHits > 1 ? lk_hit(P, l, 1) : 0u;
    l.prevV = 0;
}

__device__ __forceinline__ uint64_t best_key(bool have, uint32_t v, int lane) {
    return have ? ((uint64_t)v << 8) | (uint64_t)(255 - lane) : 0ull;
}
__device__ __forceinline__ bool take_best(Walk &w, uint64_t k, uint32_t &loc, uint32_t &seedOff) {
    if (k == 0) return false;
    loc = (uint32_t)(k >> 8);
    seedOff = (uint32_t)__builtin_amdgcn_readlane((int)w.l.so, 255 - (int)(k & 255));
    w.last = loc;
    return true;
}

// getFirstHit (:1270-1284)
__device__ bool hs_first(Walk &w, uint32_t &loc, uint32_t &seedOff) {
    const int lane = lane_id();
    const LaneLk &l = w.l;
    const uint32_t v = l.curV - l.so;
    const uint64_t k = uni64(max_reduce64(best_key(l.on && l.nHits > 0 && v > 0, v, lane)));
    loc = 0;
    return take_best(w, k, loc, seedOff);
}

// getNextHitLessThanOrEqualTo, the version the reference compiles (:1219-1266)
__device__ bool hs_next_le(const PArgs &P, Walk &w, uint32_t maxOff, uint32_t &loc, uint32_t &seedOff) {
    const int lane = lane_id();
    LaneLk &l = w.l;
    bool have = false;
    uint32_t v = 0;
    if (l.on) {
        int lim0 = (int)l.cur, lim1 = (int)l.nHits - 1;
        const uint32_t maxThis = maxOff + l.so;
        while (lim0 <= lim1) {
            const uint32_t probe = (uint32_t)(lim0 + lim1) / 2;
            const uint32_t hp = lk_hit(P, l, probe);
            const uint32_t hq = probe == 0 ? 0u : lk_hit(P, l, probe - 1);
            if (hp <= maxThis && (probe == 0 || hq > maxThis)) {
                v = hp - l.so;
                have = v > 0;
                l.cur = probe;
                l.curV = hp;
                l.prevV = hq;
                l.nextV = probe + 1 < l.nHits ? lk_hit(P, l, probe + 1) : 0u;
                break;
            }
            if (hp > maxThis) lim0 = (int)probe + 1;
            else lim1 = (int)(probe - 1);
        }
        if (lim0 > lim1 && l.cur != l.nHits) {   // exhausted: hits[cur - 1] is now the last hit
            l.cur = l.nHits;
            l.prevV = l.nHits ? lk_hit(P, l, l.nHits - 1) : 0u;
        }
    }
    const uint64_t k = uni64(max_reduce64(best_key(have, v, lane)));
    return take_best(w, k, loc, seedOff);
}

// getNextLowerHit (:1286-1322)
__device__ bool hs_next_lower(const PArgs &P, Walk &w, uint32_t &loc, uint32_t &seedOff) {
    const int lane = lane_id();
    LaneLk &l = w.l;
    bool have = false;
    uint32_t v = 0;
    if (l.on) {
        if (l.cur != l.nHits && l.curV - l.so == w.last) {
            l.cur++;
            l.prevV = l.curV;
            l.curV = l.nextV;
            l.nextV = l.cur + 1 < l.nHits ? lk_hit(P, l, l.cur + 1) : 0u;
        }
        if (l.cur != l.nHits && l.curV >= l.so) { v = l.curV - l.so; have = v > 0; }
    }
    const uint64_t k = uni64(max_reduce64(best_key(have, v, lane)));
    return take_best(w, k, loc, seedOff);
}

// computeBestPossibleScoreForCurrentHit (:901-929): the largest miss count of any disjoint hit set
template <int MAXLEN>
__device__ uint32_t hs_best_possible(PLds<MAXLEN> &S, const Walk &w, uint32_t maxMerge) {
    const int lane = lane_id();
    const int nSets = w.curSet + 1;
    if (lane < nSets) S.miss[lane] = w.exhausted[lane];
    wave_sync();
    const LaneLk &l = w.l;
    if (l.on) {
        const uint32_t target = w.last + l.so;
        const bool nearCur = l.cur != l.nHits && is_within(l.curV, target, maxMerge);
        const bool nearPrev = l.cur != 0 && is_within(l.prevV, target, maxMerge);
        if (!(nearCur || nearPrev)) atomicAdd(&S.miss[l.set], 1u);
    }
    wave_sync();
    const uint32_t m = lane < nSets ? S.miss[lane] : 0u;
    return uni(max_reduce32(m));
}

// recordLookup (:859-899), uniform: every lane writes the same values
// (nHits as looked up; trimmed = after the trim of :882-884, done by the lookup lane)
__device__ __forceinline__ void hs_record(HitSet &h, uint32_t seedOffset, uint32_t nHits, uint32_t trimmed, uint32_t at,
                                          uint32_t single, bool begins) {
    if (begins) { h.curSet = h.curSet + 1; h.exhausted[h.curSet] = 0; }
    if (nHits == 0) { h.exhausted[h.curSet] = h.exhausted[h.curSet] + 1; wave_sync(); return; }
    Lookup l;
    l.nHits = trimmed; l.seedOffset = (uint16_t)seedOffset; l.set = (uint8_t)h.curSet; l.at = at; l.single = (uint8_t)single;
    h.lk[h.nLookups] = l;
    h.nLookups = h.nLookups + 1;
    wave_sync();
}

// ------------------------------------------------------------ scoreLocation
// IntersectingPairedEndAligner::scoreLocation (:755-841).  *offset is written only when the
// reverse LV runs (its netIndel, 0 when it fails), as the reference's genomeLocationOffset.
template <int MAXLEN>
__device__ void score_location(const PArgs &P, PLds<MAXLEN> &S, int r, int dir, uint32_t n, uint32_t loc,
                               uint32_t seedOffset, uint32_t scoreLimit, uint32_t &score, double &prob,
                               int32_t &offset, uint32_t &nScored) {
    constexpr int NB = MAXLEN / 64;
    const KArgs &X = P.X;
    const int lane = lane_id();
    nScored++;
    uint32_t glen = n + MAX_K;
    bool ok = substring_ok(X, loc, glen);
    if (!ok) {
        uint32_t endOffset;
        if ((uint64_t)loc + n + MAX_K >= X.nBases) endOffset = X.nBases;
        else {   // getPieceAtLocation(loc + n + MAX_K)->beginningOffset (Genome.cpp:356-374)
            const uint32_t at = loc + n + MAX_K;
            int lo = 0, hi = X.nPieces - 1, pc = -1;
            while (lo <= hi) {
                const int m = (lo + hi) / 2;
                if (X.pieces[m] <= at && (m == X.nPieces - 1 || X.pieces[m + 1] > at)) { pc = m; break; }
                else if (X.pieces[m] <= at) lo = m + 1;
                else hi = m - 1;
            }
            endOffset = pc >= 0 ? X.pieces[pc] : 0u;
        }
        glen = endOffset - loc - 1;
        if (glen >= n - (uint32_t)MAX_K) ok = substring_ok(X, loc, glen);
    }
    if (!ok) { score = FAIL_SCORE; prob = 0; return; }
    Bitmap<NB> F;
    if constexpr (MAXLEN <= 256) {
        // lane l holds diagonal x = l - 31: F_x[m] = read[m] != genome[loc + x + m] from the genome
        // and read bit planes (as lv_pass, align_score.h); bytes past the read are not ACGT
        const int64_t gp = (int64_t)loc + (lane - 31) + PACK_GUARD;
        const GPlane *src = X.gpl + (gp >> 5);
        const uint32_t sh = (uint32_t)gp & 31;
        GPlane w[2 * NB + 1];
#pragma unroll
        for (int j = 0; j < 2 * NB + 1; j++) w[j] = src[j];
        const uint64_t(*rp)[PLds<MAXLEN>::PW] = S.rpl[r][dir];
#pragma unroll
        for (int b = 0; b < NB; b++) {
            uint32_t f[2];
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const int j = 2 * b + h;
                const uint32_t gh = __builtin_amdgcn_alignbit(w[j + 1].hi, w[j].hi, sh);
                const uint32_t gl = __builtin_amdgcn_alignbit(w[j + 1].lo, w[j].lo, sh);
                const uint32_t gm = __builtin_amdgcn_alignbit(w[j + 1].nm, w[j].nm, sh);
                const uint32_t sft = 32 * h;
                f[h] = (gh ^ (uint32_t)(rp[0][b] >> sft)) | (gl ^ (uint32_t)(rp[1][b] >> sft)) | gm | (uint32_t)(rp[2][b] >> sft);
            }
            F.w[b] = ((uint64_t)f[1] << 32) | f[0];
        }
    } else {
        // genome bytes [loc - 64, loc + n + 128) into LDS (4-byte aligned start), byte compares
        const int64_t astart = ((int64_t)loc - 64) & ~(int64_t)3;
        const int nwords = ((int)n + 192 + 4) / 4;
        const uint32_t *src = (const uint32_t *)(X.genome + astart);
        for (int i = lane; i < nwords && i < (MAXLEN + 192) / 4; i += WAVE) S.win[i] = src[i];
        wave_sync();
        const int w0 = (int)((int64_t)loc - astart);
        const int kmax = scoreLimit < (uint32_t)(MAX_K - 1) ? (int)scoreLimit : MAX_K - 1;
        uint32_t rb[NB];
#pragma unroll
        for (int b = 0; b < NB; b++) rb[b] = (uint8_t)S.rd[r][dir][b * 64 + lane];
        build_bitmap<NB>(F, rb, rb, false, (const char *)S.win, w0, (int)n, kmax);
    }
    const char *q = S.rq[r][dir];
    const int s = (int)seedOffset, t = s + (int)X.seedLen;
    const LvOut r1 = lv_wave<1, NB>(F, t, (int)n - t, (int)glen - t, (int)scoreLimit, q, S.u.lv.rows, S.u.lv.btAct,
                                    S.u.lv.btMatched, X.tab);
    if (r1.score == -1) { score = FAIL_SCORE; prob = 0; return; }
    const int limitLeft = (int)scoreLimit - r1.score;
    const LvOut r2 = lv_wave<-1, NB>(F, s - 1, s, s + MAX_K, limitLeft, q, S.u.lv.rows, S.u.lv.btAct, S.u.lv.btMatched, X.tab);
    offset = r2.netIndel;
    if (r2.score == -1) { score = FAIL_SCORE; prob = 0; return; }
    score = (uint32_t)(r1.score + r2.score);
    prob = r1.prob * r2.prob * X.tab->seedProb;
}

// ------------------------------------------------------------------ a pair
struct PairOut {
    snapgpu_pair_result_t r;
};

template <int MAXLEN>
__device__ void write_result(const PArgs &P, uint32_t pi, const snapgpu_pair_result_t &res) {
    if (lane_id() == 0) {
        snapgpu_pair_result_t o = res;
        o.writtenBy = P.passId;   // routing record (diagnostic): which pass wrote it
        P.out[pi] = o;
    }
}

__device__ __forceinline__ void pre_state(snapgpu_pair_result_t &r) {
    r.location[0] = r.location[1] = INVALID;
    r.score[0] = r.score[1] = -1;
    r.mapq[0] = r.mapq[1] = 0;
    r.status[0] = r.status[1] = SNAPGPU_NOT_FOUND;
    r.direction[0] = r.direction[1] = 0;
    r.fromAlignTogether = 0; r.alignedAsPair = 0; r.flags = 0;
    r.nLocationsScored = 0; r.nSingleScored = 0; r.popularSeedsSkipped = 0; r.writtenBy = 0;
    r.probabilityOfAllPairs = 0; r.probabilityOfBestPair = 0;
}

template <int MAXLEN>
__device__ void defer_pair(const PArgs &P, uint32_t pi) {
    if (!P.deferList) {   // pass 2 never defers (its pools are the reference's); flag instead of losing the pair
        snapgpu_pair_result_t res;
        pre_state(res);
        res.flags = SNAPGPU_PFLAG_POOL_EXHAUSTED;
        write_result<MAXLEN>(P, pi, res);
        return;
    }
    if (lane_id() == 0) P.deferList[atomicAdd(P.deferCount, 1u)] = pi;
}

// Phase 1 (IntersectingPairedEndAligner.cpp:259-340).  The seed walk of a read depends only on
// its bases, so both reads' seeds are chosen first, then looked up in one round, one lane per seed.
template <int MAXLEN>
__device__ __forceinline__ uint32_t choose_seeds(const PArgs &P, PLds<MAXLEN> &S, const int r, const uint32_t nr,
                                                 const uint32_t maxSeeds) {
    constexpr int NB = MAXLEN / 64;
    const KArgs &X = P.X;
    const int lane = lane_id();
    const uint32_t seedLen = X.seedLen;
#pragma unroll
    for (int d = 0; d < 2; d++)
        if (lane == 0) { S.u.walk.hs[r][d].nLookups = 0; S.u.walk.hs[r][d].curSet = -1; S.u.walk.hs[r][d].lastReturned = 0; }
    const uint32_t nPossible = nr - seedLen + 1;
    // Seed::DoesTextRepresentASeed per start position, and a clear seedUsed
#pragma unroll
    for (int b = 0; b < NB; b++) {
        const uint32_t p = (uint32_t)(b * 64 + lane);
        bool valid = p < nPossible;
        for (uint32_t i = 0; valid && i < seedLen; i++) {
            const char c = S.rd[r][0][p + i];
            valid = c == 'A' || c == 'C' || c == 'G' || c == 'T';
        }
        const uint64_t vb = ballot(valid);
        if (lane == 0) { S.validBits[b] = vb; S.usedBits[b] = 0; }
    }
    wave_sync();
    // SeedSequencer walk (scalar): offsets do not depend on lookup results
    uint32_t nSel = 0, next = 0, wrap = 0;
    bool wrapped = false;
    for (uint32_t guard = 0; nSel < nPossible && nSel < maxSeeds && guard < 4096; guard++) {
        if (next >= nPossible) {
            wrap++;
            wrapped = true;
            if (wrap >= seedLen) break;
            next = X.tab->wrap[wrap];
        }
        while (next < nPossible && ((S.usedBits[next >> 6] >> (next & 63)) & 1)) next++;
        if (next >= nPossible) continue;
        const uint64_t ub = S.usedBits[next >> 6] | (1ull << (next & 63));
        wave_sync();
        S.usedBits[next >> 6] = ub;
        wave_sync();
        if (!((S.validBits[next >> 6] >> (next & 63)) & 1)) { next++; continue; }   // :296-302
        S.sel[r][nSel] = next | (wrapped ? 0x80000000u : 0u);
        wrapped = false;
        nSel++;
        if ((maxSeeds - nSel + 1) * seedLen + next < nPossible)                      // :333-338
            next += (nPossible + next) / (maxSeeds - nSel + 1);
        else next += seedLen;
    }
    wave_sync();
    return nSel;
}

// GenomeIndex::lookupSeed (GenomeIndex.cpp:971-1086) for the chosen seeds of both reads at
// once: lanes 0-31 take read 0's seeds, lanes 32-63 read 1's.
template <int MAXLEN>
__device__ __forceinline__ void lookup_seeds(const PArgs &P, PLds<MAXLEN> &S, const uint32_t n0, const uint32_t n1,
                                             const uint32_t nSel0, const uint32_t nSel1) {
    const KArgs &X = P.X;
    const int lane = lane_id();
    const uint32_t seedLen = X.seedLen;
    const int r = lane >> 5, k = lane & 31;
    const uint32_t nr = r ? n1 : n0;
    if ((uint32_t)k < (r ? nSel1 : nSel0)) {
        const uint32_t so = S.sel[r][k] & 0x7fffffffu;
        uint64_t f = 0, rv = 0;
        for (uint32_t i = 0; i < seedLen; i++) {
            const int v = base_value((uint8_t)S.rd[r][0][so + i]);
            f |= (uint64_t)v << ((seedLen - i - 1) * 2);
            rv |= (uint64_t)(v ^ 3) << (i * 2);
        }
        const bool comp = (int64_t)f > (int64_t)rv;
        const uint64_t canon = comp ? rv : f;
        const uint32_t table = (uint32_t)(canon >> 32), key = (uint32_t)canon;
        // SNAPHashTable::Lookup (HashTable.h:74-105) answered by the bucket image (bucket_table.h)
        uint32_t v1 = 0, v2 = 0, aux = 0, lines = 0;
        const bool found = bucket_lookup_lane(X, table, key, v1, v2, aux, lines);
        uint32_t nh[2] = {0, 0}, at[2] = {0, 0}, sg[2] = {0, 0};
        if (found) {
            for (int side = 0; side < 2; side++) {
                if (side == 1 && f == rv) { nh[1] = nh[0]; at[1] = at[0]; sg[1] = sg[0]; break; }
                const bool first = (side == 0) == !comp;
                const uint32_t v = first ? v1 : v2;
                if (v < X.nBases) { nh[side] = 1; at[side] = v; sg[side] = 1; }
                else if (v != UNUSED_SIDE) {   // the list length from the entry (saturated: from the list)
                    nh[side] = bucket_count(X, first ? (aux & BK_CSAT) : ((aux >> 15) & BK_CSAT), v);
                    at[side] = v - X.nBases + 1;
                }
            }
        }
        // recordLookup's trim of the hits below the seed offset (:882-884), one lane per seed here
        uint32_t tr[2];
#pragma unroll
        for (int d = 0; d < 2; d++) {
            const uint32_t offset = d == 0 ? so : nr - seedLen - so;
            uint32_t t = nh[d];
            if (nh[d] < P.maxBigHits)
                while (t > 0 && (sg[d] ? at[d] : X.overflow[at[d] + t - 1]) < offset) t--;
            tr[d] = t;
        }
        S.u.walk.look[r][k][0] = nh[0] | (sg[0] << 31); S.u.walk.look[r][k][1] = at[0]; S.u.walk.look[r][k][2] = tr[0];
        S.u.walk.look[r][k][3] = nh[1] | (sg[1] << 31); S.u.walk.look[r][k][4] = at[1]; S.u.walk.look[r][k][5] = tr[1];
    }
    wave_sync();
    wave_sync();
}

// The hit sets of read r in the reference's order (:313-328): where a disjoint hit set begins
// depends on which lookups were recorded (a lookup with >= maxBigHits hits is skipped).
__device__ __forceinline__ void record_hits(const PArgs &P, HitSet (&hs)[2], const uint32_t (&look)[LCAP][6],
                                            const uint32_t *sel, const uint32_t nSel, const uint32_t nr,
                                            uint32_t &totF, uint32_t &totR, uint32_t &popular) {
    const uint32_t seedLen = P.X.seedLen;
    bool begins[2] = {true, true};
    for (uint32_t k = 0; k < nSel; k++) {
        const uint32_t sk = sel[k];
        if (sk & 0x80000000u) begins[0] = begins[1] = true;
        const uint32_t so = sk & 0x7fffffffu;
#pragma unroll
        for (int d = 0; d < 2; d++) {
            const uint32_t offset = d == 0 ? so : nr - seedLen - so;
            const uint32_t nh = look[k][3 * d] & 0x7fffffffu;
            if (nh < P.maxBigHits) {
                if (d == 0) totF += nh; else totR += nh;
                hs_record(hs[d], offset, nh, look[k][3 * d + 2], look[k][3 * d + 1], look[k][3 * d] >> 31,
                          begins[d]);
                begins[d] = false;
            } else popular++;
        }
    }
    wave_sync();
}

// Read r of the pair into LDS: Read::init upper-cases; RC data and reversed qualities
// (:217-224); zero slack.  Returns this lane's count of 'N' (:220), plus 0x10000 per 0x00 byte
// inside the read (SNAPGPU_PFLAG_NUL_BYTE: a corrupted upload; no reader produces one).
template <int MAXLEN>
__device__ __forceinline__ uint32_t load_read(const PArgs &P, PLds<MAXLEN> &S, const int r, const uint32_t nr,
                                              const uint64_t offr) {
    const int lane = lane_id();
    const char *b = P.bases[r] + offr, *q = P.quals[r] + offr;
    uint32_t ns = 0;
    for (int i = lane; i < MAXLEN + 64; i += WAVE) {
        char c = 0, cq = 0, cc = 0;
        if ((uint32_t)i < nr) {
            c = b[i];
            if (c >= 'a' && c <= 'z') c = (char)(c - 0x20);
            cq = q[i];
            cc = c == 'A' ? 'T' : c == 'G' ? 'C' : c == 'C' ? 'G' : c == 'T' ? 'A' : c == 'N' ? 'N' : 0;
            ns += c == 'N' ? 1u : (c == 0 ? 0x10000u : 0u);
            S.rd[r][1][nr - 1 - i] = cc;
            S.rq[r][1][nr - 1 - i] = cq;
        } else {
            S.rd[r][1][i] = 0;
            S.rq[r][1][i] = 0;
        }
        S.rd[r][0][i] = c;
        S.rq[r][0][i] = cq;
    }
    return ns;
}

// IntersectingPairedEndAligner::align (:142-753).  Returns after writing out[pi] or deferring.
// Reads are indexed 0/1; `fewer` / `more` are selects, never array indices (no scratch).
template <int MAXLEN>
__device__ void align_pair(const PArgs &P, PLds<MAXLEN> &S, Cand *cand, Mate *mates0, Mate *mates1, Anchor *anchors,
                           uint32_t pi) {
    const KArgs &X = P.X;
    const int lane = lane_id();
    const uint32_t seedLen = X.seedLen;
    const uint32_t maxK = P.maxK, extra = P.extra;
    snapgpu_pair_result_t res;
    pre_state(res);
    if (P.deferred) res.flags |= SNAPGPU_PFLAG_DEFERRED;
    const uint32_t n0 = P.lengths[0][pi], n1 = P.lengths[1][pi];
    const uint64_t o0 = P.offsets[0][pi], o1 = P.offsets[1][pi];
    if (n0 < 50 || n1 < 50) { write_result<MAXLEN>(P, pi, res); return; }         // :186-188
    if (n0 > P.maxReadSize || n1 > P.maxReadSize) {                                // :211-215 (soft_exit)
        res.flags |= SNAPGPU_PFLAG_READ_TOO_LONG;
        write_result<MAXLEN>(P, pi, res);
        return;
    }
    if (n0 > P.maxLen || n1 > P.maxLen) { defer_pair<MAXLEN>(P, pi); return; }
    uint32_t countNs = load_read<MAXLEN>(P, S, 0, n0, o0) + load_read<MAXLEN>(P, S, 1, n1, o1);
    wave_sync();
    if constexpr (MAXLEN <= 256) {
        // read bit planes of both reads and directions; a genome with IUPAC codes and a read with
        // a non-ACGTN byte need byte compares (an IUPAC code can match itself): the <512> passes
        bool other = false;
#pragma unroll
        for (int r = 0; r < 2; r++)
#pragma unroll
            for (int dr = 0; dr < 2; dr++)
#pragma unroll
                for (int h = 0; h < PLds<MAXLEN>::NB; h++) {
                    const uint8_t c = (uint8_t)S.rd[r][dr][h * 64 + lane];
                    const uint32_t code = packed_code(c);
                    const uint64_t bh = ballot(code < 4 && (code & 2)), bl = ballot(code < 4 && (code & 1));
                    const uint64_t bm = ballot(code > 3);
                    other = other || (c != 0 && code > 3 && c != 'N');
                    if (lane == 0) { S.rpl[r][dr][0][h] = bh; S.rpl[r][dr][1][h] = bl; S.rpl[r][dr][2][h] = bm; }
                }
        wave_sync();
        if (X.hasIupac && ballot(other)) { defer_pair<MAXLEN>(P, pi); return; }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) countNs += (uint32_t)__shfl_xor((int)countNs, o);
    countNs = uni(countNs);
    if (countNs >> 16) res.flags |= SNAPGPU_PFLAG_NUL_BYTE;
    countNs &= 0xffffu;
    if (countNs > maxK) { write_result<MAXLEN>(P, pi, res); return; }              // :226-228
    uint32_t maxSeeds = P.maxSeedsCmd ? P.maxSeedsCmd
                                      : (uint32_t)((n0 > n1 ? n0 : n1) * P.seedCoverage / seedLen);   // :150-155
    if (maxSeeds > (uint32_t)LCAP) maxSeeds = LCAP;
    // ---------------------------------------------------------------- phase 1 (:259-340)
    uint32_t pop0 = 0, pop1 = 0, t00 = 0, t01 = 0, t10 = 0, t11 = 0;
    const uint32_t nSel0 = choose_seeds<MAXLEN>(P, S, 0, n0, maxSeeds);
    const uint32_t nSel1 = choose_seeds<MAXLEN>(P, S, 1, n1, maxSeeds);
    lookup_seeds<MAXLEN>(P, S, n0, n1, nSel0, nSel1);
    record_hits(P, S.u.walk.hs[0], S.u.walk.look[0], S.sel[0], nSel0, n0, t00, t01, pop0);
    record_hits(P, S.u.walk.hs[1], S.u.walk.look[1], S.sel[1], nSel1, n1, t10, t11, pop1);
    const uint32_t popularAll = pop0 + pop1;
    const int more = t00 + t01 > t10 + t11 ? 0 : 1, fewer = 1 - more;            // :342-343
    const uint32_t nFewer = fewer ? n1 : n0, nMore = fewer ? n0 : n1;
    // ---------------------------------------------------------------- phase 2 (:357-511)
    for (int k = lane; k < MAX_LISTS; k += WAVE) S.lists[k] = -1;
    wave_sync();
    uint32_t nCand = 0, nAnchor = 0, maxUsedList = 0;
    const uint32_t maxSp = P.maxSpacing, minSp = P.minSpacing;
    bool deferIt = false, exhausted = false;
    for (int sp = 0; sp < 2 && !deferIt && !exhausted; sp++) {
        // set pair 0 = read0 FORWARD + read1 RC, set pair 1 = read0 RC + read1 FORWARD (:351, :361-367)
        Walk hf, hm;
        walk_init(P, S.u.walk.hs[fewer][fewer ^ sp], hf);
        walk_init(P, S.u.walk.hs[more][more ^ sp], hm);
        Mate *ms = sp ? mates1 : mates0;
        uint32_t nM = 0;
        uint32_t fewerLoc = 0, fewerSeed = 0, moreLoc, moreSeed = 0;
        bool outOfMore = false;
        if (!hs_first(hf, fewerLoc, fewerSeed)) continue;
        moreLoc = INVALID;
        for (;;) {
            if (moreLoc > fewerLoc + maxSp) {
                if (!hs_next_le(P, hm, fewerLoc + maxSp, moreLoc, moreSeed)) break;
            }
            if (moreLoc + maxSp < fewerLoc && (nM == 0 || !is_within(ms[nM - 1].loc, fewerLoc, maxSp))) {
                if (!hs_next_le(P, hf, moreLoc + maxSp, fewerLoc, fewerSeed)) break;
                continue;
            }
            while (moreLoc + maxSp >= fewerLoc && !outOfMore) {
                const uint32_t bps = hs_best_possible<MAXLEN>(S, hm, maxK);
                if (nM >= P.refPool / 2) { exhausted = true; break; }                   // :436-439
                if (nM >= P.mateCap) { deferIt = true; break; }
                Mate m;
                m.prob = 0; m.loc = moreLoc; m.bestPossible = bps; m.score = UNSCORED; m.scoreLimit = 0xffffffffu;
                m.seedOffset = moreSeed; m.genomeOffset = 0;
                ms[nM] = m;
                nM++;
                if (!hs_next_lower(P, hm, moreLoc, moreSeed)) { moreLoc = 0; outOfMore = true; break; }
            }
            if (deferIt || exhausted) break;
            const uint32_t bpsF = hs_best_possible<MAXLEN>(S, hf, maxK);
            // lowest best possible score of the mates up to maxSpacing above this fewer hit,
            // 64 mates per step from the lowest up (:469-475)
            uint32_t lowest = maxK + extra;
            wave_sync();
            for (int base = (int)nM - 1; base >= 0; base -= WAVE) {
                const int i = base - lane;
                uint32_t ml = 0, mb = 0xffffffffu;
                if (i >= 0) { ml = ms[i].loc; mb = ms[i].bestPossible; }
                const uint64_t brk = ballot(i >= 0 && ml > fewerLoc + maxSp);
                const int first = brk ? (int)__builtin_ctzll(brk) : WAVE;
                const uint32_t c = (i >= 0 && lane < first) ? mb : 0xffffffffu;
                const uint32_t mn = ~uni(max_reduce32(~c));
                if (mn < lowest) lowest = mn;
                if (brk) break;
            }
            if (lowest + bpsF <= maxK + extra) {
                if (nCand >= P.refPool) { exhausted = true; break; }                    // :482-485
                if (nCand >= P.candCap) { deferIt = true; break; }
                const uint32_t li = lowest + bpsF;
                Cand c;
                c.next = S.lists[li]; c.anchor = -1; c.mateIndex = nM - 1; c.loc = fewerLoc;
                c.setPair = (uint32_t)sp; c.seedOffset = fewerSeed; c.bestPossible = bpsF; c.pad = 0;
                cand[nCand] = c;
                wave_sync();
                S.lists[li] = (int32_t)nCand;
                wave_sync();
                nCand++;
                if (li > maxUsedList) maxUsedList = li;
            }
            if (!hs_next_lower(P, hf, fewerLoc, fewerSeed)) break;
        }
    }
    if (exhausted) { res.flags |= SNAPGPU_PFLAG_POOL_EXHAUSTED; write_result<MAXLEN>(P, pi, res); return; }
    if (deferIt) { defer_pair<MAXLEN>(P, pi); return; }
    // ---------------------------------------------------------------- phase 3 (:516-718)
    double pBest = 0, pAll = 0;
    uint32_t bestPairScore = 65536, scoreLimit = maxK + extra, list = 0;
    uint32_t bestLocF = 0, bestLocM = 0, bestScoreF = 0, bestScoreM = 0, bestSp = 0;
    uint32_t nScored = 0;
    while (list <= maxUsedList && list <= scoreLimit) {
        const int ci = S.lists[list];
        if (ci < 0) { list++; continue; }
        const Cand c = cand[ci];
        uint32_t fewerScore = 0;
        double fewerProb = 0;
        int32_t fewerOff = 0;
        // direction of read r in set pair sp: r ^ sp (setPairDirection, :351)
        score_location<MAXLEN>(P, S, fewer, fewer ^ (int)c.setPair, nFewer, c.loc, c.seedOffset, scoreLimit, fewerScore,
                               fewerProb, fewerOff, nScored);
        if (fewerScore != FAIL_SCORE) {
            Mate *ms = c.setPair ? mates1 : mates0;
            int32_t anchorOf = c.anchor;
            uint32_t mi = c.mateIndex;
            for (;;) {
                Mate m = ms[mi];
                if (!is_within(m.loc, c.loc, minSp) && m.bestPossible <= scoreLimit - fewerScore) {
                    if (m.score == UNSCORED || (m.score == FAIL_SCORE && m.scoreLimit < scoreLimit - fewerScore)) {
                        score_location<MAXLEN>(P, S, more, more ^ (int)c.setPair, nMore, m.loc, m.seedOffset,
                                               scoreLimit - fewerScore, m.score, m.prob, m.genomeOffset, nScored);
                        m.scoreLimit = scoreLimit - fewerScore;
                        ms[mi] = m;
                        wave_sync();
                    }
                    if (m.score != FAIL_SCORE) {
                        const double pairProb = m.prob * fewerProb;
                        const uint32_t pairScore = m.score + fewerScore;
                        const uint32_t fewerAt = c.loc + (uint32_t)fewerOff, moreAt = m.loc + (uint32_t)m.genomeOffset;
                        int32_t an = anchorOf;
                        if (an < 0) {   // :602-626, including the second loop's decrement
                            for (int j = ci - 1; j >= 0; j--) {
                                const Cand o = cand[j];
                                if (!(is_within(o.loc, fewerAt, 50) && o.setPair == c.setPair)) break;
                                if (o.anchor >= 0) { an = o.anchor; break; }
                            }
                            if (an < 0)
                                for (int j = ci + 1; j >= 0 && j < (int)nCand; j--) {
                                    const Cand o = cand[j];
                                    if (!(is_within(o.loc, fewerAt, 50) && o.setPair == c.setPair)) break;
                                    if (o.anchor >= 0) { an = o.anchor; break; }
                                }
                            if (an >= 0) { anchorOf = an; cand[ci].anchor = an; wave_sync(); }
                        }
                        bool merged;
                        double oldProb;
                        if (an < 0) {
                            if (nAnchor >= P.refPool) { exhausted = true; break; }               // :634-637
                            if (nAnchor >= P.anchorCap) { deferIt = true; break; }
                            an = (int32_t)nAnchor++;
                            Anchor a;
                            a.moreLoc = moreAt; a.fewerLoc = fewerAt; a.prob = pairProb; a.pairScore = (int32_t)pairScore; a.pad = 0;
                            anchors[an] = a;
                            anchorOf = an;
                            cand[ci].anchor = an;
                            wave_sync();
                            merged = false; oldProb = 0;
                        } else {   // MergeAnchor::checkMerge (:1324-1371)
                            Anchor a = anchors[an];
                            if (a.moreLoc == INVALID ||
                                !(loc_distance(a.moreLoc, moreAt) < 50 && loc_distance(a.fewerLoc, fewerAt) < 50)) {
                                a.moreLoc = moreAt; a.fewerLoc = fewerAt; a.prob = pairProb; a.pairScore = (int32_t)pairScore;
                                oldProb = 0; merged = false;
                            } else if ((int32_t)pairScore < a.pairScore || ((int32_t)pairScore == a.pairScore && pairProb > a.prob)) {
                                oldProb = a.prob; a.prob = pairProb; a.pairScore = (int32_t)pairScore; merged = false;
                            } else { merged = true; oldProb = 0; }
                            anchors[an] = a;
                            wave_sync();
                        }
                        if (!merged) {
                            pAll = pAll - oldProb > 0 ? pAll - oldProb : 0;   // __max(0, .)
                            if (pairScore <= maxK && (pairScore < bestPairScore || (pairScore == bestPairScore && pairProb > pBest))) {
                                bestPairScore = pairScore;
                                pBest = pairProb;
                                bestLocF = fewerAt; bestLocM = moreAt;
                                bestScoreF = fewerScore; bestScoreM = m.score;
                                bestSp = c.setPair;
                                scoreLimit = bestPairScore + extra;
                            }
                            pAll += pairProb;
                            if (pAll >= 4.9) goto doneScoring;
                        }
                    }
                }
                if (mi == 0 || !is_within(ms[mi - 1].loc, c.loc, maxSp)) break;
                mi--;
            }
            if (deferIt || exhausted) break;
        }
        S.lists[list] = c.next;
        wave_sync();
    }
doneScoring:
    if (exhausted) { res.flags |= SNAPGPU_PFLAG_POOL_EXHAUSTED; write_result<MAXLEN>(P, pi, res); return; }
    if (deferIt) { defer_pair<MAXLEN>(P, pi); return; }
    res.nLocationsScored = nScored;
    res.probabilityOfAllPairs = pAll;
    res.probabilityOfBestPair = pBest;
    res.popularSeedsSkipped = popularAll;
    if (bestPairScore == 65536) {
        res.location[0] = res.location[1] = INVALID;
        res.mapq[0] = res.mapq[1] = 0;
        res.score[0] = res.score[1] = -1;
        res.status[0] = res.status[1] = SNAPGPU_NOT_FOUND;
    } else {
        const uint32_t loc0 = fewer == 0 ? bestLocF : bestLocM, loc1 = fewer == 0 ? bestLocM : bestLocF;
        const uint32_t sc0 = fewer == 0 ? bestScoreF : bestScoreM, sc1 = fewer == 0 ? bestScoreM : bestScoreF;
        uint32_t fl = 0;
        const int mq0 = mapq_dev(X.tab, pAll, pBest, sc0, popularAll, &fl);
        const int mq1 = mapq_dev(X.tab, pAll, pBest, sc1, popularAll, &fl);
        if (fl & SNAPGPU_FLAG_MAPQ_FIXED) res.flags |= SNAPGPU_PFLAG_MAPQ_FIXED;
        res.location[0] = loc0; res.location[1] = loc1;
        res.direction[0] = (uint8_t)(0 ^ bestSp); res.direction[1] = (uint8_t)(1 ^ bestSp);
        res.mapq[0] = mq0; res.mapq[1] = mq1;
        res.status[0] = mq0 > 10 ? SNAPGPU_SINGLE_HIT : SNAPGPU_MULTIPLE_HITS;
        res.status[1] = mq1 > 10 ? SNAPGPU_SINGLE_HIT : SNAPGPU_MULTIPLE_HITS;
        res.score[0] = (int32_t)sc0; res.score[1] = (int32_t)sc1;
    }
    write_result<MAXLEN>(P, pi, res);
}

template <int MAXLEN>
__global__ __launch_bounds__(64) void paired_kernel(PArgs P) {
    __shared__ PLds<MAXLEN> S;
    char *base = P.pool + (uint64_t)blockIdx.x * P.poolStride;
    Cand *cand = reinterpret_cast<Cand *>(base);
    Mate *m0 = reinterpret_cast<Mate *>(base + (uint64_t)P.candCap * sizeof(Cand));
    Mate *m1 = m0 + P.mateCap;
    Anchor *an = reinterpret_cast<Anchor *>(m1 + P.mateCap);
    for (;;) {
        uint32_t t = 0;
        if (lane_id() == 0) t = atomicAdd(P.counter, 1u);
        t = uni(t);
        if (t >= P.nPairs) break;
        const uint32_t pi = P.pairList ? P.pairList[t] : t;
        align_pair<MAXLEN>(P, S, cand, m0, m1, an, pi);
    }
}

// Weight of each long pair for the longest-first order of pass 1b (order_long.h): the summed hit
// counts of both ends' seeds at offsets 0, L, 2L, .. inside their first 128 bases, a seed counted
// only below maxBigHits (the lookups the intersecting walk records, :518-524) and only when all
// ACGT.  Two pairs per wave, 16 lanes per end (lane 32j + 16e + k: seed k of end e of pair j).
// list[i] (i < *count) = pair index; out[i] = pair | class << 28 for order_long_kernel.
__global__ __launch_bounds__(256) void pair_weight_kernel(PArgs P, const uint32_t *list, const uint32_t *count, uint32_t *out) {
    const KArgs &X = P.X;
    const int lane = lane_id();
    const uint32_t n = *count, L = X.seedLen;
    const uint32_t wave = blockIdx.x * 4u + threadIdx.x / 64u, nWaves = gridDim.x * 4u;
    for (uint32_t b = 2u * wave; b < n; b += 2u * nWaves) {   // wave-uniform trip count
        const uint32_t i = b + (uint32_t)(lane >> 5);
        const int e = (lane >> 4) & 1, k = lane & 15;
        const uint32_t pi = i < n ? list[i] : 0u;
        const uint32_t len = i < n ? P.lengths[e][pi] : 0u;
        const uint32_t lim = len < 128u ? len : 128u;
        const uint32_t so = (uint32_t)k * L;
        bool act = i < n && so + L <= lim;
        uint64_t f = 0, rv = 0;
        if (act) {
            const char *rd = P.bases[e] + P.offsets[e][pi] + so;
            for (uint32_t j = 0; j < L; j++) {
                const int v = base_value((uint8_t)rd[j]);
                act = act && v <= 3;
                f |= (uint64_t)(v & 3) << ((L - j - 1) * 2);
                rv |= (uint64_t)((v & 3) ^ 3) << (j * 2);
            }
        }
        const bool comp = (int64_t)f > (int64_t)rv;
        const uint64_t canon = comp ? rv : f;
        uint32_t v1 = 0, v2 = 0, aux = 0, lines = 0;
        const bool found = bucket_lookup_quad(X, act, (uint32_t)(canon >> 32), (uint32_t)canon, v1, v2, aux, lines);
        uint32_t w = 0;
        if (act && found) {
            auto side = [&](uint32_t v, uint32_t c) -> uint32_t {
                const uint32_t h = v == UNUSED_SIDE ? 0u : v < X.nBases ? 1u : c >= BK_CSAT ? 0xffffu : c;
                return h < P.maxBigHits ? h : 0u;
            };
            w = side(v1, aux & BK_CSAT) + (f != rv ? side(v2, (aux >> 15) & BK_CSAT) : 0u);
        }
#pragma unroll
        for (int s = 16; s >= 1; s >>= 1) w += (uint32_t)__shfl_xor((int)w, s, 64);   // the pair's 32 lanes
        if ((lane & 31) == 0 && i < n) out[i] = pi | (order_class(w) << ORDER_CLASS_SHIFT);
    }
}

}  // namespace pe
}  // namespace sgk

using namespace sgk;
using namespace sgk::pe;

// ======================================================================= host
namespace {

#define PCHK(x)                                                                         \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            snapgpu::setError(std::string(#x) + ": " + hipGetErrorString(e_));          \
            return SNAPGPU_EDEVICE;                                                     \
        }                                                                               \
    } while (0)

std::mutex g_tabMu;
bool g_tabDone[64] = {};

hipError_t ensurePairedTables(int device) {   // this translation unit's g_tab (align_device.h)
    std::lock_guard<std::mutex> lk(g_tabMu);
    if (device < 0 || device >= 64) return hipErrorInvalidDevice;
    if (g_tabDone[device]) return hipSuccess;
    DevTables t;
    snapgpu_internal_fill_tables(&t, 20);
    hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(g_tab), &t, sizeof(t), 0, hipMemcpyHostToDevice);
    if (e == hipSuccess) g_tabDone[device] = true;
    return e;
}

struct PassPool {
    char *pool = nullptr;
    uint64_t stride = 0;
    int grid = 0;
    uint32_t candCap = 0, mateCap = 0, anchorCap = 0;
};

}  // namespace

struct snapgpu_paired_aligner {
    int device = 0;
    snapgpu_paired_params_t p{};
    snapgpu_aligner_t *single = nullptr;   // the chimeric fallback's BaseAligner; owns the index upload
    KArgs X{};
    hipStream_t stream = nullptr;
    PassPool pass[3];                      // [0] passes 1 and 1b, [1] pass 3 (the reference's pools), [2] pass 2
    int grid256 = 0;                       // pass 1b (<256>) grid: at most pass[0].grid (its pools)
    uint32_t refPool = 0, maxSeedsCmd = 0;
    uint32_t *dCounter = nullptr;          // [0] pass 1 queue, [1] pass 3 queue, [2] pass-1 defer count,
                                           // [3] pass 2 queue, [4] pass-2 defer count, [5] pass 1b queue,
                                           // [6] pass-1b defer count
    uint32_t *dDefer = nullptr, *dDefer2 = nullptr;
    uint32_t *dOrder = nullptr, *dOrderW = nullptr;   // long pairs before / after pair_weight_kernel
    bool orderLong = true;                 // pass 1b longest-first (SNAPGPU_ORDER_LONG=0: input order)
    snapgpu_pair_result_t *dOut = nullptr;
    char *dB[2] = {}, *dQ[2] = {};
    uint64_t *dO[2] = {};
    uint32_t *dL[2] = {};
    uint64_t capPairs = 0, capBytes[2] = {0, 0};
};

static void pfree(void *p) { if (p) (void)hipFree(p); }

static int ensurePairCapacity(snapgpu_paired_aligner_t *pa, uint64_t n, const uint64_t bytes[2]) {
    if (n > pa->capPairs) {
        pfree(pa->dOut); pfree(pa->dDefer); pfree(pa->dDefer2); pfree(pa->dO[0]); pfree(pa->dO[1]); pfree(pa->dL[0]); pfree(pa->dL[1]);
        pfree(pa->dOrder); pfree(pa->dOrderW);
        pa->dOut = nullptr; pa->dDefer = nullptr; pa->dDefer2 = nullptr; pa->dO[0] = pa->dO[1] = nullptr; pa->dL[0] = pa->dL[1] = nullptr;
        pa->dOrder = pa->dOrderW = nullptr;
        pa->capPairs = 0;
        PCHK(hipMalloc(&pa->dOut, n * sizeof(snapgpu_pair_result_t)));
        PCHK(hipMalloc(&pa->dDefer, n * 4 + 16));
        PCHK(hipMalloc(&pa->dDefer2, n * 4 + 16));
        PCHK(hipMalloc(&pa->dOrder, n * 4 + 16));
        PCHK(hipMalloc(&pa->dOrderW, n * 4 + 16));
        for (int r = 0; r < 2; r++) {
            PCHK(hipMalloc(&pa->dO[r], n * 8 + 16));
            PCHK(hipMalloc(&pa->dL[r], n * 4 + 16));
        }
        pa->capPairs = n;
    }
    for (int r = 0; r < 2; r++)
        if (bytes[r] + 1024 > pa->capBytes[r]) {
            pfree(pa->dB[r]); pfree(pa->dQ[r]);
            pa->dB[r] = pa->dQ[r] = nullptr;
            pa->capBytes[r] = 0;
            const uint64_t c = bytes[r] + (bytes[r] >> 3) + 4096;
            PCHK(hipMalloc(&pa->dB[r], c));
            PCHK(hipMalloc(&pa->dQ[r], c));
            // zeroed on the aligner's stream, ahead of the uploads into them: a plain hipMemset runs
            // on the null stream, which the non-blocking aligner stream does not wait for
            PCHK(hipMemsetAsync(pa->dB[r], 0, c, pa->stream));
            PCHK(hipMemsetAsync(pa->dQ[r], 0, c, pa->stream));
            pa->capBytes[r] = c;
        }
    return SNAPGPU_OK;
}

static int allocPass(PassPool &pp, int grid, uint32_t candCap, uint32_t mateCap, uint32_t anchorCap) {
    pp.grid = grid;
    pp.candCap = candCap; pp.mateCap = mateCap; pp.anchorCap = anchorCap;
    pp.stride = ((uint64_t)candCap * sizeof(Cand) + 2ull * mateCap * sizeof(Mate) + (uint64_t)anchorCap * sizeof(Anchor) +
                 255) & ~255ull;
    PCHK(hipMalloc(&pp.pool, pp.stride * (uint64_t)grid));
    return SNAPGPU_OK;
}

// the intersecting aligner over the whole batch (both passes); records left in pa->dOut
static int runIntersect(snapgpu_paired_aligner_t *pa, const snapgpu_reads_t *r0, const snapgpu_reads_t *r1,
                        snapgpu_pair_result_t *out) {
    const snapgpu_reads_t *R[2] = {r0, r1};
    const uint64_t n = r0->n;
    uint64_t bytes[2] = {r0->totalBytes, r1->totalBytes};
    int rc = ensurePairCapacity(pa, n, bytes);
    if (rc) return rc;
    hipStream_t s = pa->stream;
    for (int r = 0; r < 2; r++) {
        PCHK(hipMemcpyAsync(pa->dB[r], R[r]->bases, R[r]->totalBytes, hipMemcpyHostToDevice, s));
        PCHK(hipMemcpyAsync(pa->dQ[r], R[r]->quals, R[r]->totalBytes, hipMemcpyHostToDevice, s));
        PCHK(hipMemcpyAsync(pa->dO[r], R[r]->offsets, n * 8, hipMemcpyHostToDevice, s));
        PCHK(hipMemcpyAsync(pa->dL[r], R[r]->lengths, n * 4, hipMemcpyHostToDevice, s));
    }
    PCHK(hipMemsetAsync(pa->dCounter, 0, 32, s));
    // records pre-filled with 0xff (status 0xff is no AlignmentResult): a pair that no pass writes
    // fails the call below instead of coming back as a stale or zeroed NotFound-looking record
    PCHK(hipMemsetAsync(pa->dOut, 0xff, n * sizeof(snapgpu_pair_result_t), s));
    PArgs P;
    memset(&P, 0, sizeof(P));
    P.X = pa->X;
    for (int r = 0; r < 2; r++) { P.bases[r] = pa->dB[r]; P.quals[r] = pa->dQ[r]; P.offsets[r] = pa->dO[r]; P.lengths[r] = pa->dL[r]; }
    P.out = pa->dOut;
    P.maxK = pa->p.maxK; P.extra = pa->p.extraSearchDepth; P.maxSeedsCmd = pa->maxSeedsCmd;
    P.minSpacing = pa->p.minSpacing; P.maxSpacing = pa->p.maxSpacing; P.maxBigHits = pa->p.maxBigHits;
    P.maxReadSize = pa->p.maxReadSize; P.seedCoverage = pa->p.seedCoverage;
    P.refPool = pa->refPool;
    auto usePool = [&P](const PassPool &pp) {
        P.pool = pp.pool; P.poolStride = pp.stride;
        P.candCap = pp.candCap; P.mateCap = pp.mateCap; P.anchorCap = pp.anchorCap;
    };
    // The host routes the pairs by length (as pass 0 does for the single-end passes): a pair with a
    // read over 128 bases goes straight onto pass 1b's list, so pass 1 does not visit it only to defer
    // it with an atomic (2.3 ms per 100k 2 x 150 RNA pairs).  Pass 1 takes the rest through its own
    // list (pass 1b's output list, unused until then), or in input order when every pair is short.
    std::vector<uint32_t> shortL, longL;
    for (uint64_t i = 0; i < n; i++)
        (R[0]->lengths[i] > 128 || R[1]->lengths[i] > 128 ? longL : shortL).push_back((uint32_t)i);
    if (!longL.empty()) {
        // longL / shortL outlive the copies (the stream is synchronised below, before they go out of
        // scope); the pass-1 defer count starts at the long pairs' count, set by value (a stack
        // scalar as the source of an asynchronous copy could be read after its scope ended)
        const bool order = pa->orderLong && n < (1ull << ORDER_CLASS_SHIFT);
        PCHK(hipMemcpyAsync(order ? pa->dOrder : pa->dDefer, longL.data(), longL.size() * 4, hipMemcpyHostToDevice, s));
        PCHK(hipMemsetD32Async((hipDeviceptr_t)(pa->dCounter + 2), (int)longL.size(), 1, s));
        if (order) {   // pass 1b's list heaviest first (order_long.h); pass 1 appends its defers after it
            const unsigned blocks = (unsigned)std::min<uint64_t>((longL.size() + 7) / 8, 2048);
            hipLaunchKernelGGL(pair_weight_kernel, dim3(blocks), dim3(256), 0, s, P, pa->dOrder, pa->dCounter + 2, pa->dOrderW);
            PCHK(hipGetLastError());
            hipLaunchKernelGGL(order_long_kernel, dim3(1), dim3(256), 0, s, pa->dOrderW, pa->dCounter + 2, pa->dDefer);
            PCHK(hipGetLastError());
        }
        if (!shortL.empty()) PCHK(hipMemcpyAsync(pa->dDefer2, shortL.data(), shortL.size() * 4, hipMemcpyHostToDevice, s));
    }
    // pass 1: reads <= 128 bases, pools for ordinary pairs, the full grid
    P.nPairs = (uint32_t)shortL.size(); P.pairList = longL.empty() ? nullptr : pa->dDefer2; P.counter = pa->dCounter;
    P.maxLen = 128; P.passId = 1;
    P.deferList = pa->dDefer; P.deferCount = pa->dCounter + 2;
    usePool(pa->pass[0]);
    int grid = pa->pass[0].grid;
    if ((uint64_t)grid > shortL.size()) grid = (int)shortL.size();
    if (grid > 0) hipLaunchKernelGGL(paired_kernel<128>, dim3(grid), dim3(64), 0, s, P);
    PCHK(hipGetLastError());
    P.deferred = 1;   // every later pass takes deferred pairs
    uint32_t nDefer = 0;
    PCHK(hipMemcpyAsync(&nDefer, pa->dCounter + 2, 4, hipMemcpyDeviceToHost, s));
    PCHK(hipStreamSynchronize(s));
    if (nDefer) {   // pass 1b: reads of 129..256 bases on the 256-bit planes, pass 1's pools
        P.nPairs = nDefer; P.pairList = pa->dDefer; P.counter = pa->dCounter + 5; P.maxLen = 256; P.passId = 2;
        P.deferList = pa->dDefer2; P.deferCount = pa->dCounter + 6;
        usePool(pa->pass[0]);
        grid = pa->grid256;
        if ((uint32_t)grid > nDefer) grid = (int)nDefer;
        hipLaunchKernelGGL(paired_kernel<256>, dim3(grid), dim3(64), 0, s, P);
        PCHK(hipGetLastError());
        PCHK(hipMemcpyAsync(&nDefer, pa->dCounter + 6, 4, hipMemcpyDeviceToHost, s));
        PCHK(hipStreamSynchronize(s));
    }
    if (nDefer) {   // pass 2: reads of 257..512 bases, IUPAC cases and pool overflows, ordinary pools, full grid
        // (pass 1b has consumed list 1: it is pass 2's output)
        P.nPairs = nDefer; P.pairList = pa->dDefer2; P.counter = pa->dCounter + 3; P.maxLen = 512; P.passId = 3;
        P.deferList = pa->dDefer; P.deferCount = pa->dCounter + 4;
        usePool(pa->pass[2]);
        grid = pa->pass[2].grid;
        if ((uint32_t)grid > nDefer) grid = (int)nDefer;
        hipLaunchKernelGGL(paired_kernel<512>, dim3(grid), dim3(64), 0, s, P);
        PCHK(hipGetLastError());
        PCHK(hipMemcpyAsync(&nDefer, pa->dCounter + 4, 4, hipMemcpyDeviceToHost, s));
        PCHK(hipStreamSynchronize(s));
    }
    if (nDefer) {   // pass 3: pool overflows, the reference's pool sizes on a small grid
        P.nPairs = nDefer; P.pairList = pa->dDefer; P.counter = pa->dCounter + 1; P.maxLen = 512; P.passId = 4;
        P.deferList = nullptr; P.deferCount = nullptr;
        usePool(pa->pass[1]);
        grid = pa->pass[1].grid;
        if ((uint32_t)grid > nDefer) grid = (int)nDefer;
        hipLaunchKernelGGL(paired_kernel<512>, dim3(grid), dim3(64), 0, s, P);
        PCHK(hipGetLastError());
    }
    PCHK(hipMemcpyAsync(out, pa->dOut, n * sizeof(snapgpu_pair_result_t), hipMemcpyDeviceToHost, s));
    PCHK(hipStreamSynchronize(s));
    uint64_t unwritten = 0, first = 0;
    for (uint64_t i = 0; i < n; i++)
        if (out[i].status[0] > SNAPGPU_UNKNOWN && !unwritten++) first = i;
    if (unwritten) {
        snapgpu::setError("paired: " + std::to_string(unwritten) + " pair record(s) written by no pass (first: pair " +
                          std::to_string(first) + "); results are not valid");
        return SNAPGPU_EDEVICE;
    }
    // MAPQ threshold cases re-derived with glibc log10 (as snapgpu_results_download does)
    for (uint64_t i = 0; i < n; i++) {
        snapgpu_pair_result_t &r = out[i];
        if (!(r.flags & SNAPGPU_PFLAG_MAPQ_FIXED)) continue;
        for (int k = 0; k < 2; k++) {
            r.mapq[k] = snapgpu_compute_mapq(r.probabilityOfAllPairs, r.probabilityOfBestPair, r.score[k],
                                             (int)r.popularSeedsSkipped);
            r.status[k] = r.mapq[k] > 10 ? SNAPGPU_SINGLE_HIT : SNAPGPU_MULTIPLE_HITS;
        }
    }
    for (uint64_t i = 0; i < n; i++)
        if (out[i].flags & (SNAPGPU_PFLAG_POOL_EXHAUSTED | SNAPGPU_PFLAG_READ_TOO_LONG)) {
            snapgpu::setError(out[i].flags & SNAPGPU_PFLAG_READ_TOO_LONG
                                  ? "paired: read longer than maxReadSize (the reference exits, IntersectingPairedEndAligner.cpp:211-215)"
                                  : "paired: scoring candidate pool exhausted (the reference exits; raise maxCandidatePoolSize)");
            return SNAPGPU_EINVAL;
        }
    return SNAPGPU_OK;
}

extern "C" {

void snapgpu_paired_params_default(snapgpu_paired_params_t *p) {
    if (!p) return;
    memset(p, 0, sizeof(*p));
    p->maxHits = 16000;                // AlignerOptions.cpp:73-77 (forPairedEnd)
    p->maxK = 15;
    p->maxSeedsToUse = 8;
    p->extraSearchDepth = 2;
    p->minSpacing = 50;                // PairedAligner.cpp:57-58
    p->maxSpacing = 1000;
    p->maxBigHits = 16000;             // DEFAULT_INTERSECTING_ALIGNER_MAX_HITS
    p->maxCandidatePoolSize = 1000000; // DEFAULT_MAX_CANDIDATE_POOL_SIZE
    p->maxReadSize = 500;              // MAX_READ_LENGTH
    p->forceSpacing = 0;
    p->seedCoverage = 0;
}

snapgpu_paired_aligner_t *snapgpu_paired_aligner_create(int device, const snapgpu_index_t *idx,
                                                        const snapgpu_paired_params_t *params) {
    if (!idx) { snapgpu::setError("paired_aligner_create: null index"); return nullptr; }
    snapgpu_paired_params_t p;
    if (params) p = *params; else snapgpu_paired_params_default(&p);
    if (p.maxK + p.extraSearchDepth + 1 > (uint32_t)MAX_LISTS || p.maxK > (uint32_t)MAX_K - 1) {
        snapgpu::setError("paired_aligner_create: maxK + extraSearchDepth too large");
        return nullptr;
    }
    if (p.maxReadSize > 512) { snapgpu::setError("paired_aligner_create: maxReadSize > 512"); return nullptr; }
    snapgpu_aligner_params_t bp;
    snapgpu_aligner_params_default(&bp);
    bp.maxHitsToConsider = p.maxHits; bp.maxK = p.maxK; bp.maxReadSize = p.maxReadSize;
    bp.maxSeedsToUse = p.maxSeedsToUse; bp.maxSeedCoverage = p.seedCoverage; bp.extraSearchDepth = p.extraSearchDepth;
    snapgpu_aligner_t *single = snapgpu_aligner_create(device, idx, &bp);   // fails loudly without a GPU
    if (!single) return nullptr;
    auto *pa = new snapgpu_paired_aligner_t();
    pa->device = device;
    pa->p = p;
    pa->single = single;
    auto fail = [&](const char *what, hipError_t e) -> snapgpu_paired_aligner_t * {
        snapgpu::setError(std::string("paired_aligner_create: ") + what + ": " + hipGetErrorString(e));
        snapgpu_paired_aligner_free(pa);
        return nullptr;
    };
    if (snapgpu_internal_index_args(single, &pa->X, nullptr)) { snapgpu_paired_aligner_free(pa); return nullptr; }
    hipError_t e;
    if ((e = hipSetDevice(device)) != hipSuccess) return fail("device", e);
    if ((e = ensurePairedTables(device)) != hipSuccess) return fail("tables", e);
    if ((e = hipStreamCreateWithFlags(&pa->stream, hipStreamNonBlocking)) != hipSuccess) return fail("stream", e);
    if ((e = hipMalloc(&pa->dCounter, 64)) != hipSuccess) return fail("counter", e);
    // IntersectingPairedEndAligner ctor (:47-57, :128): numSeedsFromCommandLine = min(30, -n)
    pa->maxSeedsCmd = p.maxSeedsToUse < 30 ? p.maxSeedsToUse : 30;
    const uint32_t maxSeedsToUse = pa->maxSeedsCmd ? pa->maxSeedsCmd
                                                   : (uint32_t)(p.maxReadSize * p.seedCoverage / idx->seedLen);
    const uint64_t pool = (uint64_t)p.maxBigHits * maxSeedsToUse * 2;
    pa->refPool = (uint32_t)std::min<uint64_t>(pool, p.maxCandidatePoolSize);
    hipDeviceProp_t prop;
    if ((e = hipGetDeviceProperties(&prop, device)) != hipSuccess) return fail("props", e);
    int perCU = 0;
    hipOccupancyMaxActiveBlocksPerMultiprocessor(&perCU, (const void *)paired_kernel<128>, 64, 0);
    if (perCU <= 0) perCU = 4;
    uint32_t c1 = std::min<uint32_t>(pa->refPool, 4096);
    if (const char *t = getenv("SNAPGPU_PAIRED_POOL1"); t && atoi(t) > 1) c1 = std::min<uint32_t>(pa->refPool, (uint32_t)atoi(t));
    if (allocPass(pa->pass[0], prop.multiProcessorCount * perCU, c1, std::max<uint32_t>(1, std::min(pa->refPool / 2, c1 / 2)), c1))
        { snapgpu_paired_aligner_free(pa); return nullptr; }
    int perCU256 = 0;
    hipOccupancyMaxActiveBlocksPerMultiprocessor(&perCU256, (const void *)paired_kernel<256>, 64, 0);
    if (perCU256 <= 0) perCU256 = 2;
    pa->grid256 = std::min(prop.multiProcessorCount * perCU256, pa->pass[0].grid);
    int perCU2 = 0;
    hipOccupancyMaxActiveBlocksPerMultiprocessor(&perCU2, (const void *)paired_kernel<512>, 64, 0);
    if (perCU2 <= 0) perCU2 = 2;
    // pass 2 pools hold the reference's whole pool; as many waves as fit in 8 GB
    const uint64_t stride2 = (uint64_t)pa->refPool * sizeof(Cand) + (uint64_t)pa->refPool * sizeof(Mate) +
                             (uint64_t)pa->refPool * sizeof(Anchor) + 256;
    int grid2 = prop.multiProcessorCount * perCU2;
    while (grid2 > 8 && (uint64_t)grid2 * stride2 > (8ull << 30)) grid2 /= 2;
    if (allocPass(pa->pass[1], grid2, pa->refPool, std::max<uint32_t>(1, pa->refPool / 2), pa->refPool))
        { snapgpu_paired_aligner_free(pa); return nullptr; }
    // pass 2 (reads of 129..512 bases): pass 1's pool sizes on the full <512> grid
    if (allocPass(pa->pass[2], prop.multiProcessorCount * perCU2, c1, std::max<uint32_t>(1, std::min(pa->refPool / 2, c1 / 2)), c1))
        { snapgpu_paired_aligner_free(pa); return nullptr; }
    // test hook: at most this many waves per pass, so each wave aligns many pairs in a row (a pair's
    // result must not depend on the pairs its wave aligned before: tests/test_paired.py)
    if (const char *t = getenv("SNAPGPU_ORDER_LONG")) pa->orderLong = atoi(t) != 0;
    if (const char *t = getenv("SNAPGPU_PAIRED_GRID"); t && atoi(t) > 0) {
        const int g = atoi(t);
        for (auto &pp : pa->pass) pp.grid = std::min(pp.grid, g);
        pa->grid256 = std::min(pa->grid256, g);
    }
    return pa;
}

void snapgpu_paired_aligner_free(snapgpu_paired_aligner_t *pa) {
    if (!pa) return;
    if (pa->single && snapgpu_internal_aligner_failed(pa->single)) {
        // a timed-out kernel may still run on these buffers: leak them (see aligner.hip)
    } else {
        (void)hipSetDevice(pa->device);
        if (pa->stream) (void)hipStreamSynchronize(pa->stream);
        pfree(pa->dCounter); pfree(pa->dDefer); pfree(pa->dDefer2); pfree(pa->dOrder); pfree(pa->dOrderW); pfree(pa->dOut);
        for (int r = 0; r < 2; r++) { pfree(pa->dB[r]); pfree(pa->dQ[r]); pfree(pa->dO[r]); pfree(pa->dL[r]); }
        for (auto &pp : pa->pass) pfree(pp.pool);
        if (pa->stream) (void)hipStreamDestroy(pa->stream);
    }
    if (pa->single) snapgpu_aligner_free(pa->single);
    delete pa;
}

snapgpu_aligner_t *snapgpu_paired_aligner_single(snapgpu_paired_aligner_t *pa) { return pa ? pa->single : nullptr; }

int snapgpu_paired_intersect_batch(snapgpu_paired_aligner_t *pa, const snapgpu_reads_t *reads0,
                                   const snapgpu_reads_t *reads1, snapgpu_pair_result_t *out) {
    if (!pa || !reads0 || !reads1 || !out) return SNAPGPU_EINVAL;
    if (reads0->n != reads1->n) { snapgpu::setError("paired: the two read batches differ in length"); return SNAPGPU_EINVAL; }
    if (reads0->n == 0) return SNAPGPU_OK;
    if (reads0->n > 0xffffffffull) { snapgpu::setError("paired: batch too large"); return SNAPGPU_EINVAL; }
    PCHK(hipSetDevice(pa->device));
    return runIntersect(pa, reads0, reads1, out);
}

// ChimericPairedEndAligner::align (ChimericPairedEndAligner.cpp:56-126) for every pair: the
// intersecting aligner on the GPU, then the pairs it left NotFound through the single-end GPU
// BaseAligner, each end on its own, MAPQ / 4.
int snapgpu_paired_align_batch(snapgpu_paired_aligner_t *pa, const snapgpu_reads_t *reads0,
                               const snapgpu_reads_t *reads1, snapgpu_pair_result_t *out) {
    int rc = snapgpu_paired_intersect_batch(pa, reads0, reads1, out);
    if (rc) return rc;
    const uint64_t n = reads0->n;
    std::vector<uint64_t> fb;   // pairs for the single-end fallback
    for (uint64_t i = 0; i < n; i++) {
        snapgpu_pair_result_t &r = out[i];
        const uint32_t n0 = reads0->lengths[i], n1 = reads1->lengths[i];
        if (n0 < 50 && n1 < 50) {   // :61-64: status NotFound, nothing else written
            const uint16_t f = r.flags;
            memset(&r, 0, sizeof(r));
            r.location[0] = r.location[1] = 0xffffffffu;
            r.score[0] = r.score[1] = -1;
            r.flags = f;
            continue;
        }
        r.fromAlignTogether = 1;
        r.alignedAsPair = 1;
        if (pa->p.forceSpacing) {
            if (r.status[0] == SNAPGPU_NOT_FOUND) r.fromAlignTogether = 0;
            continue;
        }
        if (r.status[0] != SNAPGPU_NOT_FOUND && r.status[1] != SNAPGPU_NOT_FOUND) continue;
        fb.push_back(i);
    }
    if (fb.empty()) return SNAPGPU_OK;
    const snapgpu_reads_t *R[2] = {reads0, reads1};
    // both ends' batches go into the aligner's stream before one wait: they run on its two lanes,
    // the second end's persistent kernel filling the first one's tail (two blocking calls paid
    // both tails: 33 -> ? ms of fallback per 100k 2x150 RNA pairs)
    std::vector<uint64_t> o[2];
    std::vector<uint32_t> l[2];
    std::vector<snapgpu_result_t> res[2];
    snapgpu_reads_t *sub[2] = {nullptr, nullptr};
    rc = snapgpu_align_batch_wait(pa->single);   // a stream the caller left open
    for (int e = 0; e < 2 && rc == SNAPGPU_OK; e++) {
        o[e].resize(fb.size());
        l[e].resize(fb.size());
        res[e].resize(fb.size());
        for (size_t j = 0; j < fb.size(); j++) { o[e][j] = R[e]->offsets[fb[j]]; l[e][j] = R[e]->lengths[fb[j]]; }
        sub[e] = snapgpu::readsView(R[e], fb.size(), o[e].data(), l[e].data());   // the fallback ends, no copy
        if (!sub[e]) { rc = SNAPGPU_ENOMEM; break; }
        rc = snapgpu_align_batch_submit(pa->single, sub[e], res[e].data());
    }
    const int wrc = snapgpu_align_batch_wait(pa->single);   // always closes what was submitted
    if (rc == SNAPGPU_OK) rc = wrc;
    for (auto *x : sub) snapgpu_reads_free(x);
    if (rc) return rc;
    for (int e = 0; e < 2; e++) {
        for (size_t j = 0; j < fb.size(); j++) {
            snapgpu_pair_result_t &r = out[fb[j]];
            const snapgpu_result_t &s = res[e][j];
            if (s.flags & SNAPGPU_FLAG_READ_TOO_LONG) {
                snapgpu::setError("paired: read longer than maxReadSize (the reference exits, BaseAligner.cpp:609-613)");
                return SNAPGPU_EINVAL;
            }
            r.status[e] = s.result;
            r.location[e] = s.location;
            r.direction[e] = s.direction;
            r.score[e] = s.score;
            r.mapq[e] = s.mapq / 4;   // :118
            r.nSingleScored += s.nLocationsScored;
        }
    }
    for (uint64_t i : fb) { out[i].fromAlignTogether = 0; out[i].alignedAsPair = 0; }
    return SNAPGPU_OK;
}

}  // extern "C"
