// aligner.hip -- gfx950 kernels for batched BaseAligner::AlignRead and the C-ABI
// aligner of include/snapgpu.h.  See align_device.h for the device data layout.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cmath>
#include <cstring>
#include <algorithm>
#include <atomic>
#include <mutex>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

#include "align_device.h"
#include "align_score.h"
#include "seed_lookup.h"
#include "cigar.h"
#include "internal.h"

using namespace sgk;

int snapgpu_internal_index_args(const snapgpu_aligner_t *a, sgk::KArgs *A, int *device);   // below

namespace sgk {

// ------------------------------------------------------------------ score()
// BaseAligner::score, BaseAligner.cpp:977-1399.  Returns true iff a final
// result was produced (written into st / *result).
template <int MAXLEN, bool EXT>
__device__ __forceinline__ bool score_wave(const KArgs &A, Lds<MAXLEN> &S, Elem512 *ar, ReadState &st, bool force,
                                           uint32_t n, const uint32_t (&rbF)[MAXLEN / 64],
                                           const uint32_t (&rbR)[MAXLEN / 64], int *result, uint32_t *flags) {
    constexpr int NB = MAXLEN / 64;
    const int lane = lane_id();
    const DevTables *tab = A.tab;
    for (int d = 0; d < 2; d++)
        if (st.mostSeeds[d]) {
            uint32_t v = uni(st.nSeedsApplied[d] / st.mostSeeds[d]);
            if (v > st.lps[d]) st.lps[d] = v;
        }
    do {
        if (overdue(A, st, 4)) return true;
        // head of the highest non-empty weight list == max sortkey over linked elements
        uint64_t sel = uni64(max_reduce64(S.laneMax[lane]));
        uint32_t minLps = st.lps[0] < st.lps[1] ? st.lps[0] : st.lps[1];
        if (minLps > st.scoreLimit || force) {
            if (sel == 0) {
                st.outScore = (int32_t)st.bestScore;
                if (st.bestScore <= A.maxK) {
                    st.outLoc = st.bestLoc;
                    const int mq = mapq_dev(A.tab, st.pAll, st.pBest, st.bestScore, sv_get(st, SV_POPULAR), flags);
                    st.outMapq = mq;
                    *result = mq >= 10 ? SNAPGPU_SINGLE_HIT : SNAPGPU_MULTIPLE_HITS;
                } else {
                    *result = (st.nSeedsApplied[0] == 0 && st.nSeedsApplied[1] == 0) ? SNAPGPU_MULTIPLE_HITS
                                                                                      : SNAPGPU_NOT_FOUND;
                    st.outMapq = 0;
                }
                return true;
            }
            force = true;
        } else if (sel == 0) {
            return false;
        }
        const uint32_t e = (uint32_t)sel;
        // One round trip for the whole element: lane i holds dword i (Elem layout,
        // align_device.h); fields are read into SGPRs with v_readlane.
        const uint32_t *ew = (const uint32_t *)(ar + e);
        const uint32_t ev = lane < ELEM_DWORDS ? ew[lane] : 0u;
        const uint64_t used = rl64(ev, 0);
        uint64_t scored = rl64(ev, 2);
        double eprob = rld(ev, 4);
        const uint32_t ekey = rl(ev, 6);
        uint32_t ebest = rl(ev, 8);
        uint32_t ebestLoc = rl(ev, 9);
        const uint32_t ewl = rl(ev, 11);
        const uint32_t dir = ekey & 1;
        const uint32_t ebase = (ekey >> 1) * ELEM;
        // unlink now (allExtantCandidatesScored = true, BaseAligner.cpp:1391-1394): no
        // insertion happens while an element is scored, so the next selection is known
        sk_set(A, S, ar, e, 0);
        wave_sync();
        recompute_lane_max(A, S, ar, (int)(e % WAVE));
        wave_sync();
        if (((ewl >> 8) & 0xff) <= st.scoreLimit) {
            uint64_t mask = used;
            while (mask) {
                const int bit = __builtin_ctzll(mask);
                const uint64_t cb = 1ull << bit;
                mask &= ~cb;
                if (scored & cb) continue;
                bool anyNearby = scored != 0;
                scored |= cb;
                uint32_t loc = ebase + bit;
                const uint32_t elemLoc = loc;
                uint32_t sc = FAIL_SCORE;
                double prob = 0;
                uint32_t glen = n + MAX_K;
                bool ok = substring_ok(A, loc, glen);
                if (!ok) {   // BaseAligner.cpp:1163-1185
                    uint32_t endOffset = 0;
                    bool have = false;
                    if ((uint64_t)loc + n + MAX_K >= A.nBases) { endOffset = A.nBases; have = true; }
                    else {
                        int np = next_piece_after(A, loc);
                        if (np >= 0) { endOffset = A.pieces[np]; have = true; }
                    }
                    if (have) {
                        glen = endOffset - loc - 1;
                        if (glen >= n - (uint32_t)MAX_K) ok = substring_ok(A, loc, glen);
                    }
                }
                if (ok) {
                    const int s = (int)((rl(ev, 12 + bit / 2) >> (16 * (bit & 1))) & 0xffff);
                    const int t = s + (int)A.seedLen;
                    int w0 = stage_window(S, A.genome, loc, (int)n);
                    int kmax = st.scoreLimit < (uint32_t)(MAX_K - 1) ? (int)st.scoreLimit : MAX_K - 1;
                    Bitmap<NB> F;
                    build_bitmap<NB>(F, rbF, rbR, dir != 0, (const char *)S.win, w0, (int)n, kmax);
                    const char *q = dir ? S.rcQ : S.fwdQ;
                    LvOut r1 = lv_wave<1, NB>(F, t, (int)n - t, (int)glen - t, (int)st.scoreLimit, q, S.rows,
                                              S.btAct, S.btMatched, tab);
                    if (r1.score != -1) {
                        int limitLeft = (int)st.scoreLimit - r1.score;
                        LvOut r2 = lv_wave<-1, NB>(F, s - 1, s, s + MAX_K, limitLeft, q, S.rows, S.btAct,
                                                   S.btMatched, tab);
                        if (r2.score != -1) {
                            sc = (uint32_t)(r1.score + r2.score);
                            prob = r1.prob * r2.prob * tab->seedProb;
                            loc += (uint32_t)r2.netIndel;
                        }
                    }
                }
                if (sc != FAIL_SCORE) record_hit<EXT>(A, loc, dir, sc);
                sv_add(st, lane, SV_SCORED, 1);
                if (anyNearby) {
                    if (ebest < sc || (ebest == sc && prob <= eprob)) continue;
                }
                ebestLoc = loc;
                uint32_t nb = NONE;
                if (sc != FAIL_SCORE) {
                    uint32_t nl = elemLoc + (2 * (elemLoc % ELEM / (ELEM / 2)) - 1) * (ELEM / 2);
                    uint32_t nkey = ((nl / ELEM) << 1) | dir;
                    nb = uni(chain_find(A, S, ar, nkey, (uint32_t)A.arenaElems));
                }
                if (nb != NONE) {
                    const uint32_t *nw = (const uint32_t *)(ar + nb);
                    const uint32_t nv = lane < 12 ? nw[lane] : 0u;
                    if (rl64(nv, 2) == 0) nb = NONE;   // nearby element not scored yet
                    if (nb != NONE) {
                        uint32_t nbase = (rl(nv, 6) >> 1) * ELEM;
                        uint32_t nbl = rl(nv, 9);
                        if (!((nbase > ebase && loc - nbl <= (uint32_t)ELEM) || (nbase < ebase && nbl <= (uint32_t)ELEM)))
                            nb = NONE;   // sic: BaseAligner.cpp:1311-1312
                    }
                    if (nb != NONE) {
                        uint32_t nbs = rl(nv, 8);
                        double np = rld(nv, 4);
                        if (nbs < sc || (nbs == sc && np >= prob)) continue;
                        anyNearby = true;
                        st.pAll = st.pAll - np > 0.0 ? st.pAll - np : 0.0;
                        if (lane == 4 || lane == 5) ((uint32_t *)(ar + nb))[lane] = 0u;   // nearby prob = 0
                    }
                }
                st.pAll = st.pAll - eprob > 0.0 ? st.pAll - eprob : 0.0;
                st.pAll += prob;
                eprob = prob;
                ebest = sc;
                if (st.bestScore > sc || (st.bestScore == sc && prob > st.pBest)) {
                    st.bestScore = sc;
                    st.pBest = prob;
                    st.bestLoc = loc;
                    st.outLoc = loc;
                    st.outScore = (int32_t)sc;
                    st.outDir = dir;
                }
                if (A.stopOnFirst && st.bestScore <= A.maxK) {
                    *result = SNAPGPU_MULTIPLE_HITS;
                    st.outMapq = 0;
                    return true;
                }
                st.scoreLimit = (st.bestScore < A.maxK ? st.bestScore : A.maxK) + A.extra;
            }
        }
        // write back the element in one store: scored, prob, bestScore, bestLoc, allScored
        {
            const uint64_t pb = (uint64_t)__double_as_longlong(eprob);
            uint32_t w = ev;
            bool st_ = true;
            if (lane == 2) w = (uint32_t)scored;
            else if (lane == 3) w = (uint32_t)(scored >> 32);
            else if (lane == 4) w = (uint32_t)pb;
            else if (lane == 5) w = (uint32_t)(pb >> 32);
            else if (lane == 8) w = ebest;
            else if (lane == 9) w = ebestLoc;
            else if (lane == 11) w = (ewl & ~0x00ff0000u) | (1u << 16);
            else st_ = false;
            if (st_) ((uint32_t *)(ar + e))[lane] = w;
        }
        wave_sync();
    } while (force);
    return false;
}

// ------------------------------------------------------------ hit insertion
// The per-hit loop of BaseAligner.cpp:829-869 (findCandidate / incrementWeight /
// allocateNewCandidate) for one seed, both directions in one pass: the forward hits
// [0, lim0) then the reverse-complement hits [lim0, lim0 + lim1), the order and
// timestamps of applying the directions one after the other (their elements never
// coincide: the direction is part of the element key).
template <int MAXLEN, bool EXT>
__device__ __forceinline__ void insert_hits(const KArgs &A, Lds<MAXLEN> &S, ElemOf<MAXLEN> *ar, ReadState &st,
                                            uint32_t lim0, uint32_t lim1, uint32_t off0, uint32_t off1,
                                            const uint32_t *list0, const uint32_t *list1, uint32_t single0,
                                            uint32_t single1, uint32_t numWeightLists, uint32_t minLoc,
                                            uint32_t maxLoc) {
    constexpr bool C64 = std::is_same<ElemOf<MAXLEN>, Elem64>::value;
    const int lane = lane_id();
    const uint32_t lim = lim0 + lim1;
    for (uint32_t b0 = 0; b0 < lim; b0 += WAVE) {
        if (overdue(A, st, 5)) break;
        const uint32_t i = b0 + lane;
        const uint32_t dir = i >= lim0 ? 1u : 0u;
        const uint32_t ii = dir ? i - lim0 : i;
        const uint32_t *list = dir ? list1 : list0;
        const uint32_t offset = dir ? off1 : off0;
        const uint32_t lpsNow = dir ? st.lps[1] : st.lps[0];
        const bool allowAlloc = lpsNow <= st.scoreLimit;
        bool valid = i < lim;
        uint32_t h = valid ? (list ? list[ii] : (dir ? single1 : single0)) : 0;
        uint32_t loc = h - offset;
        valid = valid && h >= offset;
        if constexpr (EXT) valid = valid && loc >= minLoc && loc <= maxLoc;   // BaseAligner.cpp:849-853
        uint32_t key = ((loc / ELEM) << 1) | dir;
        S.u.ins.scrLoc[lane] = loc;
        uint32_t slot = 0;
        // Group the batch's hits by element.  A seed's hits come in descending location order (the
        // index keeps overflow lists sorted), so the hits of one element are neighbours among the valid
        // lanes: a lane leads its group when its key differs from the previous valid lane's, and the
        // group runs to the next leader.  A batch whose keys are not ordered that way (within each
        // direction) takes the LDS hash table instead.
        const uint64_t vm = ballot(valid);
        const uint64_t lowV = vm & ((1ull << lane) - 1);
        const bool hasPrev = lowV != 0;
        const uint32_t pkey = (uint32_t)shfl_idx((int)key, hasPrev ? 63 - (int)__builtin_clzll(lowV) : lane);
        const bool useTab = ballot(valid && hasPrev && ((pkey ^ key) & 1u) == 0 && key > pkey) != 0;
        uint64_t grp;
        bool leader;
        if (!useTab) {
            leader = valid && (!hasPrev || pkey != key);
            const uint64_t lm = ballot(leader);
            const uint64_t above = lm & ~((2ull << lane) - 1);              // leaders after this lane
            const uint64_t upto = above ? (above & (~above + 1)) - 1 : ~0ull;  // lanes before the next one
            grp = leader ? vm & upto & ~((1ull << lane) - 1) : 0ull;
            wave_sync();
        } else {
            if (valid) {
                uint32_t s = (key * 2654435761u) >> 25;
                for (int probe = 0;; probe++) {
                    uint32_t old = atomicCAS(&S.u.ins.btKey[s], NONE, key);
                    if (old == NONE || old == key) break;
                    if (probe >= BT) { diag_report(A.diag, DIAG_BATCH_TABLE, st.rid, key); valid = false; break; }
                    s = (s + 1) & (BT - 1);
                }
                slot = s;
            }
            wave_sync();
            if (valid) atomicOr((unsigned long long *)&S.u.ins.btMask[slot], 1ull << lane);
            wave_sync();
            grp = valid ? S.u.ins.btMask[slot] : 0;
            leader = valid && (__builtin_ctzll(grp) == lane);
            wave_sync();
        }
        bool overflow = false;   // element arena exhausted (cannot happen at (maxSeeds+2)*maxHits; guarded)
        if (leader) {
            if (useTab) {
                S.u.ins.btKey[slot] = NONE;
                S.u.ins.btMask[slot] = 0;
            }
            uint32_t e = chain_find(A, S, ar, key, (uint32_t)A.arenaElems);
            if (e != NONE || allowAlloc) {
                uint64_t used = 0;
                uint32_t weight = 0, allScored = 0, sortkey = 0;
                // header dword 11 = weight | lps << 8 | allScored << 16 (| Elem64 spill << 17); a new
                // element's header is written at the end in 16-byte stores instead of field by field
                uint32_t w11 = 0, chainNext = NONE;
                uint32_t sl4[4] = {0u, 0u, 0u, 0u};   // Elem64: the inline (bit + 1, offset) slots
                bool isNew = false;
                if (e != NONE) {
                    auto rd = [&](const uint32_t *eh) __attribute__((always_inline)) {
                        used = *reinterpret_cast<const uint64_t *>(eh);
                        w11 = eh[11];
                        if constexpr (C64) {
                            const uint4 q = *reinterpret_cast<const uint4 *>(eh + 12);
                            sl4[0] = q.x; sl4[1] = q.y; sl4[2] = q.z; sl4[3] = q.w;
                        }
                    };
                    if (C64 && e < ELCAP) rd(S.eloc[e]);   // (two call sites: LDS and global loads, not flat)
                    else rd(reinterpret_cast<const uint32_t *>(ar + e));
                    weight = w11 & 0xff; allScored = (w11 >> 16) & 1u; sortkey = sk_get(A, S, ar, e);
                }
                uint64_t m = grp;
                while (m) {
                    int j = __builtin_ctzll(m);
                    m &= m - 1;
                    uint32_t bit = S.u.ins.scrLoc[j] % ELEM;
                    uint32_t t = st.ts + b0 + j;
                    const uint64_t cb = 1ull << bit;
                    const bool had = (used & cb) != 0;
                    if (e == NONE) {
                        // allocateNewCandidate (BaseAligner.cpp:1485-1568): tail of weight list 1
                        if (atomicAdd(&S.nUsed, 1u) >= (uint32_t)A.arenaElems) {
                            if (!A.ovfList) diag_report(A.diag, DIAG_ARENA, st.rid, S.nElems);
                            overflow = true;
                            break;
                        }
                        e = atomicAdd(&S.nElems, 1u);
                        isNew = true;
                        w11 = (lpsNow & 0xffu) << 8;
                        const uint32_t old = head_exchange(S, elem_hash(key), e);
                        if (e < MIRCAP) { S.ekey[e] = key; S.enext[e] = (uint16_t)(old == NONE ? 0xffffu : old); }
                        chainNext = old;
                        used = cb;
                        weight = 1;
                        allScored = 0;
                        sortkey = (1u << 24) | (0xffffffu - t);
                    } else {
                        // findCandidate (BaseAligner.cpp:1474-1479) + incrementWeight (1689-1727)
                        allScored = (allScored && had) ? 1 : 0;
                        used |= cb;
                        if (!allScored && weight < numWeightLists - 1) {
                            weight++;
                            sortkey = (weight << 24) | (0xffffffu - t);
                        }
                    }
                    // candidate->seedOffset = offset (BaseAligner.cpp:858)
                    if constexpr (C64) {
                        const uint32_t sp = spill_index(w11);
                        if (sp) {
                            reinterpret_cast<uint8_t *>(ar + sp)[bit] = (uint8_t)offset;
                        } else {
                            // slots hold the used candidates in first-use order: candidate `bit` has
                            // one iff it was used before; a new one takes slot popcount(used before)
                            const uint32_t k = had ? slot_of(sl4, bit) : (uint32_t)__popcll(used & ~cb);
                            if (k < (uint32_t)NSLOT) {
                                slot_set(sl4, k, bit, offset);
                            } else {
                                // a ninth candidate: a spill block from the arena's top takes them all
                                if (atomicAdd(&S.nUsed, 1u) >= (uint32_t)A.arenaElems) {
                                    if (!A.ovfList) diag_report(A.diag, DIAG_ARENA, st.rid, S.nElems);
                                    overflow = true;
                                    break;
                                }
                                const uint32_t spn = (uint32_t)A.arenaElems - 1u - atomicAdd(&S.nSpill, 1u);
                                uint8_t *blk = reinterpret_cast<uint8_t *>(ar + spn);
#pragma unroll
                                for (int q = 0; q < NSLOT; q++) {
                                    const uint32_t pr = (sl4[q >> 1] >> (16 * (q & 1))) & 0xffffu;
                                    blk[(pr & 0xffu) - 1u] = (uint8_t)(pr >> 8);
                                }
                                blk[bit] = (uint8_t)offset;
                                w11 |= spn << W11_SPILL_SHIFT;
                            }
                        }
                    } else {
                        ar[e].seedOffset[bit] = (std::remove_reference_t<decltype(ar[e].seedOffset[0])>)offset;
                    }
                }
                if (overflow) e = NONE;
                if (e != NONE) {
                    w11 = (w11 & 0xfffeff00u) | (weight & 0xffu) | ((allScored & 1u) << 16);
                    auto wr = [&](uint32_t *eh) __attribute__((always_inline)) {
                        if (isNew) {
                            // {used, scored = 0}, {prob = 0, key, next}, {bestScore, bestLoc, sortkey, w11}
                            uint4 *h4 = reinterpret_cast<uint4 *>(eh);
                            h4[0] = make_uint4((uint32_t)used, (uint32_t)(used >> 32), 0u, 0u);
                            h4[1] = make_uint4(0u, 0u, key, chainNext);
                            h4[2] = make_uint4(UNUSED_SCORE, 0u, sortkey, w11);
                            if constexpr (C64) h4[3] = make_uint4(sl4[0], sl4[1], sl4[2], sl4[3]);
                        } else {
                            *reinterpret_cast<uint64_t *>(eh) = used;
                            eh[11] = w11;
                            if constexpr (C64)
                                if (!spill_index(w11)) *reinterpret_cast<uint4 *>(eh + 12) = make_uint4(sl4[0], sl4[1], sl4[2], sl4[3]);
                        }
                    };
                    if (C64 && e < ELCAP) wr(S.eloc[e]);
                    else wr(reinterpret_cast<uint32_t *>(ar + e));
                    sk_set(A, S, ar, e, sortkey);
                    if (sortkey) atomicMax((unsigned long long *)&S.laneMax[e % WAVE], ((uint64_t)sortkey << 32) | e);
                }
            }
        }
        // a capped arena hands the read to the big-arena pass (align_one); a worst-case one cannot
        // fill up, and if it did the watchdog record makes the host call fail
        if (ballot(overflow)) st.abort = A.ovfList ? 2u : 1u;
        wave_sync();
    }
    st.ts += lim;
}

// pass 1 -> pass 2 hand-off (KArgs::deferList)
__device__ __forceinline__ void defer_read(const KArgs &A, uint32_t r) {
    if (lane_id() == 0) A.deferList[atomicAdd(A.deferCount, 1u)] = r;
}

// ------------------------------------------------------------- AlignRead
// EXT: windowed search / multi-hit export compiled in (snapgpu_align_batch_ex)
template <int MAXLEN, bool EXT>
__device__ __forceinline__ void align_one(const KArgs &A, Lds<MAXLEN> &S, ElemOf<MAXLEN> *ar, uint32_t r) {
    constexpr int NB = MAXLEN / 64;
    const int lane = lane_id();
    PH_T(A, tsetup);
    const uint32_t n = A.lengths[r];
    const uint64_t off = A.offsets[r];
    const uint32_t seedLen = A.seedLen;
    ReadState st;
    st.outLoc = INVALID; st.outDir = 0; st.outScore = (int32_t)UNUSED_SCORE; st.outMapq = 0;
    st.pAll = 0; st.pBest = 0;
    st.statv = 0;
    st.ts = 0;
    st.rid = r;
    st.abort = 0;
    st.t0 = __builtin_amdgcn_s_memrealtime();
    st.tick = 32;
    st.nSeedsApplied[0] = st.nSeedsApplied[1] = 0;
    uint32_t flags = MAXLEN > 128 ? SNAPGPU_FLAG_DEFERRED : 0u;   // passes 2 and 3 align only deferred reads
    if constexpr (Lds<MAXLEN>::BYTE_PATH) flags |= SNAPGPU_FLAG_BYTE_PATH;
    int result = SNAPGPU_NOT_FOUND;
    // maxSeedsToUse from the seed coverage (BaseAligner.cpp:563-568) by a host table, no device
    // double division (its hoisted operand was align_kernel<256>'s one scratch spill); a read
    // longer than 512 bases is not aligned (READ_TOO_LONG)
    const uint32_t maxSeeds = A.maxSeedsCmd ? A.maxSeedsCmd : (n <= 512u ? A.tab->maxSeedsForLen[n] : 0u);
    const uint32_t numWeightLists = maxSeeds + 1;
    bool run = true;
    if constexpr (!Lds<MAXLEN>::BYTE_PATH) {   // bit-plane kernels: longer reads go on to the next pass
        if (n > (uint32_t)MAXLEN) {
            if (!(MAXLEN == 128 && A.longCount)) defer_read(A, r);   // (pass 0 has listed them already)
            return;
        }
    }
    // search window (BaseAligner.cpp:596-602); multiHitsFound = 0 up front (:586-590)
    uint32_t radius = 0, sDir = 0, minLoc = 0, maxLoc = INVALID;
    if (EXT && A.search) {
        radius = uni(A.search[r].searchRadius);
        if (radius) {
            const uint32_t sLoc = uni(A.search[r].searchLocation);
            sDir = uni(A.search[r].searchDirection);
            minLoc = sLoc > radius ? sLoc - radius : 0;
            maxLoc = sLoc < INVALID - radius ? sLoc + radius : INVALID;
        }
    }
    bool fillHits = false;
    if (EXT && A.maxHitsToGet && lane < MAX_K) A.hitScratch[(uint64_t)blockIdx.x * A.hitStride + lane] = 0;
    if (n > A.maxReadSize || n > (uint32_t)MAXLEN) { flags |= SNAPGPU_FLAG_READ_TOO_LONG; run = false; }
    else if (n < seedLen) run = false;
    uint32_t rbF[NB], rbR[NB];
    if (run) {
        // Read::init upper-casing + BaseAligner.cpp:636-650 (RC read, qualities)
        uint32_t nN = 0;
        bool other = false, nul = false;
        for (int i = lane; i < Lds<MAXLEN>::RL; i += WAVE) {
            uint32_t c = 0, q = 0;
            if (i < (int)n) {
                c = (uint8_t)A.bases[off + i];
                q = (uint8_t)A.quals[off + i];
                if (c >= 'a' && c <= 'z') c -= 0x20;
                if constexpr (Lds<MAXLEN>::BYTE_PATH) {
                    S.rc[n - 1 - i] = (char)complement_of(c);
                    S.rcQ[n - 1 - i] = (char)q;
                }
            } else if constexpr (Lds<MAXLEN>::BYTE_PATH) {
                S.rc[i] = 0;
                S.rcQ[i] = 0;
            }
            S.fwd[i] = (char)c;
            S.fwdQ[i] = (char)q;
            nN += __popcll(ballot(i < (int)n && c == 'N'));
            other |= ballot(i < (int)n && c != 'A' && c != 'C' && c != 'G' && c != 'T' && c != 'N') != 0;
            nul |= ballot(i < (int)n && c == 0) != 0;   // no reader produces 0x00: a corrupted upload
        }
        if (nul) flags |= SNAPGPU_FLAG_NUL_BYTE;
        if constexpr (!Lds<MAXLEN>::BYTE_PATH) {
            // bit planes compare bytes exactly unless both the read and the genome hold
            // non-ACGTN bytes (an IUPAC code could then match itself): byte path
            if (A.hasIupac && other) { defer_read(A, r); return; }
        }
        for (int i = lane; i < NBUCKET; i += WAVE) S.head[i] = Lds<MAXLEN>::HEAD_NONE;
        for (int i = lane; i < BT; i += WAVE) { S.u.ins.btKey[i] = NONE; S.u.ins.btMask[i] = 0; }
        S.laneMax[lane] = 0;
        if (lane == 0) { S.nElems = 0; S.nSpill = 0; S.nUsed = 0; }
        wave_sync();
        if constexpr (Lds<MAXLEN>::BYTE_PATH) {
#pragma unroll
            for (int b = 0; b < NB; b++) { rbF[b] = (uint8_t)S.fwd[b * 64 + lane]; rbR[b] = (uint8_t)S.rc[b * 64 + lane]; }
        } else {
            // read bit planes {hi, lo, notACGT} of both directions; zero slack past n is not ACGT.
            // read[RC][m] = complement of read[FORWARD][n-1-m] (BaseAligner.cpp:636-650): the 2-bit
            // code xor 3 (A<->T, C<->G); N and the other bytes stay not ACGT
#pragma unroll
            for (int dr = 0; dr < 2; dr++)
#pragma unroll
                for (int h = 0; h < NB; h++) {
                    const int m = h * 64 + lane;
                    uint32_t code;
                    if (dr == 0) code = packed_code((uint8_t)S.fwd[m]);
                    else {
                        code = m < (int)n ? packed_code((uint8_t)S.fwd[n - 1 - m]) : 4u;
                        if (code < 4) code ^= 3u;
                    }
                    const uint64_t bh = ballot(code < 4 && (code & 2)), bl = ballot(code < 4 && (code & 1));
                    const uint64_t bm = ballot(code > 3);
                    if (lane == 0) { S.grp[0].rpl[dr][0][h] = bh; S.grp[0].rpl[dr][1][h] = bl; S.grp[0].rpl[dr][2][h] = bm; }
                }
            wave_sync();
        }
        if (nN > A.maxK) { flags |= SNAPGPU_FLAG_TOO_MANY_NS; run = false; }
    }
    PH_ADD(A, S, PH_SETUP, tsetup);
    if (run) {
        st.lps[0] = st.lps[1] = 0;
        st.mostSeeds[0] = st.mostSeeds[1] = 1;
        st.bestScore = UNUSED_SCORE;
        st.bestLoc = 0;
        st.scoreLimit = A.maxK + A.extra;
        const uint32_t nPossible = n - seedLen + 1;
        uint64_t *seedUsed = S.seedUsed;
        if (lane <= NB) seedUsed[lane] = 0;
        wave_sync();
        uint32_t next = 0, wrapCount = 0;
        bool wrapForced = false;
        // BaseAligner.cpp:749-751
        const uint32_t minSeedLoc = minLoc < n ? 0 : minLoc - n;
        const uint32_t maxSeedLoc = maxLoc > INVALID - n ? INVALID : maxLoc + n;
        const bool windowed = EXT && (minSeedLoc != 0 || maxSeedLoc != INVALID);
        // first-round lookups resolved by seed_lookup_kernel: lane 4k+f holds field f of record k
        uint32_t srec = 0, pfIdx = SEEDS_PER_READ;
        if (MAXLEN <= 256 && A.seedRecs && A.maxHits < 0xffffu && radius == 0) {
            srec = ((const uint32_t *)(A.seedRecs + (uint64_t)r * SEEDS_PER_READ))[lane & (4 * SEEDS_PER_READ - 1)];
            pfIdx = 0;
        }
        // One call site for the scorer (it is large): `force` marks the final scoring
        // pass after the seed loop ends (BaseAligner.cpp:707-723, 879-891).
        const uint32_t seedGuard = (nPossible + 2) * (seedLen + 2) + maxSeeds;
        PH_T(A, tsl);
        for (uint32_t guard = 0;; guard++) {
            // lane id re-read per seed (volatile asm): lane-derived masks are recomputed here,
            // not hoisted out of the seed loop and kept live in spilled SGPRs
            const int lane = lane_id();
            bool force = st.nSeedsApplied[0] + st.nSeedsApplied[1] >= maxSeeds;
            if (guard > seedGuard) {   // each pass consumes a seed position or a wrap
                if (lane == 0) diag_report(A.diag, DIAG_SEED_LOOP, r, next);
                st.abort = 1;
            }
            if (overdue(A, st, 3)) break;
            if (!force && next >= nPossible) {
                wrapCount++;
                if (wrapCount >= seedLen) { force = true; wrapForced = true; }
                else {
                    next = A.tab->wrap[wrapCount];
                    st.mostSeeds[0] = st.mostSeeds[1] = wrapCount + 1;
                }
            }
            if (!force) {
                PH_T(A, tlk);
                while (next < nPossible && ((uni64(seedUsed[next >> 6]) >> (next & 63)) & 1)) next++;
                if (next >= nPossible) continue;
                {
                    uint64_t w = uni64(seedUsed[next >> 6]) | (1ull << (next & 63));
                    wave_sync();
                    seedUsed[next >> 6] = w;
                    wave_sync();
                }
                bool found = false, comp = false, pal = false, pre = false;
                uint32_t v1 = 0, v2 = 0, cntF = 0, cntR = 0;   // overflow-list lengths, value-forward / -reverse side
                if (pfIdx < (uint32_t)SEEDS_PER_READ) {
                    const uint32_t meta = readlaneu(srec, 4 * pfIdx);
                    pre = (meta >> 31) && (meta & 0xff) == next && ((meta >> 16) & 0x7fff) != 0x7fff;
                    if (pre) {
                        found = (meta >> 8) & 1; comp = (meta >> 9) & 1; pal = (meta >> 10) & 1;
                        sv_add(st, lane, SV_PROBES, (meta >> 16) & 0x7fff);
                        v1 = readlaneu(srec, 4 * pfIdx + 1);
                        v2 = readlaneu(srec, 4 * pfIdx + 2);
                        const uint32_t pcnt = readlaneu(srec, 4 * pfIdx + 3);   // u16 each, saturated (maxHits < 0xffff)
                        cntF = pcnt & 0xffff; cntR = pcnt >> 16;
                        pfIdx++;
                    }
                }
                if (!pre) {
                // Seed::DoesTextRepresentASeed + Seed::Seed (Seed.cpp:28-42, Seed.h:38-51)
                int v = lane < (int)seedLen ? base_value((uint8_t)S.fwd[next + lane]) : 0;
                if (ballot(lane < (int)seedLen && v > 3)) continue;
                uint64_t fpart = lane < (int)seedLen ? (uint64_t)v << ((seedLen - lane - 1) * 2) : 0;
                uint64_t rpart = lane < (int)seedLen ? (uint64_t)(v ^ 3) << (lane * 2) : 0;
                const uint64_t f = uni64(or_reduce64(fpart));
                const uint64_t rcv = uni64(or_reduce64(rpart));
                // GenomeIndex::lookupSeed + SNAPHashTable::Lookup
                comp = (int64_t)f > (int64_t)rcv;
                pal = f == rcv;
                const uint64_t canon = comp ? rcv : f;
                const uint32_t table = (uint32_t)(canon >> 32);
                const uint32_t key = (uint32_t)canon;
                uint32_t aux = 0, lines = 0;   // the bucket image (bucket_table.h): home line + the next
                found = bucket_lookup_wave(A, table, key, lane, v1, v2, aux, lines);
                sv_add(st, lane, SV_PROBES, lines);
                if (found) {   // the entry's overflow-list lengths (a saturated one re-read from the list)
                    const uint32_t c1 = aux & BK_CSAT, c2 = (aux >> 15) & BK_CSAT;
                    const uint32_t vf = comp ? v2 : v1, vr = comp ? v1 : v2;
                    if (vf >= A.nBases && vf != UNUSED_SIDE) cntF = uni(bucket_count(A, comp ? c2 : c1, vf));
                    if (vr >= A.nBases && vr != UNUSED_SIDE) cntR = uni(bucket_count(A, comp ? c1 : c2, vr));
                }
                }
                if (overdue(A, st, 6)) break;
                // fillInLookedUpResults (GenomeIndex.cpp:1013-1086), both directions
                uint32_t nH0 = 0, nH1 = 0, sg0 = 0, sg1 = 0;
                const uint32_t *ls0 = nullptr, *ls1 = nullptr;
                if (found) {
                    uint32_t vf = comp ? v2 : v1, vr = comp ? v1 : v2;
                    if (vf < A.nBases) { nH0 = 1; sg0 = vf; }
                    else if (vf != UNUSED_SIDE) {
                        uint32_t o = vf - A.nBases;
                        nH0 = cntF;
                        ls0 = A.overflow + o + 1;
                        sv_add(st, lane, SV_OVF, 1);
                    }
                    if (pal) { nH1 = nH0; sg1 = sg0; ls1 = ls0; }   // palindrome (GenomeIndex.cpp:1003-1006)
                    else if (vr < A.nBases) { nH1 = 1; sg1 = vr; }
                    else if (vr != UNUSED_SIDE) {
                        uint32_t o = vr - A.nBases;
                        nH1 = cntR;
                        ls1 = A.overflow + o + 1;
                        sv_add(st, lane, SV_OVF, 1);
                    }
                    if (windowed) {   // the hits within [minSeedLoc, maxSeedLoc] (GenomeIndex.cpp:1029-1078)
                        for (int sd = 0; sd < 2; sd++) {
                            uint32_t &nh = sd ? nH1 : nH0;
                            const uint32_t *&ls = sd ? ls1 : ls0;
                            const uint32_t sg = sd ? sg1 : sg0;
                            if (sd && pal) { nH1 = nH0; ls1 = ls0; break; }
                            if (!ls) { if (nh && (sg < minSeedLoc || sg > maxSeedLoc)) nh = 0; continue; }
                            const uint32_t lo = uni(count_above_desc(ls, nh, maxSeedLoc));
                            uint32_t end = minSeedLoc ? uni(count_above_desc(ls, nh, minSeedLoc - 1)) : nh;
                            if (end < lo) end = lo;
                            nh = end - lo;
                            ls += lo;
                        }
                    }
                }
                sv_add(st, lane, SV_LOOKUPS, 1);
                PH_ADD(A, S, PH_LOOKUP, tlk);
                bool applied = false;
                uint32_t lims[2] = {0, 0};
#pragma unroll
                for (uint32_t dir = 0; dir < 2; dir++) {
                    const uint32_t nh = dir ? nH1 : nH0;
                    if (EXT && radius && dir != sDir) continue;   // BaseAligner.cpp:781-786
                    if (nh > A.maxHits && !A.explore) {
                        sv_add(st, lane, SV_POPULAR, 1);   // popularSeedsSkipped == nHitsIgnored per read
                    } else {
                        lims[dir] = nh < A.maxHits ? nh : A.maxHits;
                        sv_add(st, lane, SV_HITWORDS, lims[dir]);
                        applied = true;
                    }
                }
                if (applied) {
                    PH_T(A, tins);
                    insert_hits<MAXLEN, EXT>(A, S, ar, st, lims[0], lims[1], next, n - seedLen - next, ls0, ls1, sg0,
                                             sg1, numWeightLists, minLoc, maxLoc);
                    PH_ADD(A, S, PH_INSERT, tins);
                }
#pragma unroll
                for (uint32_t dir = 0; dir < 2; dir++) {   // nSeedsApplied (after both directions' hits)
                    const uint32_t nh = dir ? nH1 : nH0;
                    if (EXT && radius && dir != sDir) continue;
                    if (!(nh > A.maxHits && !A.explore)) st.nSeedsApplied[dir]++;
                }
                next += seedLen;
                if (!applied) continue;
            }
            if (overdue(A, st, 7)) break;
            PH_T(A, tsc);
            bool fin;
            if constexpr (Lds<MAXLEN>::BYTE_PATH) fin = score_wave<MAXLEN, EXT>(A, S, ar, st, force, n, rbF, rbR, &result, &flags);
            else {
                fin = score_batched<EXT, MAXLEN>(A, S, ar, st, force, n, &result, &flags);
                if (!fin && !force) {   // the scorer's LV rows overlay the insertion table
                    for (int i = lane; i < BT; i += WAVE) { S.u.ins.btKey[i] = NONE; S.u.ins.btMask[i] = 0; }
                    wave_sync();
                }
            }
            PH_ADD(A, S, PH_SCORE, tsc);
            if (fin || force) { fillHits = !wrapForced; break; }
            if (overdue(A, st, 8)) break;
        }
        PH_ADD(A, S, PH_SEEDLOOP, tsl);
    }
    PH_T(A, tout);
    if (st.abort == 2u) {   // outgrew the capped arena: no record here, the big-arena pass aligns it afresh
        if (lane_id() == 0) A.ovfList[atomicAdd(A.ovfCount, 1u)] = r;
        wave_sync();
        PH_ADD(A, S, PH_OUT, tout);
        return;
    }
    const uint32_t svLookups = sv_get(st, SV_LOOKUPS), svScored = sv_get(st, SV_SCORED);
    const uint32_t svPopular = sv_get(st, SV_POPULAR), svProbes = sv_get(st, SV_PROBES);
    const uint32_t svHitWords = sv_get(st, SV_HITWORDS), svOvf = sv_get(st, SV_OVF);
    if (lane_id() == 0) {   // (re-read: the setup's lane id is not kept live across the seed loop)
        snapgpu_result_t o;
        o.location = st.outLoc;
        o.score = st.outScore;
        o.mapq = st.outMapq;
        o.result = (uint8_t)result;
        o.direction = (uint8_t)st.outDir;
        o.flags = (uint8_t)flags;
        o.reserved = 0;
        o.nLookups = svLookups;
        o.nLocationsScored = svScored;
        o.popularSeedsSkipped = (uint16_t)svPopular;
        o.nHitsIgnored = (uint16_t)svPopular;
        o.nProbes = svProbes;
        o.nHitWords = svHitWords;
        o.nOverflowLists = svOvf;
        o.nElements = run ? S.nElems : 0;
        o.reserved2 = 0;
        o.probabilityOfAllCandidates = st.pAll;
        o.probabilityOfBestCandidate = st.pBest;
        A.out[r] = o;
    }
    if constexpr (EXT) { if (A.maxHitsToGet) fill_hits(A, r, run && fillHits); }
    wave_sync();
    PH_ADD(A, S, PH_OUT, tout);
    PH_ADD(A, S, PH_READCYC, tsetup);
    if (run && S.nElems >= 64) { PH_ADD(A, S, PH_HEAVYCYC, tsetup); PH_CNT(A, S, PH_NHEAVY, 1); }
}

template <int MAXLEN, bool EXT>
// amdgpu_waves_per_eu: <128> at 5 waves/SIMD (<= 96 VGPRs: the forced-mode prefilter's peak costs
// ~10 VGPRs of spills around it, 2.5 % faster than 4 waves without them,
// profiles/r05/ab/prefilter_pairs_r05l.txt), <256> at 4, <512> at 3 (<= 168 VGPRs: a few cold
// spills are cheaper than dropping to 2 waves/SIMD).
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(MAXLEN <= 128 ? 5 : (MAXLEN <= 256 ? 4 : 3)))) void align_kernel(KArgs A) {
    __shared__ Lds<MAXLEN> S;
    ElemOf<MAXLEN> *ar = reinterpret_cast<ElemOf<MAXLEN> *>(A.arena) + (uint64_t)blockIdx.x * A.arenaElems;
    const int lane = lane_id();
    uint32_t total = A.readList ? uni(*A.readCount) : A.nReads;
    // pass 1 after pass 0's routing: nothing to do when every read is long
    if (!A.readList && A.longCount && uni(*A.longCount) == A.nReads) total = 0;
    // a read is listed at most once per pass, so a list as long as the batch holds every read: take
    // them in input order without the list load (pass 2 of an all-long batch)
    const uint32_t *list = A.readList && total != A.nReads ? A.readList : nullptr;
    for (;;) {
        uint32_t i = 0;
        if (lane == 0) i = atomicAdd(A.counter, 1u);
        i = uni((uint32_t)readlane((int)i, 0));
        if (i >= total) break;
        const uint32_t r = list ? uni(list[i]) : i;
        if (__hip_atomic_load(&A.diag[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;   // watchdog: drain
        if (r == A.tripRead && lane == 0) diag_report(A.diag, DIAG_TEST_TRIP, r, 0);   // test hook
        align_one<MAXLEN, EXT>(A, S, ar, r);
    }
}

// LV parity kernel: one wave per task; the task's "read" and virtual genome are
// prepared on the host (see snapgpu_lv_batch).
struct LvTask {
    uint64_t readOff;   // into reads / quals buffers
    uint64_t genOff;    // into genome buffer: position of virtual genome coordinate 0
    int32_t n, p0, patternLen, textLen, k, g, dir, pad;
};

__global__ __launch_bounds__(64) void lv_kernel(const LvTask *tasks, const char *reads, const char *quals,
                                                const char *gbuf, const DevTables *tab, int32_t *outScore,
                                                int32_t *outNet, double *outProb) {
    __shared__ Lds<512> S;
    const int lane = lane_id();
    const LvTask T = tasks[blockIdx.x];
    for (int i = lane; i < 512 + 64; i += WAVE) {
        S.fwd[i] = i < T.n ? reads[T.readOff + i] : 0;
        S.fwdQ[i] = i < T.n ? quals[T.readOff + i] : 0;
    }
    wave_sync();
    uint32_t rb[8];
#pragma unroll
    for (int b = 0; b < 8; b++) rb[b] = (uint8_t)S.fwd[b * 64 + lane];
    int w0 = stage_window(S, gbuf + T.genOff, (uint32_t)T.g, T.n);
    Bitmap<8> F;
    int kmax = T.k < MAX_K - 1 ? T.k : MAX_K - 1;
    if (kmax < 0) kmax = 0;
    build_bitmap<8>(F, rb, rb, false, (const char *)S.win, w0, T.n, kmax);
    LvOut r = T.dir > 0 ? lv_wave<1, 8>(F, T.p0, T.patternLen, T.textLen, T.k, S.fwdQ, S.rows, S.btAct, S.btMatched, tab)
                        : lv_wave<-1, 8>(F, T.p0, T.patternLen, T.textLen, T.k, S.fwdQ, S.rows, S.btAct, S.btMatched, tab);
    if (lane == 0) { outScore[blockIdx.x] = r.score; outNet[blockIdx.x] = r.netIndel; outProb[blockIdx.x] = r.prob; }
}

// Unit-test kernel of the production bit-plane LV (align_score.h): one task per wave, group 0
// of lv_group<DIR, GS> (GS chosen from k as score_batched does) on the mismatch mask a pass
// would build, then lv_prob_pair for the match probability.  The task's text and pattern are
// mapped onto a virtual read and genome window exactly as lv_pass sees them:
//   forward: read = pattern, genome[loc + y] = text[y]; pattern index i = read position i;
//   reverse: read[m] = pattern[pl-1-m], genome[loc + y] = text[tl - pl + y], and the reverse LV
//            runs on the bit-reversed mask with q0 = 127 - (pl - 1), as lv_pass calls it.
struct LvgTask {
    uint64_t pOff, tOff;   // pattern/quals offset, text offset
    int32_t pl, tl, k, dir;
};

template <int GS, int DIR, int NW>
__device__ __forceinline__ void lvg_run(Lds<64 * NW> &S, const LvgTask &T, const char *pats, const char *texts,
                                        int32_t *outScore, int32_t *outNet, double *outProb) {
    auto &G = S.grp[0];
    const int lane = lane_id();
    const int li = lane & (GS - 1), gi = lane / GS, c = GS / 2 - 1;
    const bool act = gi == 0;
    const int pl = T.pl, tl = T.tl;
    // F_x[m] = read[m] != genome[loc + x + m], x = li - c; mismatch past the read or the text
    MaskW<NW> F;
    uint32_t f[2 * NW];
#pragma unroll
    for (int j = 0; j < 2 * NW; j++) f[j] = 0xffffffffu;
    if (act) {
        const int x = li - c;
        for (int m = 0; m < 64 * NW; m++) {
            bool mm = true;
            if (m < pl) {
                const char r = DIR > 0 ? pats[T.pOff + m] : pats[T.pOff + pl - 1 - m];
                const int y = DIR > 0 ? x + m : tl - pl + x + m;
                if (y >= 0 && y < tl) {
                    const char g = texts[T.tOff + y];
                    const uint32_t rc = packed_code((uint8_t)r), gc = packed_code((uint8_t)g);
                    mm = rc > 3 || gc > 3 || rc != gc;
                }
            }
            if (!mm) f[m >> 5] &= ~(1u << (m & 31));
        }
    }
#pragma unroll
    for (int j = 0; j < NW; j++) F.w[j] = ((uint64_t)f[2 * j + 1] << 32) | f[2 * j];
    int e = -1;
    if (DIR > 0) lv_group<1, GS, NW>(G, lv_rows(S), F, act, 0, pl, tl, T.k, T.k, e);
    else lv_group<-1, GS, NW>(G, lv_rows(S), mk_reverse(F), act, 64 * NW - 1 - (pl - 1), pl, tl, T.k, T.k, e);
    e = readlane(e, 0);
    wave_sync();
    double p1 = 1.0, p2 = 1.0;
    int net2 = 0;
    if (e >= 0) {
        if (lane == 0) G.plen[DIR > 0 ? 1 : 0][0] = 0;   // only this direction's path
        wave_sync();
        // forward: patternLen = n - t0 = pl (t0 = 0); reverse: patternLen = s0 = pl (t0 = n)
        lv_prob_pair(nullptr, G, 0, 0, pl, DIR > 0 ? 0 : pl, DIR > 0 ? 0 : pl, S.fwdQ, 0u, p1, p2, net2);
    }
    if (lane == 0) {
        outScore[blockIdx.x] = e;
        outNet[blockIdx.x] = DIR > 0 ? 0 : net2;
        outProb[blockIdx.x] = e >= 0 ? (DIR > 0 ? p1 : p2) : 1.0;
    }
}

template <int NW>
__global__ __launch_bounds__(64) void lv_group_kernel(const LvgTask *tasks, const char *pats, const char *quals,
                                                      const char *texts, int32_t *outScore, int32_t *outNet,
                                                      double *outProb) {
    __shared__ Lds<64 * NW> S;
    const int lane = lane_id();
    const LvgTask T = tasks[blockIdx.x];
    // qualities in read coordinates (reverse: read[m] = pattern[pl-1-m])
    for (int m = lane; m < Lds<64 * NW>::RL; m += WAVE)
        S.fwdQ[m] = m < T.pl ? (T.dir > 0 ? quals[T.pOff + m] : quals[T.pOff + T.pl - 1 - m]) : 0;
    wave_sync();
    const int k = T.k < MAX_K - 1 ? T.k : MAX_K - 1;
    const int GS = k <= 3 ? 8 : (k <= 7 ? 16 : (k <= 15 ? 32 : 64));   // score_batched's choice
    if (T.dir > 0) {
        if (GS == 8) lvg_run<8, 1, NW>(S, T, pats, texts, outScore, outNet, outProb);
        else if (GS == 16) lvg_run<16, 1, NW>(S, T, pats, texts, outScore, outNet, outProb);
        else if (GS == 32) lvg_run<32, 1, NW>(S, T, pats, texts, outScore, outNet, outProb);
        else lvg_run<64, 1, NW>(S, T, pats, texts, outScore, outNet, outProb);
    } else {
        if (GS == 8) lvg_run<8, -1, NW>(S, T, pats, texts, outScore, outNet, outProb);
        else if (GS == 16) lvg_run<16, -1, NW>(S, T, pats, texts, outScore, outNet, outProb);
        else if (GS == 32) lvg_run<32, -1, NW>(S, T, pats, texts, outScore, outNet, outProb);
        else lvg_run<64, -1, NW>(S, T, pats, texts, outScore, outNet, outProb);
    }
}

}  // namespace sgk

// ======================================================================= host
namespace {

std::mutex g_errMu;

#define HIPCHK(x)                                                                       \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            snapgpu::setError(std::string(#x) + ": " + hipGetErrorString(e_));          \
            return SNAPGPU_EDEVICE;                                                     \
        }                                                                               \
    } while (0)
// inside a loop whose exit path cleans up (sets rc and leaves the enclosing loop)
#define HIPBRK(x)                                                                       \
    if (hipError_t e_ = (x); e_ != hipSuccess) {                                        \
        snapgpu::setError(std::string(#x) + ": " + hipGetErrorString(e_));              \
        rc = SNAPGPU_EDEVICE;                                                           \
        break;                                                                          \
    }
#define HIPCHKN(x)                                                                      \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            snapgpu::setError(std::string(#x) + ": " + hipGetErrorString(e_));          \
            return nullptr;                                                             \
        }                                                                               \
    } while (0)

// libgcc __powidf2 (see oracle / DESIGN.md): the reference's pow(double, int).
double powi_libgcc(double x, int m) {
    unsigned nn = m < 0 ? -(unsigned)m : (unsigned)m;
    double y = (nn % 2) ? x : 1;
    while (nn >>= 1) { x = x * x; if (nn % 2) y = y * x; }
    return m < 0 ? 1 / y : y;
}

const uint8_t kWrap[10][25] = {   // SeedSequencer.h:28-287
    {0, 8, 4, 12, 2, 6, 10, 14, 1, 3, 5, 7, 9, 11, 13, 15},
    {0, 8, 4, 12, 2, 6, 10, 14, 1, 3, 5, 7, 9, 11, 13, 15, 16},
    {0, 9, 4, 13, 2, 6, 11, 15, 1, 3, 5, 7, 8, 10, 12, 14, 16, 17},
    {0, 10, 4, 14, 2, 6, 8, 12, 16, 18, 1, 3, 5, 7, 9, 11, 13, 15, 17},
    {0, 10, 5, 15, 2, 7, 12, 17, 3, 9, 11, 13, 19, 1, 4, 6, 8, 14, 18, 16},
    {0, 11, 6, 16, 3, 9, 13, 17, 18, 2, 5, 8, 15, 20, 1, 4, 7, 10, 12, 14, 19},
    {0, 11, 6, 16, 3, 9, 14, 19, 2, 7, 12, 17, 20, 4, 1, 10, 13, 15, 18, 21, 5, 8},
    {0, 12, 6, 17, 3, 9, 20, 14, 1, 4, 7, 10, 15, 18, 21, 4, 2, 5, 11, 16, 19, 22, 8},
    {0, 12, 6, 18, 3, 15, 21, 9, 1, 13, 19, 7, 16, 4, 22, 10, 2, 14, 20, 5, 17, 8, 23, 11},
    {0, 13, 6, 19, 3, 16, 22, 9, 11, 1, 14, 7, 20, 4, 17, 23, 2, 15, 5, 21, 8, 24, 10, 18, 12},
};

// initializeLVProbabilitiesToPhredPlus33 (LandauVishkin.cpp:601-649), host glibc.
void fillTables(DevTables &t, uint32_t seedLen) {
    memset(&t, 0, sizeof(t));
    t.indel[0] = 1.0;
    t.indel[1] = 0.001;
    for (int i = 2; i < 64; i++) t.indel[i] = t.indel[i - 1] * 0.5;
    for (int i = 0; i < 33; i++) t.phred[i] = 0.001;
    for (int i = 33; i <= 93 + 33; i++) t.phred[i] = 1.0 - (1.0 - pow(10.0, -1.0 * (i - 33.0) / 10.0)) * (1.0 - 0.001);
    for (int i = 93 + 33 + 1; i < 256; i++) t.phred[i] = 0.001;
    t.perfect[0] = 1.0;
    for (int i = 1; i < 512; i++) t.perfect[i] = t.perfect[i - 1] * (1 - 0.001);
    t.seedProb = powi_libgcc(1 - 0.001, (int)seedLen);
    for (int q = 0; q < 72; q++) t.mapqT[q] = q < 70 ? pow(10.0, -q / 10.0) : 0.0;
    if (seedLen >= 16 && seedLen <= 25)
        for (int i = 0; i < 25; i++) t.wrap[i] = kWrap[seedLen - 16][i];
    // seed_lookup_kernel's walk (seed_lookup.h) on an all-ACGT read of each length: rounds 0,
    // seedLen, ... then the wrap table's starts, skipping used offsets (BaseAligner.cpp:686-746)
    memset(t.seedSeq, 0xff, sizeof(t.seedSeq));
    const int L = (int)seedLen;
    for (int n = L; n <= 128; n++) {
        const int nPossible = n - L + 1;
        bool used[128] = {};
        int p = 0, wrap = 0, idx = 0;
        for (int guard = 0; guard < 4 * 128 && idx < 16; guard++) {
            if (p >= nPossible) {
                if (++wrap >= L) break;
                p = (int)t.wrap[wrap];
            }
            while (p < nPossible && used[p]) p++;
            if (p >= nPossible) continue;
            used[p] = true;
            t.seedSeq[n][idx++] = (uint8_t)p;
            p += L;
        }
    }
}

// g_tab (align_device.h) on the current device, once per device per process
hipError_t ensureDeviceTables(int device) {
    static std::mutex mu;
    static bool done[64] = {};
    std::lock_guard<std::mutex> lk(mu);
    if (device < 0 || device >= 64) return hipErrorInvalidDevice;
    if (done[device]) return hipSuccess;
    DevTables t;
    fillTables(t, 20);   // the seedLen-dependent fields (seedProb, wrap) are read from KArgs::tab
    hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(g_tab), &t, sizeof(t), 0, hipMemcpyHostToDevice);
    if (e == hipSuccess) done[device] = true;
    return e;
}

uint32_t packedCode(char c) {   // 2-bit code of the packed genome (4 = not ACGT)
    return c == 'A' ? 0u : c == 'C' ? 1u : c == 'G' ? 2u : c == 'T' ? 3u : 4u;
}

int hostMapq(double pAll, double pBest, int score, int popular) {   // mapq.h:32-65
    if (pAll < pBest) pAll = pBest;
    if (pAll == pBest && popular == 0 && score < 5) return 70;
    double c = pBest / pAll;
    int base;
    if (c >= 1) base = 69;
    else { base = (int)(-10 * log10(1 - c)); if (base > 69) base = 69; }
    int pen = popular - 10;
    if (pen < 0) pen = 0;
    base -= pen / 2;
    return base < 0 ? 0 : base;
}

}  // namespace

// One execution lane = one HIP stream with everything a pass set needs to run beside the
// other lane: its own element arenas (persistent waves index them by blockIdx), work
// counters, lookup statistics and timing events.  Lane 0 serves the resident API
// (snapgpu_reads_upload / snapgpu_align_resident); snapgpu_align_batch alternates chunks
// over both lanes so one chunk's copies and host tail overlap the other chunk's kernels,
// and the second lane's kernel fills the first one's tail.
// One chunk's input/output staging of the pipelined snapgpu_align_batch.  Two per lane: the
// H2D of a lane's next chunk (on the aligner's copy stream) runs while the lane's current chunk
// is still in its kernels, so the lane's next kernel can start the moment the current one ends.
struct ChunkSlot {
    char *dBases = nullptr, *dQuals = nullptr;  // device inputs
    uint64_t *dOffsets = nullptr;
    uint32_t *dLengths = nullptr;
    uint64_t *hOffsets = nullptr;               // pinned staging
    uint32_t *hLengths = nullptr;
    snapgpu_result_t *hOut = nullptr;
    hipEvent_t h2d = nullptr;                   // inputs on the device (copy stream)
    hipEvent_t done = nullptr;                  // records back in host memory (lane stream)
    bool pending = false;
    uint64_t seq = 0, chunkBegin = 0, chunkN = 0, chunkEv = 0;
    snapgpu_result_t *chunkOut = nullptr;       // the caller's record array of the pending chunk
};

struct ExecLane {
    hipStream_t stream = nullptr;
    void *arena = nullptr;                     // main passes: arenaCap elements per wave
    void *bigArena = nullptr;                  // big-arena pass: arenaElems per wave (only when arenaCap < arenaElems)
    uint32_t *counter = nullptr;               // [0] pass-1 work, [1] pass-3 work, [2] pass-1 defers, [3] pass-2 work,
                                               // [4] pass-2 defers, [5] long reads (pass 0), [6] arena overflows,
                                               // [7] big-arena pass work
    unsigned long long *lookupStats = nullptr; // seed_lookup_kernel: [256][4] seeds, probes, overflow counts (per call)
    hipEvent_t done = nullptr;                 // scratch event: waitLane, cross-lane ordering
    // chunk buffers of the pipelined snapgpu_align_batch (grown on demand)
    uint64_t capReads = 0, capBytes = 0;
    uint32_t *dDefer = nullptr;
    snapgpu_result_t *dOut = nullptr;
    SeedRec *dSeeds = nullptr;
    ChunkSlot slot[2];
    uint32_t nextSlot = 0;
    unsigned long long *hLookupStats = nullptr; // pinned copy of lookupStats
};

// Timing events of one pass set (one chunk) and the pinned copy of its work counters.
struct EvSet {
    hipEvent_t e[4] = {};   // 3: before pass 0, 0: before pass 1, 1: after pass 1, 2: after pass 2
    uint32_t *hCounter = nullptr;
};

struct snapgpu_device_reads {
    snapgpu_aligner_t *owner = nullptr;
    char *dBases = nullptr, *dQuals = nullptr;
    uint64_t *dOffsets = nullptr;
    uint32_t *dLengths = nullptr;
    snapgpu_result_t *dOut = nullptr;
    uint32_t *dDefer = nullptr;   // pass 1 -> pass 2 read list
    SeedRec *dSeeds = nullptr;    // seed_lookup_kernel records, SEEDS_PER_READ per read
    int32_t *dCigEd = nullptr;    // cigar_kernel outputs (allocated by the first snapgpu_cigar_resident)
    uint32_t *dCigN = nullptr, *dCigOps = nullptr;
    uint64_t n = 0;
    uint32_t maxLen = 0;
    int device = 0;
};

struct snapgpu_aligner {
    int device = 0;
    const snapgpu_index_t *idx = nullptr;
    snapgpu_aligner_params_t p{};
    uint32_t *dOverflow = nullptr, *dPieces = nullptr;
    // the seed tables' bucket image (bucket_table.h), built on the device at creation
    uint4 *dBuckets = nullptr;
    uint64_t *dBucketBase = nullptr;
    uint32_t *dBucketCount = nullptr;
    snapgpu_bucket_info_t bucketInfo{};
    char *dGenomeAlloc = nullptr;
    GPlane *dGPlanes = nullptr;   // genome bit planes (KArgs::gpl)
    const char *dGenome = nullptr;
    DevTables *dTab = nullptr;
    ExecLane lane[2];
    std::vector<EvSet> evs;       // one per pass set of the current call (grown on demand)
    uint64_t nEvUsed = 0;
    // Pass sets of the two lanes run concurrently: the second lane's waves fill the tail of the
    // first one's persistent kernel (the last, heavy reads of a launch).  SNAPGPU_OVERLAP=0 runs
    // them one after the other (copies and host tails still overlap).  With overlap, launch
    // durations overlap too: snapgpu_timing_t also carries the union of the launch intervals.
    bool overlapKernels = true;
    // snapgpu_align_batch_submit: chunks of consecutive batches stream through the lanes until
    // snapgpu_align_batch_wait; timing and statistics cover that whole stream
    bool streamOpen = false;
    uint64_t nextLane = 0;
    uint64_t chunkSeq = 0;        // submission order of pipelined chunks (finished oldest first)
    hipStream_t copyStream = nullptr;   // H2D of the pipelined chunks
    // CIGAR (cigar_kernel) and seed-census (charseeds.hip) calls: their own stream and buffers, so a
    // host thread can run them while another thread's align call keeps the lanes busy (the RNA
    // paired path's sub-batch pipeline); a caller serialises them among themselves
    hipStream_t sideStream = nullptr;
    std::chrono::steady_clock::time_point streamStart;
    uint64_t arenaElems = 0;      // worst case per read: (maxSeeds + 2) * maxHits (+ 64)
    uint64_t arenaCap = 0;        // per wave in the main passes (= arenaElems unless that cannot fit the grid)
    int grid = 0, grid256 = 0, grid512 = 0, gridBig = 0;
    // snapgpu_align_batch chunk (SNAPGPU_CHUNK_READS): a streaming caller's 1M-read batches go
    // as one chunk each, alternating lanes (fewest persistent-kernel tails; A/B in
    // profiles/r02/ab/chunk_size_slots.txt); resident runs keep 2^18-read chunks over both lanes
    uint64_t chunkReads = 1u << 20;
    uint64_t residentChunk = 1u << 18;
    // forced mode: reads with at least this many elements get a radix-sorted pop order instead of
    // windowed ranks (SNAPGPU_RADIX_MIN; beyond SKCAP the ranks stage keys from HBM per window)
    uint32_t radixMin = SKCAP + 1;
    bool orderLong = true;        // pass 2's list longest-first (SNAPGPU_ORDER_LONG=0: pass 0's order)
    uint32_t tripRead = 0xffffffffu;   // test hook (snapgpu_aligner_debug_trip): trip the watchdog at this read
    snapgpu_timing_t timing{};
    snapgpu_aligner_stats_t stats{};
    snapgpu_device_reads_t *lastReads = nullptr;
    bool pendingTiming = false;
    uint32_t *dDiag = nullptr;    // this aligner's watchdog record (KArgs::diag)
    unsigned long long *dPhase = nullptr;   // [grid][PH_SLOTS] (SNAPGPU_PHASES=1 diagnostics)
    double timeoutSec = 0;        // SNAPGPU_TIMEOUT_S
    // A wait that timed out leaves kernels running on buffers this aligner owns: from then on
    // nothing is freed or reused (hipFree would block on the running kernel, a reuse could
    // fault it); every call fails and the process is expected to exit.
    bool failed = false;
    hipError_t (*eventQuery)(hipEvent_t) = hipEventQuery;   // test hook (snapgpu_selftest_timeout_path)
    hipEvent_t cev[2] = {};       // cigar_kernel timing
    // snapgpu_cigar_resident reads a resident batch's records (d->dOut) on the side stream; the
    // next pass set over resident reads (launch_resident: its 0xff pre-fill and the passes rewrite
    // those records) waits for this event on both lanes first
    hipEvent_t residentSideDone = nullptr;
    bool residentSidePending = false;
    int cigarGrid = 0;
    // snapgpu_align_batch_ex buffers, kept across calls (grow-only): search windows, multi-hit
    // scratch per block, found counts, hit rows, compaction offsets and the packed hits
    struct ExBuf { void *p = nullptr; uint64_t cap = 0; } exSearch, exScratch, exFound, exHits, exOff, exDense;
    // snapgpu_cigar_batch (device inputs, device outputs, pinned staging of the packed inputs) and
    // the internal scratch slots of snapgpu_internal_devbuf (charseeds.hip), grow-only: a
    // hipMalloc / hipFree pair per call cost more than the kernels, and hipFree waits for the
    // whole device (the RNA path's other host thread included)
    ExBuf cgIn, cgOut, aux[8];
    // snapgpu_internal_align_batch_packed: its device reads, kept (grow-only) across calls -- a
    // snapgpu_reads_upload / _free per call is ten hipMalloc / hipFree pairs, and each hipFree waits
    // for the whole device, the RNA path's concurrent genome aligner included
    snapgpu_device_reads_t *exReads = nullptr;
    uint64_t exReadsCapN = 0, exReadsCapBytes = 0;
    void *cgPin = nullptr, *cgPinOut = nullptr;
    uint64_t cgPinCap = 0, cgPinOutCap = 0;
    hipStream_t stream() const { return lane[0].stream; }
};

static const size_t kDevGuard = 1024;
static std::atomic<uint64_t> g_devFrees{0};   // hipFree calls made by devFree (selftest)

// Random-gather ceiling of the hash-table memory (roofline calibration for
// seed_lookup_kernel): one independent 64-byte bucket line per load, four
// loads per lane, at hashed positions of the resident bucket image -- the lookup kernel's access
// pattern (one whole line per lookup, four 16-B loads) without its dependency chain.  The xor of
// the loaded words goes to `sink` only when it equals the salt (practically never), so the loads
// cannot be dropped.
__global__ __launch_bounds__(256) void gather_peak_kernel(const uint4 *buckets, uint32_t nBuckets, uint32_t nLoads,
                                                          uint32_t salt, uint32_t *sink) {
    const uint32_t i = (blockIdx.x * 256u + threadIdx.x) * 4u;   // 4 independent lines per lane
    uint32_t x = 0;
#pragma unroll
    for (uint32_t j = 0; j < 4; j++)
        if (i + j < nLoads) {
            const uint4 *p = buckets + 4ull * (sgk::fmix32((i + j) ^ salt) % nBuckets);
#pragma unroll
            for (int q = 0; q < 4; q++) { const uint4 v = p[q]; x ^= v.x ^ v.y ^ v.z ^ v.w; }
        }
    if (x == salt) sink[0] = x;   // data-dependent: the loads stay
}

// Streaming-copy ceiling of this GPU's HBM (roofline peak calibration, BASELINE.md:47-50):
// 16-byte vector loads and stores, grid-stride, nWords uint4 read and written.
__global__ __launch_bounds__(256) void copy_peak_kernel(const uint4 *__restrict__ src, uint4 *__restrict__ dst,
                                                        uint64_t nWords) {
    // four independent 16-B loads in flight per lane, then four stores (nWords % 1024 == 0)
    const uint64_t stride = (uint64_t)gridDim.x * 1024u;
    for (uint64_t i = (uint64_t)blockIdx.x * 1024u + threadIdx.x; i < nWords; i += stride) {
        uint4 v[4];
#pragma unroll
        for (int j = 0; j < 4; j++) v[j] = src[i + 256 * j];
#pragma unroll
        for (int j = 0; j < 4; j++) dst[i + 256 * j] = v[j];
    }
}

// Multi-hit download (snapgpu_align_batch_ex): the found hits of every read, rows of
// maxHitsToGet on the device, packed into one dense array at host-computed offsets so only
// they cross PCIe (the RNA path asks for 1000 per read and finds a handful).  Wave per read.
__global__ __launch_bounds__(256) void compact_hits_kernel(const snapgpu_multi_hit_t *__restrict__ src,
                                                           const int32_t *__restrict__ found,
                                                           const uint64_t *__restrict__ off, uint64_t n, uint32_t mh,
                                                           snapgpu_multi_hit_t *__restrict__ dst) {
    const uint64_t waves = (uint64_t)gridDim.x * 4u;
    for (uint64_t r = (uint64_t)blockIdx.x * 4u + threadIdx.x / 64u; r < n; r += waves) {
        const uint32_t c = (uint32_t)found[r];
        for (uint32_t j = threadIdx.x % 64u; j < c; j += 64u) dst[off[r] + j] = src[r * mh + j];
    }
}

// Genome bit planes {hi, lo, notACGT} for 32 bases per 12-B GPlane (KArgs::gpl), built on the
// device from the uploaded genome bytes: word w covers device-genome bytes [32w, 32w + 32)
// of the guarded copy (position -kDevGuard at byte 0); bytes past `span` are not ACGT.
__global__ __launch_bounds__(256) void pack_planes_kernel(const char *g, uint64_t span, uint64_t nWords, sgk::GPlane *out) {
    const uint64_t w = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    if (w >= nWords) return;
    uint32_t hi = 0, lo = 0, nm = 0;
    const uint64_t b0 = w * 32;
#pragma unroll 4
    for (int i = 0; i < 32; i++) {
        const uint64_t p = b0 + (uint64_t)i;
        const uint32_t c = p < span ? (uint8_t)g[p] : 0u;
        const uint32_t v = sgk::packed_code(c), bit = 1u << i;
        if (v > 3) nm |= bit;
        else { if (v & 2) hi |= bit; if (v & 1) lo |= bit; }
    }
    out[w] = sgk::GPlane{hi, lo, nm};
}

// ------------------------------------------------- bucket image of the seed tables (bucket_table.h)
// Table of global slot i: tables are concatenated in order (tableBase ascending, sizes >= 1).
__device__ __forceinline__ uint32_t table_of_slot(const uint64_t *tableBase, uint32_t nTables, uint64_t i) {
    uint32_t lo = 0, hi = nTables;   // largest t with tableBase[t] <= i
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (tableBase[mid] <= i) lo = mid; else hi = mid;
    }
    return lo;
}

// SNAPHashTable::Lookup (HashTable.h:74-105) of `key` in table T of `size` slots: the slot it
// stops at when it reports the key found, else ~0.
__device__ __forceinline__ uint64_t ref_lookup_slot(const uint32_t *T, uint32_t size, uint32_t key) {
    const uint32_t h0 = sgk::fmix32(key) % size;
    for (uint32_t j = 0;; j++) {
        if (j > size + 5) return ~0ull;
        const uint32_t S_j = j <= 4 ? j * (j + 1) * (2 * j + 1) / 6 : 30 + (j - 4);
        uint64_t pos = h0 + S_j;
        if (pos >= size) pos %= size;
        const uint32_t kj = T[3 * pos], v1j = T[3 * pos + 1];
        const bool stop = (j == 0) ? (kj == key && v1j != sgk::INVALID) : (kj == key || v1j == sgk::INVALID);
        if (stop) return (j == 0 || v1j != sgk::INVALID) ? pos : ~0ull;
    }
}

// Per table, the slots the reference's Lookup of their own key returns (the keys the bucket image
// holds): each thread counts 256 consecutive slots and adds per table it crossed.
__global__ __launch_bounds__(256) void bucket_count_kernel(const uint32_t *slots, const uint64_t *tableBase,
                                                           const uint64_t *tableSize, uint32_t nTables,
                                                           uint64_t nSlots, unsigned long long *cnt) {
    const uint64_t i0 = ((uint64_t)blockIdx.x * 256u + threadIdx.x) * 256u;
    if (i0 >= nSlots) return;
    const uint64_t i1 = i0 + 256 < nSlots ? i0 + 256 : nSlots;
    uint32_t t = table_of_slot(tableBase, nTables, i0);
    uint64_t end = tableBase[t] + tableSize[t];
    unsigned long long c = 0;
    for (uint64_t i = i0; i < i1; i++) {
        while (i >= end) {
            if (c) atomicAdd(cnt + t, c);
            c = 0;
            t++;
            end = tableBase[t] + tableSize[t];
        }
        if (slots[3 * i + 1] == sgk::INVALID) continue;
        const uint64_t b = tableBase[t];
        if (ref_lookup_slot(slots + 3 * b, (uint32_t)tableSize[t], slots[3 * i]) == i - b) c++;
    }
    if (c) atomicAdd(cnt + t, c);
}

// Place every key the reference's Lookup returns into its table's buckets, deterministically.
// Phase 1 (bucket_place_kernel) works on the entries' first 8 bytes {key, 1 = occupied} only:
// bucketed linear probing from the key's home bucket in which a smaller key has priority -- a key
// that finds its bucket full takes the entry of the largest occupant greater than itself (64-bit
// CAS) and that occupant moves on to the next bucket, else the key moves on; a bucket left behind
// is flagged BK_OVF.  Keys only ever move forward, and the layout that results is the one
// sequential insertion in ascending key order gives, whatever order the claims race in
// (priority-ordered linear probing, Shun & Blelloch 2014), so which keys share a line -- the
// lookups' line counts, snapgpu_result_t::nProbes -- is the same on every build.  Phase 2
// (bucket_fill_kernel) gives each placed key its values and overflow-list counts from the
// reference table.  info: [0] keys placed, [1] buckets flagged, [2] keys that found no room (build
// error), [3] most buckets a key lives past its home.
// The counters are summed per thread and reduced over the wave before one atomic per wave: the
// library is built with the atomic optimizer off (Makefile), and one same-address atomic per key
// had serialised the whole kernel on info[0] (488 ms for C2's 38 M keys, 32 s of C3's upload).
__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
    for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o, 64));
    return v;
}
__global__ __launch_bounds__(256) void bucket_place_kernel(const uint32_t *slots, const uint64_t *tableBase,
                                                           const uint64_t *tableSize, uint32_t nTables, uint64_t nSlots,
                                                           uint4 *buckets, const uint64_t *bucketBase,
                                                           const uint32_t *bucketCount, unsigned long long *info) {
    constexpr uint64_t OCC = 1ull << 32;
    unsigned long long nPlaced = 0, nFailed = 0, nFlagged = 0;
    uint32_t maxD = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < nSlots; i += (uint64_t)gridDim.x * 256u) {
        if (slots[3 * i + 1] == sgk::INVALID) continue;
        const uint32_t t = table_of_slot(tableBase, nTables, i);
        const uint64_t b0 = tableBase[t];
        uint32_t x = slots[3 * i];
        if (ref_lookup_slot(slots + 3 * b0, (uint32_t)tableSize[t], x) != i - b0) continue;   // unreachable slot
        const uint32_t nB = bucketCount[t];
        uint4 *T = buckets + 4ull * bucketBase[t];
        uint32_t b = sgk::bucket_home(x, nB), moved = 0;
        bool placed = false;
        // every bucket step is a key moving forward: at most (keys in the table) * nB steps in all
        for (uint64_t guard = 0; guard < 8ull * nB + 64; guard++) {
            unsigned long long *E = reinterpret_cast<unsigned long long *>(T + 4ull * b);   // entry e: E[2e]
            int free = -1, victim = -1;
            uint32_t vk = 0;
            for (int e = 0; e < 4; e++) {
                const unsigned long long w = __hip_atomic_load(E + 2 * e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (w == 0ull) { if (free < 0) free = e; }
                else if ((uint32_t)w > x && (victim < 0 || (uint32_t)w > vk)) { victim = e; vk = (uint32_t)w; }
            }
            if (free >= 0) {
                if (atomicCAS(E + 2 * free, 0ull, OCC | x) == 0ull) {
                    maxD = max(maxD, (b + nB - sgk::bucket_home(x, nB)) % nB);
                    placed = true;
                    break;
                }
                continue;   // lost the entry: look at the bucket again
            }
            if (victim >= 0) {
                if (atomicCAS(E + 2 * victim, OCC | vk, OCC | x) != (OCC | vk)) continue;
                x = vk;   // the larger key moves on
            }
            if (!(atomicOr(&T[4ull * b].w, sgk::BK_OVF) & sgk::BK_OVF)) nFlagged++;
            b = sgk::bucket_next(b, nB);
            if (++moved > nB) break;
        }
        (placed ? nPlaced : nFailed)++;
    }
    nPlaced = wave_sum_u64(nPlaced);
    nFailed = wave_sum_u64(nFailed);
    nFlagged = wave_sum_u64(nFlagged);
    maxD = wave_max_u32(maxD);
    if ((threadIdx.x & 63) == 0) {
        if (nPlaced) atomicAdd(info + 0, nPlaced);
        if (nFlagged) atomicAdd(info + 1, nFlagged);
        if (nFailed) atomicAdd(info + 2, nFailed);
        if (maxD) atomicMax(info + 3, (unsigned long long)maxD);
    }
}

// Phase 2: {key, value1, value2, counts} of every placed key (the entry 0 flag kept).  Thread per entry.
__global__ __launch_bounds__(256) void bucket_fill_kernel(const uint32_t *slots, const uint64_t *tableBase,
                                                          const uint64_t *tableSize, uint32_t nTables,
                                                          const uint32_t *overflow, uint64_t nOverflow, uint32_t nBases,
                                                          uint4 *buckets, const uint64_t *bucketBase, uint64_t nEntries) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < nEntries; i += (uint64_t)gridDim.x * 256u) {
        uint4 &E = buckets[i];
        if (E.y != 1u) continue;   // empty
        const uint32_t t = table_of_slot(bucketBase, nTables, i / 4);
        const uint64_t b0 = tableBase[t];
        const uint64_t slot = ref_lookup_slot(slots + 3 * b0, (uint32_t)tableSize[t], E.x);
        const uint32_t v1 = slots[3 * (b0 + slot) + 1], v2 = slots[3 * (b0 + slot) + 2];
        uint32_t c[2] = {0, 0};
        const uint32_t vs[2] = {v1, v2};
        for (int s = 0; s < 2; s++)   // overflow-list lengths (GenomeIndex.cpp:1013-1086), saturated
            if (vs[s] >= nBases && vs[s] != sgk::UNUSED_SIDE && (uint64_t)(vs[s] - nBases) < nOverflow) {
                const uint32_t n = overflow[vs[s] - nBases];
                c[s] = n < sgk::BK_CSAT ? n : sgk::BK_CSAT;
            }
        E.y = v1;
        E.z = v2;
        E.w = (E.w & sgk::BK_OVF) | sgk::BK_OCC | c[0] | (c[1] << 15);
    }
}

// snapgpu_aligner_lookup_seeds: GenomeIndex::lookupSeed + fillInLookedUpResults (GenomeIndex.cpp:
// 971-1086, unwindowed) of given seeds through the bucket image, by either device lookup: lane per
// seed (bucket_lookup_lane, mode 0; bucket_lookup_quad, mode 2) or the whole wave per seed
// (bucket_lookup_wave, mode 1).  Per
// seed: {nFwd, nRc, hash of the forward hits, of the RC hits, first forward hit, first RC hit}, the
// hash acc = acc * 1000003 + hit over the hits in list order; `lines` = bucket lines loaded.
__device__ __forceinline__ void lookup_fill(const KArgs &A, uint32_t v, uint32_t c, uint64_t *o) {
    uint32_t n = 0;
    uint64_t acc = 0, first = ~0ull;
    if (v < A.nBases) { n = 1; acc = v; first = v; }
    else if (v != UNUSED_SIDE) {
        n = bucket_count(A, c, v);
        const uint32_t *ls = A.overflow + (v - A.nBases) + 1;
        for (uint32_t i = 0; i < n; i++) acc = acc * 1000003ull + ls[i];
        if (n) first = ls[0];
    }
    o[0] = n; o[1] = acc; o[2] = first;
}
__global__ __launch_bounds__(64) void lookup_seeds_kernel(KArgs A, const char *seeds, uint32_t n, int mode,
                                                          unsigned long long *out, uint32_t *lines) {
    const int lane = lane_id();
    const uint32_t L = A.seedLen;
    for (uint32_t base = blockIdx.x * 64u; base < n; base += gridDim.x * 64u) {
        const uint32_t cnt = n - base < 64u ? n - base : 64u;
        // mode 0 / 2: lane per seed; mode 2 (bucket_lookup_quad, seed_lookup_kernel's lookup) runs in
        // two rounds, each with a scattered half of the wave's lanes active (and the tail block's
        // lanes past n inactive in both), so partially active waves are what it is checked on
        const uint32_t rounds = mode == 1 ? cnt : (mode == 2 ? 2u : 1u);
        for (uint32_t k = 0; k < rounds; k++) {
            const uint32_t i = mode == 1 ? base + k : base + lane;   // mode 1: seed base+k, uniform
            bool act = mode == 1 || (uint32_t)lane < cnt;
            if (mode == 2) act = act && ((fmix32(i) & 1u) == k);
            if (mode == 0 && !act) break;
            uint64_t f = 0, rc = 0;
            if (act)
                for (uint32_t j = 0; j < L; j++) {
                    const int v = base_value((uint8_t)seeds[(uint64_t)i * L + j]) & 3;
                    f |= (uint64_t)v << ((L - j - 1) * 2);
                    rc |= (uint64_t)(v ^ 3) << (j * 2);
                }
            const bool comp = (int64_t)f > (int64_t)rc;
            const uint64_t canon = comp ? rc : f;
            uint32_t v1 = 0, v2 = 0, aux = 0, ln = 0;
            bool found;
            if (mode == 1) found = bucket_lookup_wave(A, (uint32_t)(canon >> 32), (uint32_t)canon, lane, v1, v2, aux, ln);
            else if (mode == 2) found = bucket_lookup_quad(A, act, (uint32_t)(canon >> 32), (uint32_t)canon, v1, v2, aux, ln);
            else found = bucket_lookup_lane(A, (uint32_t)(canon >> 32), (uint32_t)canon, v1, v2, aux, ln);
            if ((mode == 1 && lane != 0) || !act) continue;
            uint64_t o[6] = {0, 0, 0, 0, ~0ull, ~0ull};
            if (found) {
                const uint32_t c1 = aux & BK_CSAT, c2 = (aux >> 15) & BK_CSAT;
                uint64_t a[3], b[3];
                lookup_fill(A, comp ? v2 : v1, comp ? c2 : c1, a);
                if (f == rc) { b[0] = a[0]; b[1] = a[1]; b[2] = a[2]; }   // palindrome (GenomeIndex.cpp:1003-1006)
                else lookup_fill(A, comp ? v1 : v2, comp ? c1 : c2, b);
                o[0] = a[0]; o[1] = b[0]; o[2] = a[1]; o[3] = b[1]; o[4] = a[2]; o[5] = b[2];
            }
            for (int q = 0; q < 6; q++) out[6ull * i + q] = o[q];
            lines[i] = ln;
        }
    }
}

// ------------------------------------------------------------------ host helpers
namespace {

std::atomic<int> g_hostDevices{-2};   // HIP devices visible to hostAlloc (-2: not probed yet)

// Page-locked batch buffers are parked on free and reused by the next hostAlloc of a similar size
// (a FASTQ batch of 1M reads pins 2 x 100 MB; hipHostMalloc + hipHostFree of them was most of a
// parse).  At most kPinParkBytes stay parked; larger frees go back to the runtime.  A batch must not
// be freed while a submitted call still reads it -- as with the runtime's free.
constexpr size_t kPinParkBytes = 2ull << 30;
std::mutex g_pinMu;
std::vector<std::pair<void *, size_t>> g_pinParked;            // (block, capacity)
std::vector<std::pair<void *, size_t>> g_pinLive;              // blocks handed out, with their capacity
size_t g_pinParkedBytes = 0;

// Every device free goes through here: after a timeout the aligner's buffers may still be
// in use by a running kernel, so they are left alone (see snapgpu_aligner::failed).
void devFree(const snapgpu_aligner_t *a, void *p) {
    if (!p || (a && a->failed)) return;
    g_devFrees++;
    hipFree(p);
}

void hostPinnedFree(void *p) { if (p) hipHostFree(p); }

// Wait for an event, honouring SNAPGPU_TIMEOUT_S: on expiry the aligner is marked failed.
int waitEvent(snapgpu_aligner_t *a, hipEvent_t ev) {
    if (a->failed) { snapgpu::setError("aligner failed earlier (device timeout): no further work accepted"); return SNAPGPU_EDEVICE; }
    if (a->timeoutSec > 0) {
        const auto t0 = std::chrono::steady_clock::now();
        for (;;) {
            const hipError_t q = a->eventQuery(ev);
            if (q == hipSuccess) break;
            if (q != hipErrorNotReady) HIPCHK(q);
            if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > a->timeoutSec) {
                a->failed = true;
                snapgpu::setError("align kernel did not finish within SNAPGPU_TIMEOUT_S; the aligner is unusable "
                                  "and its device buffers are not released (exit the process)");
                return SNAPGPU_EDEVICE;
            }
            std::this_thread::sleep_for(std::chrono::microseconds(200));
        }
    }
    HIPCHK(hipEventSynchronize(ev));
    return SNAPGPU_OK;
}

// Wait for everything queued on a lane's stream (an event recorded now, then waitEvent).
int waitLane(snapgpu_aligner_t *a, ExecLane &L) {
    if (a->failed) return waitEvent(a, nullptr);
    HIPCHK(hipEventRecord(L.done, L.stream));
    return waitEvent(a, L.done);
}

// Host -> device copy of a large pageable buffer through two pinned staging buffers: host
// threads fill one while the DMA engine drains the other (the index tables, up to tens of
// GB for a human-sized genome; a plain pageable hipMemcpy runs far below PCIe speed).
int uploadLarge(hipStream_t s, void *dst, const void *src, uint64_t bytes) {
    if (bytes == 0) return SNAPGPU_OK;
    if (bytes < (64ull << 20)) {
        HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s));
        HIPCHK(hipStreamSynchronize(s));
        return SNAPGPU_OK;
    }
    const uint64_t CH = 256ull << 20;
    void *stg[2] = {nullptr, nullptr};
    hipEvent_t ev[2] = {nullptr, nullptr};
    int rc = SNAPGPU_OK;
    auto fail = [&](hipError_t e) {
        snapgpu::setError(std::string("uploadLarge: ") + hipGetErrorString(e));
        rc = SNAPGPU_EDEVICE;
    };
    hipError_t e;
    for (int i = 0; i < 2 && rc == SNAPGPU_OK; i++) {
        if ((e = hipHostMalloc(&stg[i], CH, hipHostMallocDefault)) != hipSuccess) fail(e);
        else if ((e = hipEventCreateWithFlags(&ev[i], hipEventDisableTiming)) != hipSuccess) fail(e);
    }
    const unsigned nt = snapgpu::hostThreads(8);
    for (uint64_t off = 0, k = 0; off < bytes && rc == SNAPGPU_OK; off += CH, k++) {
        const int b = (int)(k & 1);
        const uint64_t len = std::min(CH, bytes - off);
        if (k >= 2 && (e = hipEventSynchronize(ev[b])) != hipSuccess) { fail(e); break; }
        std::vector<std::thread> th;
        for (unsigned t = 0; t < nt; t++)
            th.emplace_back([&, t] {
                const uint64_t a0 = len * t / nt, a1 = len * (t + 1) / nt;
                memcpy((char *)stg[b] + a0, (const char *)src + off + a0, a1 - a0);
            });
        for (auto &x : th) x.join();
        if ((e = hipMemcpyAsync((char *)dst + off, stg[b], len, hipMemcpyHostToDevice, s)) != hipSuccess) { fail(e); break; }
        if ((e = hipEventRecord(ev[b], s)) != hipSuccess) { fail(e); break; }
    }
    if ((e = hipStreamSynchronize(s)) != hipSuccess && rc == SNAPGPU_OK) fail(e);
    for (int i = 0; i < 2; i++) {
        if (stg[i]) hipHostFree(stg[i]);
        if (ev[i]) hipEventDestroy(ev[i]);
    }
    return rc;
}

}  // namespace

namespace snapgpu {
void *hostAlloc(size_t bytes, bool *pinned, bool zero) {
    *pinned = false;
    int nd = g_hostDevices.load();
    if (nd == -2) {
        if (hipGetDeviceCount(&nd) != hipSuccess) nd = 0;
        g_hostDevices = nd;
    }
    // batches of >= 1 MB that a GPU will copy from live in page-locked memory
    if (nd > 0 && bytes >= (1u << 20)) {
        void *p = nullptr;
        size_t cap = bytes;
        {
            std::lock_guard<std::mutex> lk(g_pinMu);
            int best = -1;
            for (size_t i = 0; i < g_pinParked.size(); i++)   // the smallest parked block that fits, within 2x
                if (g_pinParked[i].second >= bytes && g_pinParked[i].second <= 2 * bytes &&
                    (best < 0 || g_pinParked[i].second < g_pinParked[(size_t)best].second))
                    best = (int)i;
            if (best >= 0) {
                p = g_pinParked[(size_t)best].first;
                cap = g_pinParked[(size_t)best].second;
                g_pinParkedBytes -= cap;
                g_pinParked.erase(g_pinParked.begin() + best);
            }
        }
        if (!p && (hipHostMalloc(&p, bytes, hipHostMallocPortable) != hipSuccess || !p)) p = nullptr;
        if (p) {
            if (zero) memset(p, 0, bytes);
            std::lock_guard<std::mutex> lk(g_pinMu);
            g_pinLive.push_back({p, cap});
            *pinned = true;
            return p;
        }
    }
    return zero ? calloc(bytes, 1) : malloc(bytes ? bytes : 1);
}
void hostFree(void *p, bool pinned) {
    if (!p) return;
    if (!pinned) { free(p); return; }
    {
        std::lock_guard<std::mutex> lk(g_pinMu);
        for (size_t i = 0; i < g_pinLive.size(); i++)
            if (g_pinLive[i].first == p) {
                const size_t cap = g_pinLive[i].second;
                g_pinLive.erase(g_pinLive.begin() + i);
                if (g_pinParkedBytes + cap <= kPinParkBytes) {
                    g_pinParked.push_back({p, cap});
                    g_pinParkedBytes += cap;
                    return;
                }
                break;
            }
    }
    hipHostFree(p);
}
}  // namespace snapgpu

extern "C" {

void snapgpu_aligner_params_default(snapgpu_aligner_params_t *p) {
    // AlignerOptions.cpp:33-85 defaults used by SingleAligner.cpp:167-179
    p->maxHitsToConsider = 300;
    p->maxK = 14;
    p->maxReadSize = 500;
    p->maxSeedsToUse = 25;
    p->maxSeedCoverage = 0;
    p->extraSearchDepth = 2;
    p->explorePopularSeeds = 0;
    p->stopOnFirstHit = 0;
}

int snapgpu_compute_mapq(double pAll, double pBest, int score, int popular) { return hostMapq(pAll, pBest, score, popular); }

int snapgpu_device_cu_count(int device) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return 0;
    return prop.multiProcessorCount;
}

int snapgpu_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

// The seed tables' bucket image (bucket_table.h): the reference-format slots go to the device once,
// bucket_count_kernel counts per table the keys SNAPHashTable::Lookup can return, the host sizes
// the tables (ceil(keys / BK_KEYS_PER_BUCKET) buckets each), bucket_place_kernel places the keys
// (deterministically) and bucket_fill_kernel their values, and the slots are freed again: the
// kernels read only the buckets.
static int buildBuckets(snapgpu_aligner_t *a, hipStream_t s0) {
    const snapgpu_index_t *idx = a->idx;
    const auto t0 = std::chrono::steady_clock::now();
    const uint64_t nSlots = idx->slots.size() / 3;
    const uint32_t nT = idx->nTables;
    uint32_t *dSlots = nullptr;
    uint64_t *dTB = nullptr, *dTS = nullptr;
    unsigned long long *dCnt = nullptr;
    int rc = SNAPGPU_OK;
    hipError_t e = hipSuccess;
    auto chk = [&](hipError_t x, const char *what) {
        if (x != hipSuccess && rc == SNAPGPU_OK) {
            e = x;
            snapgpu::setError(std::string("bucket image: ") + what + ": " + hipGetErrorString(x));
            rc = x == hipErrorOutOfMemory ? SNAPGPU_ENOMEM : SNAPGPU_EDEVICE;
        }
        return rc == SNAPGPU_OK;
    };
    std::vector<unsigned long long> cnt(nT + 4, 0);
    if (chk(hipMalloc(&dSlots, nSlots * 12 + 16), "slots") && uploadLarge(s0, dSlots, idx->slots.data(), nSlots * 12))
        rc = SNAPGPU_EDEVICE;
    if (rc == SNAPGPU_OK && chk(hipMalloc(&dTB, nT * 8ull), "tables") && chk(hipMalloc(&dTS, nT * 8ull), "tables") &&
        chk(hipMalloc(&dCnt, (nT + 4) * 8ull), "counts") &&
        chk(hipMemcpyAsync(dTB, idx->tableBase.data(), nT * 8ull, hipMemcpyHostToDevice, s0), "tables") &&
        chk(hipMemcpyAsync(dTS, idx->tableSize.data(), nT * 8ull, hipMemcpyHostToDevice, s0), "tables") &&
        chk(hipMemsetAsync(dCnt, 0, (nT + 4) * 8ull, s0), "counts")) {
        const uint64_t nThreads = (nSlots + 255) / 256;
        hipLaunchKernelGGL(bucket_count_kernel, dim3((unsigned)((nThreads + 255) / 256)), dim3(256), 0, s0, dSlots, dTB, dTS,
                           nT, nSlots, dCnt);
        if (chk(hipGetLastError(), "bucket_count_kernel") &&
            chk(hipMemcpyAsync(cnt.data(), dCnt, nT * 8ull, hipMemcpyDeviceToHost, s0), "counts") &&
            chk(hipStreamSynchronize(s0), "bucket_count_kernel")) {
            std::vector<uint64_t> base(nT);
            std::vector<uint32_t> nb(nT);
            uint64_t total = 0, keys = 0;
            for (uint32_t t = 0; t < nT; t++) {
                const uint64_t want = std::max<uint64_t>(1, (cnt[t] + BK_KEYS_PER_BUCKET - 1) / BK_KEYS_PER_BUCKET);
                if (want >= (1ull << 32)) { snapgpu::setError("bucket image: table too large"); rc = SNAPGPU_EINVAL; break; }
                base[t] = total; nb[t] = (uint32_t)want; total += want; keys += cnt[t];
            }
            if (rc == SNAPGPU_OK && chk(hipMalloc(&a->dBuckets, total * 64), "buckets") &&
                chk(hipMalloc(&a->dBucketBase, nT * 8ull), "buckets") && chk(hipMalloc(&a->dBucketCount, nT * 4ull), "buckets") &&
                chk(hipMemsetAsync(a->dBuckets, 0, total * 64, s0), "buckets") &&
                chk(hipMemcpyAsync(a->dBucketBase, base.data(), nT * 8ull, hipMemcpyHostToDevice, s0), "buckets") &&
                chk(hipMemcpyAsync(a->dBucketCount, nb.data(), nT * 4ull, hipMemcpyHostToDevice, s0), "buckets") &&
                chk(hipMemsetAsync(dCnt, 0, 4 * 8, s0), "counts")) {
                hipLaunchKernelGGL(bucket_place_kernel, dim3((unsigned)std::min<uint64_t>((nSlots + 255) / 256, 1u << 20)),
                                   dim3(256), 0, s0, dSlots, dTB, dTS, nT, nSlots, a->dBuckets, a->dBucketBase,
                                   a->dBucketCount, dCnt);
                hipLaunchKernelGGL(bucket_fill_kernel, dim3((unsigned)std::min<uint64_t>((4 * total + 255) / 256, 1u << 20)),
                                   dim3(256), 0, s0, dSlots, dTB, dTS, nT, a->dOverflow, (uint64_t)idx->overflow.size(),
                                   idx->genome->nBases, a->dBuckets, a->dBucketBase, 4 * total);
                unsigned long long info[4] = {0, 0, 0, 0};
                if (chk(hipGetLastError(), "bucket_place_kernel / bucket_fill_kernel") &&
                    chk(hipMemcpyAsync(info, dCnt, sizeof(info), hipMemcpyDeviceToHost, s0), "counts") &&
                    chk(hipStreamSynchronize(s0), "bucket image build")) {
                    if (info[2] || info[0] != keys) {
                        snapgpu::setError("bucket image: " + std::to_string(info[2]) + " keys found no bucket, " +
                                          std::to_string(info[0]) + " of " + std::to_string(keys) + " inserted");
                        rc = SNAPGPU_EDEVICE;
                    }
                    snapgpu_bucket_info_t &bi = a->bucketInfo;
                    bi.nBuckets = total; bi.nKeys = info[0]; bi.nSlots = nSlots;
                    bi.nOverflowBuckets = info[1]; bi.maxDisplacement = info[3]; bi.bytes = total * 64;
                }
            }
        }
    }
    devFree(a, dSlots); devFree(a, dTB); devFree(a, dTS); devFree(a, dCnt);
    a->bucketInfo.buildMs = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return rc;
}

static void freeLaneChunkBuffers(snapgpu_aligner_t *a, ExecLane &L) {
    devFree(a, L.dDefer); devFree(a, L.dOut); devFree(a, L.dSeeds);
    L.dDefer = nullptr; L.dOut = nullptr; L.dSeeds = nullptr;
    for (ChunkSlot &S : L.slot) {
        devFree(a, S.dBases); devFree(a, S.dQuals); devFree(a, S.dOffsets); devFree(a, S.dLengths);
        S.dBases = S.dQuals = nullptr; S.dOffsets = nullptr; S.dLengths = nullptr;
        if (!a->failed) { hostPinnedFree(S.hOffsets); hostPinnedFree(S.hLengths); hostPinnedFree(S.hOut); }
        S.hOffsets = nullptr; S.hLengths = nullptr; S.hOut = nullptr;
    }
    L.capReads = L.capBytes = 0;
}

void snapgpu_aligner_free(snapgpu_aligner_t *a) {
    if (!a) return;
    if (a->failed) {   // kernels may still run on these buffers: leave them (the process must exit)
        delete a;
        return;
    }
    hipSetDevice(a->device);
    for (auto &L : a->lane) if (L.stream) hipStreamSynchronize(L.stream);
    devFree(a, a->dBuckets); devFree(a, a->dOverflow); devFree(a, a->dPieces);
    devFree(a, a->dBucketBase); devFree(a, a->dBucketCount); devFree(a, a->dGenomeAlloc); devFree(a, a->dTab);
    devFree(a, a->dGPlanes); devFree(a, a->dPhase); devFree(a, a->dDiag);
    for (auto &L : a->lane) {
        freeLaneChunkBuffers(a, L);
        devFree(a, L.arena); devFree(a, L.bigArena); devFree(a, L.counter); devFree(a, L.lookupStats);
        hostPinnedFree(L.hLookupStats);
        if (L.done) hipEventDestroy(L.done);
        for (ChunkSlot &S : L.slot) {
            if (S.h2d) hipEventDestroy(S.h2d);
            if (S.done) hipEventDestroy(S.done);
        }
        if (L.stream) hipStreamDestroy(L.stream);
    }
    if (a->copyStream) { hipStreamSynchronize(a->copyStream); hipStreamDestroy(a->copyStream); }
    if (a->sideStream) { hipStreamSynchronize(a->sideStream); hipStreamDestroy(a->sideStream); }
    for (auto &v : a->evs) {
        for (auto &e : v.e) if (e) hipEventDestroy(e);
        hostPinnedFree(v.hCounter);
    }
    for (auto &e : a->cev) if (e) hipEventDestroy(e);
    if (a->residentSideDone) hipEventDestroy(a->residentSideDone);
    for (auto *b : {&a->cgIn, &a->cgOut}) devFree(a, b->p);
    for (auto &b : a->aux) devFree(a, b.p);
    hostPinnedFree(a->cgPin);
    hostPinnedFree(a->cgPinOut);
    snapgpu_device_reads_free(a->exReads);
    for (auto *b : {&a->exSearch, &a->exScratch, &a->exFound, &a->exHits, &a->exOff, &a->exDense}) devFree(a, b->p);
    delete a;
}

snapgpu_aligner_t *snapgpu_aligner_create(int device, const snapgpu_index_t *idx, const snapgpu_aligner_params_t *params) {
    if (!idx || !params) { snapgpu::setError("aligner_create: null argument"); return nullptr; }
    if (params->maxK + params->extraSearchDepth > (uint32_t)MAX_K) {   // SingleAligner.cpp:117-121
        snapgpu::setError("maxK + extraSearchDepth must be <= MAX_K (31)");
        return nullptr;
    }
    if (params->maxReadSize > 512) { snapgpu::setError("maxReadSize > 512 unsupported"); return nullptr; }
    if (idx->seedLen < 16 || idx->seedLen > 25) { snapgpu::setError("seedLen must be 16..25 (SeedSequencer.h)"); return nullptr; }
    int ndev = snapgpu_device_count();
    if (ndev <= 0 || device < 0 || device >= ndev) { snapgpu::setError("no such HIP device"); return nullptr; }
    auto *a = new snapgpu_aligner_t();
    a->device = device;
    a->idx = idx;
    a->p = *params;
    if (const char *t = getenv("SNAPGPU_TIMEOUT_S")) a->timeoutSec = atof(t);
    if (const char *t = getenv("SNAPGPU_CHUNK_READS"); t && atoll(t) > 0) a->chunkReads = (uint64_t)atoll(t);
    if (const char *t = getenv("SNAPGPU_RADIX_MIN"); t && atoll(t) > 0) a->radixMin = (uint32_t)atoll(t);
    if (const char *t = getenv("SNAPGPU_OVERLAP")) a->overlapKernels = atoi(t) != 0;
    if (const char *t = getenv("SNAPGPU_ORDER_LONG")) a->orderLong = atoi(t) != 0;
    auto fail = [&](const char *what, hipError_t e) {
        snapgpu::setError(std::string(what) + ": " + hipGetErrorString(e));
        snapgpu_aligner_free(a);
        return (snapgpu_aligner_t *)nullptr;
    };
    hipError_t e;
    if ((e = hipSetDevice(device)) != hipSuccess) return fail("hipSetDevice", e);
    for (auto &L : a->lane) {
        if ((e = hipStreamCreateWithFlags(&L.stream, hipStreamNonBlocking)) != hipSuccess) return fail("stream", e);
        if ((e = hipEventCreateWithFlags(&L.done, hipEventDisableTiming)) != hipSuccess) return fail("event", e);
        for (ChunkSlot &S : L.slot)
            if ((e = hipEventCreateWithFlags(&S.h2d, hipEventDisableTiming)) != hipSuccess ||
                (e = hipEventCreateWithFlags(&S.done, hipEventDisableTiming)) != hipSuccess)
                return fail("event", e);
        if ((e = hipMalloc(&L.counter, 64)) != hipSuccess) return fail("counter", e);
        if ((e = hipMalloc(&L.lookupStats, 1024 * sizeof(unsigned long long))) != hipSuccess) return fail("lookup stats", e);
        if ((e = hipHostMalloc(&L.hLookupStats, 1024 * sizeof(unsigned long long), hipHostMallocDefault)) != hipSuccess)
            return fail("pinned lookup stats", e);
    }
    if ((e = hipStreamCreateWithFlags(&a->copyStream, hipStreamNonBlocking)) != hipSuccess) return fail("stream", e);
    {
        // the side stream's calls (CIGARs, seed census) sit on a caller's critical path while the
        // lanes' persistent kernels hold the CUs: its queue gets the device's highest priority, so
        // its kernels are dispatched ahead of the lanes' next ones (SNAPGPU_SIDE_PRIORITY=0: normal)
        int least = 0, greatest = 0;
        const char *t = getenv("SNAPGPU_SIDE_PRIORITY");
        const bool high = !(t && atoi(t) == 0) && hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess;
        if ((e = high ? hipStreamCreateWithPriority(&a->sideStream, hipStreamNonBlocking, greatest)
                      : hipStreamCreateWithFlags(&a->sideStream, hipStreamNonBlocking)) != hipSuccess) return fail("stream", e);
    }
    for (auto &ev : a->cev) if ((e = hipEventCreate(&ev)) != hipSuccess) return fail("event", e);
    if ((e = hipEventCreateWithFlags(&a->residentSideDone, hipEventDisableTiming)) != hipSuccess) return fail("event", e);
    hipStream_t s0 = a->stream();
    // Every buffer is initialised on the stream of its first consumer or before the device-wide
    // synchronisation at the end of this function (stream audit): no
    // null-stream fill or copy may race the non-blocking lane streams.
    if ((e = hipMalloc(&a->dDiag, 4 * sizeof(uint32_t))) != hipSuccess) return fail("watchdog record", e);
    if ((e = hipMemsetAsync(a->dDiag, 0, 4 * sizeof(uint32_t), s0)) != hipSuccess) return fail("watchdog record", e);
    if ((e = ensureDeviceTables(device)) != hipSuccess) return fail("device tables", e);
    // index upload: genome with guards, tables, overflow, pieces
    const uint32_t nBases = idx->genome->nBases;
    const size_t gbytes = kDevGuard + nBases + kDevGuard;
    if ((e = hipMalloc(&a->dGenomeAlloc, gbytes)) != hipSuccess) return fail("hipMalloc genome", e);
    if ((e = hipMemsetAsync(a->dGenomeAlloc, 'n', gbytes, s0)) != hipSuccess) return fail("genome guard", e);
    if (uploadLarge(s0, a->dGenomeAlloc + kDevGuard, idx->genome->bases(), nBases)) { snapgpu_aligner_free(a); return nullptr; }
    a->dGenome = a->dGenomeAlloc + kDevGuard;
    {
        // genome bit planes {hi, lo, notACGT}, 32 bases per 12-B GPlane, covering genome
        // positions [-kDevGuard, nBases + kDevGuard): the per-lane LV mismatch masks of
        // align_kernel<128> are built from these with funnel shifts (align_score.h).
        const uint64_t span = (uint64_t)nBases + 2 * kDevGuard;
        const uint64_t nw = (span + 31) / 32 + 8;
        if ((e = hipMalloc(&a->dGPlanes, nw * sizeof(GPlane))) != hipSuccess) return fail("hipMalloc planes", e);
        hipLaunchKernelGGL(pack_planes_kernel, dim3((unsigned)((nw + 255) / 256)), dim3(256), 0, s0, a->dGenomeAlloc,
                           span, nw, a->dGPlanes);
        if ((e = hipGetLastError()) != hipSuccess) return fail("pack_planes_kernel", e);
    }
    if ((e = hipMalloc(&a->dOverflow, idx->overflow.size() * 4 + 16)) != hipSuccess) return fail("hipMalloc ovf", e);
    if (uploadLarge(s0, a->dOverflow, idx->overflow.data(), idx->overflow.size() * 4)) { snapgpu_aligner_free(a); return nullptr; }
    for (uint32_t t = 0; t < idx->nTables; t++)   // the builder hashes with 32-bit modulo
        if (idx->tableSize[t] == 0 || idx->tableSize[t] >= (1ull << 31)) {
            snapgpu::setError("hash table size must be in [1, 2^31)");
            snapgpu_aligner_free(a);
            return nullptr;
        }
    if (int rc = buildBuckets(a, s0)) { (void)rc; snapgpu_aligner_free(a); return nullptr; }
    size_t np = idx->genome->pieceOffsets.size();
    if ((e = hipMalloc(&a->dPieces, np * 4 + 16)) != hipSuccess) return fail("pieces", e);
    if (np && (e = hipMemcpy(a->dPieces, idx->genome->pieceOffsets.data(), np * 4, hipMemcpyHostToDevice)) != hipSuccess)
        return fail("pieces", e);
    DevTables t;
    fillTables(t, idx->seedLen);
    for (uint32_t len = 0; len <= 512; len++)   // BaseAligner.cpp:563-568, double arithmetic as there
        t.maxSeedsForLen[len] = (uint32_t)(int)(params->maxSeedCoverage * (double)len / (double)idx->seedLen);
    if ((e = hipMalloc(&a->dTab, sizeof(DevTables))) != hipSuccess) return fail("tables", e);
    if ((e = hipMemcpy(a->dTab, &t, sizeof(t), hipMemcpyHostToDevice)) != hipSuccess) return fail("tables", e);
    // persistent grid: waves resident on the device; element arena per wave and lane
    hipDeviceProp_t prop;
    hipGetDeviceProperties(&prop, device);
    int perCU = 0;
    hipOccupancyMaxActiveBlocksPerMultiprocessor(&perCU, (const void *)align_kernel<128, false>, 64, 0);
    if (perCU <= 0) perCU = 8;
    // occupancy test hook: fewer resident waves per CU than the kernel's resources allow
    // (the same code, LDS caps and registers; only the persistent grid shrinks)
    if (const char *t = getenv("SNAPGPU_WAVES_PER_CU"); t && atoi(t) > 0) perCU = std::min(perCU, atoi(t));
    a->grid = prop.multiProcessorCount * perCU;
    uint32_t maxSeeds = params->maxSeedsToUse ? params->maxSeedsToUse
                                              : (uint32_t)(params->maxSeedCoverage * params->maxReadSize / idx->seedLen);
    a->arenaElems = (uint64_t)(maxSeeds + 2) * params->maxHitsToConsider + 64;
    // Element arenas.  The whole grid keeps its occupancy: when worst-case arenas for every wave
    // would pass the lane's budget (maxHits 16000 of the RNA aligners: 23 MB per wave), the main
    // passes run on capped arenas and the rare read that outgrows one is aligned again by the
    // big-arena pass, align_kernel<512> on a small grid of worst-case arenas (KArgs::ovfList).
    // (Round 2 halved the grid instead: the RNA aligners ran at 1 wave per SIMD.)
    const uint64_t budget = 8ull << 30, bigBudget = 4ull << 30;   // HBM per lane: main and big-arena pass
    a->arenaCap = std::min<uint64_t>(a->arenaElems, budget / ((uint64_t)a->grid * sizeof(Elem512)));
    // the bit-plane kernels keep u16 element indices in their LDS chain heads (Lds::HeadT)
    a->arenaCap = std::min<uint64_t>(a->arenaCap, 0xfffeu);
    // and at most ELEM64_MAX slots (an Elem64's spill index is 15 bits of w11)
    a->arenaCap = std::min<uint64_t>(a->arenaCap, ELEM64_MAX);
    if (const char *t = getenv("SNAPGPU_ARENA_CAP"); t && atoll(t) >= 1)   // test hook: force the overflow path
        a->arenaCap = std::min<uint64_t>(a->arenaCap, (uint64_t)atoll(t));
    if (a->arenaCap < a->arenaElems)
        a->gridBig = (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)a->grid, bigBudget / (a->arenaElems * sizeof(Elem512))));
    for (auto &L : a->lane) {
        if ((e = hipMalloc(&L.arena, (uint64_t)a->grid * a->arenaCap * sizeof(Elem512))) != hipSuccess) return fail("arena", e);
        if (a->gridBig &&
            (e = hipMalloc(&L.bigArena, (uint64_t)a->gridBig * a->arenaElems * sizeof(Elem512))) != hipSuccess)
            return fail("big arena", e);
    }
    int perCU256 = 0;   // passes 2 and 3 (deferred reads) reuse the arenas of the first a->grid blocks
    hipOccupancyMaxActiveBlocksPerMultiprocessor(&perCU256, (const void *)align_kernel<256, false>, 64, 0);
    if (perCU256 <= 0) perCU256 = 4;
    a->grid256 = prop.multiProcessorCount * perCU256;
    if (a->grid256 > a->grid) a->grid256 = a->grid;
    int perCU512 = 0;
    hipOccupancyMaxActiveBlocksPerMultiprocessor(&perCU512, (const void *)align_kernel<512, false>, 64, 0);
    if (perCU512 <= 0) perCU512 = 4;
    a->grid512 = prop.multiProcessorCount * perCU512;
    if (a->grid512 > a->grid) a->grid512 = a->grid;
    if (const char *t = getenv("SNAPGPU_PHASES"); t && atoi(t)) {
        const size_t pb = (size_t)a->grid * PH_SLOTS * sizeof(unsigned long long);
        if ((e = hipMalloc(&a->dPhase, pb)) != hipSuccess) return fail("phase buffer", e);
        if ((e = hipMemsetAsync(a->dPhase, 0, pb, s0)) != hipSuccess) return fail("phase buffer", e);
    }
    if ((e = hipDeviceSynchronize()) != hipSuccess) return fail("sync", e);
    return a;
}

snapgpu_device_reads_t *snapgpu_reads_upload(snapgpu_aligner_t *a, const snapgpu_reads_t *r) {
    if (!a || !r) { snapgpu::setError("reads_upload: null"); return nullptr; }
    if (a->failed) { snapgpu::setError("aligner failed earlier (device timeout)"); return nullptr; }
    HIPCHKN(hipSetDevice(a->device));
    auto *d = new snapgpu_device_reads_t();
    d->owner = a;
    d->n = r->n;
    d->device = a->device;
    const_cast<snapgpu_reads_t *>(r)->nUploads++;   // clipping is refused from now on
    uint64_t bytes = 0;
    for (uint64_t i = 0; i < r->n; i++) {
        uint64_t endb = r->offsets[i] + r->lengths[i];
        if (endb > bytes) bytes = endb;
        if (r->lengths[i] > d->maxLen) d->maxLen = r->lengths[i];
    }
    bytes += 64;
    hipStream_t s = a->stream();
    HIPCHKN(hipMalloc(&d->dBases, bytes));
    HIPCHKN(hipMalloc(&d->dQuals, bytes));
    HIPCHKN(hipMalloc(&d->dOffsets, (r->n + 1) * 8));
    HIPCHKN(hipMalloc(&d->dLengths, (r->n + 1) * 4));
    HIPCHKN(hipMalloc(&d->dOut, (r->n + 1) * sizeof(snapgpu_result_t)));
    HIPCHKN(hipMalloc(&d->dDefer, 3 * (r->n + 1) * sizeof(uint32_t)));   // pass-1 / pass-2 defers, arena overflows
    HIPCHKN(hipMalloc(&d->dSeeds, (r->n + 8) * SEEDS_PER_READ * sizeof(SeedRec)));
    HIPCHKN(hipMemsetAsync(d->dBases, 0, bytes, s));
    HIPCHKN(hipMemsetAsync(d->dQuals, 0, bytes, s));
    HIPCHKN(hipMemcpyAsync(d->dBases, r->bases, bytes - 64, hipMemcpyHostToDevice, s));
    HIPCHKN(hipMemcpyAsync(d->dQuals, r->quals, bytes - 64, hipMemcpyHostToDevice, s));
    HIPCHKN(hipMemcpyAsync(d->dOffsets, r->offsets, r->n * 8, hipMemcpyHostToDevice, s));
    HIPCHKN(hipMemcpyAsync(d->dLengths, r->lengths, r->n * 4, hipMemcpyHostToDevice, s));
    HIPCHKN(hipStreamSynchronize(s));
    return d;
}

void snapgpu_device_reads_free(snapgpu_device_reads_t *d) {
    if (!d) return;
    const snapgpu_aligner_t *a = d->owner;
    if (!(a && a->failed)) hipSetDevice(d->device);
    devFree(a, d->dBases); devFree(a, d->dQuals); devFree(a, d->dOffsets); devFree(a, d->dLengths);
    devFree(a, d->dOut); devFree(a, d->dDefer); devFree(a, d->dSeeds);
    devFree(a, d->dCigEd); devFree(a, d->dCigN); devFree(a, d->dCigOps);
    delete d;
}

// u32 words per block of the multi-hit scratch: hitCount[MAX_K], then {loc, dir} pairs at flat
// index score * hitSlot + count (record_hit), count < maxHitsToGet
static inline uint64_t multiHitStride(uint32_t maxHitsToGet) {
    const uint64_t slot = maxHitsToGet < 512 ? maxHitsToGet : 512;
    return (uint64_t)MAX_K + 2 * ((uint64_t)MAX_K * slot + (maxHitsToGet > 512 ? maxHitsToGet : 0));
}

// Extension arguments of snapgpu_align_batch_ex (device pointers; all null for the plain path)
struct AlignExt {
    const snapgpu_search_t *search = nullptr;
    uint32_t maxHitsToGet = 0;
    uint32_t *hitScratch = nullptr;
    int32_t *multiFound = nullptr;
    snapgpu_multi_hit_t *multiHits = nullptr;
};

// The device buffers one pass set reads and writes.
struct PassIO {
    const char *bases, *quals;
    const uint64_t *offsets;
    const uint32_t *lengths;
    uint64_t n;
    snapgpu_result_t *out;
    uint32_t *defer;    // pass 1 -> pass 2 read list
    uint32_t *defer2;   // pass 2 -> pass 3 read list
    uint32_t *ovf;      // passes 1-3 -> big-arena pass (reads that outgrew a capped arena)
    SeedRec *seeds;
    uint32_t maxLen;    // longest read (or a bound): no long reads, no order_long_kernel
};

// Queue pass 0 (seed lookups), pass 1 (align_kernel<128>), pass 2 (align_kernel<256> over the
// reads pass 1 deferred: 129..256 bases, bit planes) and pass 3 (align_kernel<512> over what
// pass 2 deferred: longer reads and IUPAC-on-both-sides reads, byte compare) on lane `li`, with
// HIP events around them.  The deferred counts stay on the device (each pass reads its list
// length from the counter the previous one appended with).
static int launch_passes(snapgpu_aligner_t *a, int li, const PassIO &io, const AlignExt &x, EvSet &ev,
                         const EvSet *prev) {
    ExecLane &L = a->lane[li];
    if (io.n == 0) return SNAPGPU_OK;
    if (io.n > 0xffffffffull) { snapgpu::setError("batch too large"); return SNAPGPU_EINVAL; }
    KArgs A;
    memset(&A, 0, sizeof(A));
    const snapgpu_index_t *idx = a->idx;
    A.buckets = a->dBuckets; A.bucketBase = a->dBucketBase; A.bucketCount = a->dBucketCount; A.overflow = a->dOverflow;
    A.genome = a->dGenome; A.pieces = a->dPieces; A.nPieces = (int32_t)idx->genome->pieceOffsets.size();
    A.gpl = a->dGPlanes; A.hasIupac = idx->hasIupac ? 1u : 0u;
    A.phaseBuf = a->dPhase;
    A.diag = a->dDiag;
    A.nBases = idx->genome->nBases; A.seedLen = idx->seedLen; A.nTables = idx->nTables;
    A.padding = idx->genome->chromosomePadding;
    A.maxHits = a->p.maxHitsToConsider; A.maxK = a->p.maxK; A.maxReadSize = a->p.maxReadSize;
    A.maxSeedsCmd = a->p.maxSeedsToUse; A.seedCoverage = a->p.maxSeedCoverage; A.extra = a->p.extraSearchDepth;
    A.explore = a->p.explorePopularSeeds; A.stopOnFirst = a->p.stopOnFirstHit; A.kRows = 31;
    A.radixMin = a->radixMin;
    A.tripRead = a->tripRead;
    A.tab = a->dTab;
    A.bases = io.bases; A.quals = io.quals; A.offsets = io.offsets; A.lengths = io.lengths;
    A.nReads = (uint32_t)io.n; A.out = io.out;
    A.counter = L.counter; A.arena = L.arena; A.arenaElems = a->arenaCap;
    if (a->arenaCap < a->arenaElems) { A.ovfList = io.ovf; A.ovfCount = L.counter + 6; }
    A.deferList = io.defer; A.deferCount = L.counter + 2; A.readList = nullptr;
    A.search = x.search; A.maxHitsToGet = x.maxHitsToGet;
    A.hitSlot = x.maxHitsToGet < 512 ? x.maxHitsToGet : 512;
    A.hitStride = multiHitStride(x.maxHitsToGet);
    A.hitScratch = x.hitScratch; A.multiFound = x.multiFound; A.multiHits = x.multiHits;
    int grid = a->grid;
    if ((uint64_t)grid > io.n) grid = (int)io.n;
    (void)hipGetLastError();   // clear any stale error of an unrelated earlier runtime call
    if (prev && !a->overlapKernels) HIPCHK(hipStreamWaitEvent(L.stream, prev->e[2], 0));
    HIPCHK(hipMemsetAsync(L.counter, 0, 64, L.stream));
    // every record pre-filled with 0xff (result 0xff is no AlignmentResult): a read that no pass
    // writes -- lost in the routing between passes -- fails the call on the host (finishChunk /
    // finishRecords) instead of coming back as a stale or zeroed NotFound-looking record
    HIPCHK(hipMemsetAsync(io.out, 0xff, io.n * sizeof(snapgpu_result_t), L.stream));
    // pass 0: the first SEEDS_PER_READ seed lookups of every read (4 reads per 64-lane block); it also puts the
    // reads longer than 128 bases straight onto pass 2's list
    A.seedRecs = nullptr;
    A.longCount = L.counter + 5;
    // longest-first: the long reads' order list is pass 2's defer list (free until pass 2 writes it)
    A.orderTmp = a->orderLong && io.n < (1ull << 28) ? io.defer2 : nullptr;
    HIPCHK(hipEventRecord(ev.e[3], L.stream));
    hipLaunchKernelGGL(seed_lookup_kernel, dim3((unsigned)((io.n + 4 * LOOKUP_WAVES - 1) / (4 * LOOKUP_WAVES))),
                       dim3(64 * LOOKUP_WAVES), 0, L.stream, A, io.seeds,
                       L.lookupStats);
    HIPCHK(hipGetLastError());
    if (A.orderTmp && io.maxLen > 128) {
        hipLaunchKernelGGL(order_long_kernel, dim3(1), dim3(256), 0, L.stream, A.orderTmp, A.longCount, A.deferList);
        HIPCHK(hipGetLastError());
    }
    A.orderTmp = nullptr;
    A.seedRecs = reinterpret_cast<const uint4 *>(io.seeds);
    HIPCHK(hipEventRecord(ev.e[0], L.stream));
    const bool ext = x.search || x.maxHitsToGet;
    if (ext) hipLaunchKernelGGL((align_kernel<128, true>), dim3(grid), dim3(64), 0, L.stream, A);
    else hipLaunchKernelGGL((align_kernel<128, false>), dim3(grid), dim3(64), 0, L.stream, A);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(ev.e[1], L.stream));
    // pass 2: reads of 129..256 bases (bit planes, 256-bit masks)
    KArgs M = A;
    M.counter = L.counter + 3;
    M.readList = io.defer; M.readCount = L.counter + 2;
    M.deferList = io.defer2; M.deferCount = L.counter + 4;   // (M.seedRecs: pass 0's records, long reads too)
    int grid256 = a->grid256;
    if ((uint64_t)grid256 > io.n) grid256 = (int)io.n;
    if (ext) hipLaunchKernelGGL((align_kernel<256, true>), dim3(grid256), dim3(64), 0, L.stream, M);
    else hipLaunchKernelGGL((align_kernel<256, false>), dim3(grid256), dim3(64), 0, L.stream, M);
    HIPCHK(hipGetLastError());
    // pass 3: reads longer than 256 bases or needing the byte-compare LV
    KArgs B = A;
    B.counter = L.counter + 1;
    B.readList = io.defer2; B.readCount = L.counter + 4;
    B.deferList = nullptr; B.deferCount = nullptr;
    B.seedRecs = nullptr;
    int grid2 = a->grid512;
    if ((uint64_t)grid2 > io.n) grid2 = (int)io.n;
    if (ext) hipLaunchKernelGGL((align_kernel<512, true>), dim3(grid2), dim3(64), 0, L.stream, B);
    else hipLaunchKernelGGL((align_kernel<512, false>), dim3(grid2), dim3(64), 0, L.stream, B);
    HIPCHK(hipGetLastError());
    if (a->gridBig) {
        // big-arena pass: the reads passes 1-3 abandoned when they outgrew a capped arena, aligned
        // from scratch by the byte-compare kernel (any read length) on worst-case arenas
        KArgs V = A;
        V.counter = L.counter + 7;
        V.readList = io.ovf; V.readCount = L.counter + 6;
        V.deferList = nullptr; V.deferCount = nullptr;
        V.ovfList = nullptr; V.ovfCount = nullptr;
        V.seedRecs = nullptr;
        V.arena = L.bigArena; V.arenaElems = a->arenaElems;
        int gridV = a->gridBig;
        if ((uint64_t)gridV > io.n) gridV = (int)io.n;
        if (ext) hipLaunchKernelGGL((align_kernel<512, true>), dim3(gridV), dim3(64), 0, L.stream, V);
        else hipLaunchKernelGGL((align_kernel<512, false>), dim3(gridV), dim3(64), 0, L.stream, V);
        HIPCHK(hipGetLastError());
    }
    HIPCHK(hipEventRecord(ev.e[2], L.stream));
    HIPCHK(hipMemcpyAsync(ev.hCounter, L.counter, 32, hipMemcpyDeviceToHost, L.stream));
    return SNAPGPU_OK;
}

// The event set of the next pass set of the current call (created on first use).
static EvSet *nextEvSet(snapgpu_aligner_t *a) {
    if (a->nEvUsed == a->evs.size()) {
        EvSet v;
        for (auto &e : v.e)
            if (hipEventCreate(&e) != hipSuccess) { snapgpu::setError("hipEventCreate"); return nullptr; }
        if (hipHostMalloc(&v.hCounter, 64, hipHostMallocDefault) != hipSuccess) { snapgpu::setError("pinned counter"); return nullptr; }
        a->evs.push_back(v);
    }
    return &a->evs[a->nEvUsed++];
}

// Start of a call: lookup statistics accumulate over all its pass sets.
static int beginCall(snapgpu_aligner_t *a) {
    a->nEvUsed = 0;
    a->timing = snapgpu_timing_t{};
    for (auto &L : a->lane) HIPCHK(hipMemsetAsync(L.lookupStats, 0, 1024 * sizeof(unsigned long long), L.stream));
    HIPCHK(hipMemsetAsync(a->dDiag, 0, sizeof(uint32_t) * 4, a->lane[0].stream));
    // the other lane's first kernels must not start before the watchdog record is cleared
    HIPCHK(hipStreamSynchronize(a->lane[0].stream));
    return SNAPGPU_OK;
}

// Union of the [e[from], e[to]] intervals of the call's pass sets (they overlap across lanes), ms.
static double busyUnion(snapgpu_aligner_t *a, int from, int to) {
    std::vector<std::pair<float, float>> iv;
    const hipEvent_t ref = a->evs[0].e[3];
    for (uint64_t i = 0; i < a->nEvUsed; i++) {
        float b = 0, e = 0;
        if (hipEventElapsedTime(&b, ref, a->evs[i].e[from]) != hipSuccess ||
            hipEventElapsedTime(&e, ref, a->evs[i].e[to]) != hipSuccess) return -1;
        iv.emplace_back(b, e);
    }
    std::sort(iv.begin(), iv.end());
    double total = 0, cs = -1e30, ce = -1e30;
    for (auto &x : iv) {
        if (x.first > ce) { if (ce > cs) total += ce - cs; cs = x.first; ce = x.second; }
        else if (x.second > ce) ce = x.second;
    }
    if (ce > cs) total += ce - cs;
    return total;
}

static void accountBusy(snapgpu_aligner_t *a) {
    if (a->nEvUsed == 0) return;
    a->timing.mainKernelBusyMs = busyUnion(a, 0, 1);
    a->timing.lookupKernelBusyMs = busyUnion(a, 3, 0);
}

// Kernel times and counters of one finished pass set into a->timing.
static int accountEvSet(snapgpu_aligner_t *a, const EvSet &v) {
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, v.e[0], v.e[1]));
    a->timing.mainKernelMs += ms;
    HIPCHK(hipEventElapsedTime(&ms, v.e[1], v.e[2]));
    a->timing.spillKernelMs += ms;
    HIPCHK(hipEventElapsedTime(&ms, v.e[3], v.e[0]));
    a->timing.lookupKernelMs += ms;
    a->timing.nLaunches++;
    a->timing.nSpilled += v.hCounter[2];
    a->timing.nByteReads += v.hCounter[4];
    a->timing.nArenaOverflow += v.hCounter[6];
    return SNAPGPU_OK;
}

// Device-resident reads: the same chunk-sized pass sets as snapgpu_align_batch, alternating
// over the two lanes, on sub-ranges of the resident buffers (no copies).  The extended path
// (windowed search / multi-hit scratch per block) runs as one pass set on lane 0.
int snapgpu_align_batch_wait(snapgpu_aligner_t *a);

static int launch_resident(snapgpu_aligner_t *a, snapgpu_device_reads_t *d, const AlignExt &x) {
    if (!a || !d) return SNAPGPU_EINVAL;
    if (a->failed) { snapgpu::setError("aligner failed earlier (device timeout)"); return SNAPGPU_EDEVICE; }
    HIPCHK(hipSetDevice(a->device));
    int rc = snapgpu_align_batch_wait(a);   // no submitted batch may still use the lanes
    if (rc) return rc;
    rc = beginCall(a);
    if (rc) return rc;
    if (a->residentSidePending) {   // a CIGAR call may still read resident records on the side stream
        for (auto &L : a->lane) HIPCHK(hipStreamWaitEvent(L.stream, a->residentSideDone, 0));
        a->residentSidePending = false;
    }
    const bool ext = x.search || x.maxHitsToGet;
    const uint64_t n = d->n;
    const uint64_t nChunks = ext || n == 0 ? 1 : (n + a->residentChunk - 1) / a->residentChunk;
    const uint64_t per = (n + nChunks - 1) / nChunks;
    for (uint64_t c = 0; c < nChunks; c++) {
        const uint64_t b = c * per, m = std::min(n, b + per) - b;
        EvSet *ev = nextEvSet(a);
        if (!ev) return SNAPGPU_EDEVICE;
        PassIO io{d->dBases, d->dQuals, d->dOffsets + b, d->dLengths + b, m, d->dOut + b, d->dDefer + b,
                  d->dDefer + (n + 1) + b, d->dDefer + 2 * (n + 1) + b, d->dSeeds + b * SEEDS_PER_READ, d->maxLen};
        if ((rc = launch_passes(a, (int)(c & 1), io, x, *ev, c ? &a->evs[a->nEvUsed - 2] : nullptr))) return rc;
    }
    a->lastReads = d;
    a->pendingTiming = n > 0;
    return SNAPGPU_OK;
}

int snapgpu_align_resident(snapgpu_aligner_t *a, snapgpu_device_reads_t *d) { return launch_resident(a, d, AlignExt()); }

// sum of the per-slot lookup statistics of a lane (host copy)
static void addLookupStats(snapgpu_timing_t &t, const unsigned long long *ls) {
    for (int i = 0; i < 256; i++) {
        t.lookupSeeds += ls[4 * i];
        t.lookupProbes += ls[4 * i + 1];
        t.lookupOverflowReads += ls[4 * i + 2];
    }
}

static int checkWatchdog(snapgpu_aligner_t *a) {
    uint32_t diag[4];
    HIPCHK(hipMemcpy(diag, a->dDiag, sizeof(diag), hipMemcpyDeviceToHost));
    if (diag[0]) {
        char msg[160];
        snprintf(msg, sizeof msg, "device watchdog tripped: code %u read %u detail %u", diag[0], diag[1], diag[2]);
        snapgpu::setError(msg);
        return SNAPGPU_EDEVICE;
    }
    return SNAPGPU_OK;
}

int snapgpu_synchronize(snapgpu_aligner_t *a) {
    if (!a) return SNAPGPU_EINVAL;
    if (a->failed) { snapgpu::setError("aligner failed earlier (device timeout)"); return SNAPGPU_EDEVICE; }
    HIPCHK(hipSetDevice(a->device));
    for (auto &L : a->lane) {
        const int rc = waitLane(a, L);
        if (rc) return rc;
    }
    if (a->pendingTiming) {
        a->timing = snapgpu_timing_t{};
        for (uint64_t i = 0; i < a->nEvUsed; i++) {
            const int rc = accountEvSet(a, a->evs[i]);
            if (rc) return rc;
        }
        accountBusy(a);
        std::vector<unsigned long long> ls(1024);
        for (auto &L : a->lane) {
            HIPCHK(hipMemcpy(ls.data(), L.lookupStats, 1024 * sizeof(unsigned long long), hipMemcpyDeviceToHost));
            addLookupStats(a->timing, ls.data());
        }
        a->pendingTiming = false;
        const int rc = checkWatchdog(a);
        if (rc) return rc;
    }
    return SNAPGPU_OK;
}

// Records -> caller: MAPQ fix-ups (ratio within 1e-9 of a threshold 10^(-q/10), mapq_dev,
// re-derived with glibc log10) and the aligner statistics, over out[0, n).
// A record whose result byte is still the 0xff pre-fill was written by no pass: the call fails.
static int checkRecords(snapgpu_aligner_t *a, uint64_t unwritten, uint64_t firstUnwritten) {
    a->timing.nUnwritten += unwritten;
    if (!unwritten) return SNAPGPU_OK;
    // a tripped watchdog drains the kernels (its reads stay unwritten): report it as such
    if (int rc = checkWatchdog(a)) return rc;
    snapgpu::setError("align: " + std::to_string(unwritten) + " read record(s) written by no pass (first: read " +
                      std::to_string(firstUnwritten) + " of the call); results are not valid");
    return SNAPGPU_EDEVICE;
}

static int finishRecords(snapgpu_aligner_t *a, snapgpu_result_t *out, uint64_t n) {
    uint64_t fixed = 0, nul = 0, unwritten = 0, first = 0;
    for (uint64_t i = 0; i < n; i++) {
        snapgpu_result_t &o = out[i];
        if (o.result > SNAPGPU_UNKNOWN) { if (!unwritten++) first = i; continue; }
        nul += (o.flags & SNAPGPU_FLAG_NUL_BYTE) ? 1 : 0;
        if (o.flags & SNAPGPU_FLAG_MAPQ_FIXED) {
            o.mapq = hostMapq(o.probabilityOfAllCandidates, o.probabilityOfBestCandidate, o.score, o.popularSeedsSkipped);
            o.result = o.mapq >= 10 ? SNAPGPU_SINGLE_HIT : SNAPGPU_MULTIPLE_HITS;
            fixed++;
        }
        a->stats.nHashTableLookups += o.nLookups;
        a->stats.nLocationsScored += o.nLocationsScored;
        a->stats.nHitsIgnoredBecauseOfTooHighPopularity += o.nHitsIgnored;
        a->stats.nReadsIgnoredBecauseOfTooManyNs += (o.flags & SNAPGPU_FLAG_TOO_MANY_NS) ? 1 : 0;
        a->stats.nReads++;
    }
    a->timing.nMapqFixed += fixed;
    a->timing.nNulReads += nul;
    return checkRecords(a, unwritten, first);
}

int snapgpu_results_download(snapgpu_aligner_t *a, snapgpu_device_reads_t *d, snapgpu_result_t *out) {
    if (!a || !d || !out) return SNAPGPU_EINVAL;
    HIPCHK(hipSetDevice(a->device));
    int rc = snapgpu_synchronize(a);   // before the copy: a pageable-destination copy blocks
    if (rc) return rc;
    HIPCHK(hipMemcpyAsync(out, d->dOut, d->n * sizeof(snapgpu_result_t), hipMemcpyDeviceToHost, a->stream()));
    HIPCHK(hipStreamSynchronize(a->stream()));
    auto t0 = std::chrono::steady_clock::now();
    a->timing.nMapqFixed = 0;
    a->timing.nNulReads = 0;
    a->timing.nUnwritten = 0;
    rc = finishRecords(a, out, d->n);
    a->timing.fixupMs = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return rc;
}

// (Re)allocate a lane's chunk buffers for `reads` reads spanning `bytes` read bytes.
static int ensureLaneCapacity(snapgpu_aligner_t *a, ExecLane &L, uint64_t reads, uint64_t bytes) {
    if (reads <= L.capReads && bytes <= L.capBytes) return SNAPGPU_OK;
    int rc = waitLane(a, L);
    if (rc) return rc;
    freeLaneChunkBuffers(a, L);
    reads = std::max<uint64_t>(reads, 1024);
    const uint64_t cb = bytes + 512;   // zero slack past the last read: over-reading loads stay inside
    for (ChunkSlot &S : L.slot) {
        HIPCHK(hipMalloc(&S.dBases, cb));
        HIPCHK(hipMalloc(&S.dQuals, cb));
        // zeroed on the copy stream, ahead of the uploads into them: a plain hipMemset runs on the
        // null stream, which the non-blocking copy stream does not wait for
        HIPCHK(hipMemsetAsync(S.dBases, 0, cb, a->copyStream));
        HIPCHK(hipMemsetAsync(S.dQuals, 0, cb, a->copyStream));
        HIPCHK(hipMalloc(&S.dOffsets, (reads + 1) * 8));
        HIPCHK(hipMalloc(&S.dLengths, (reads + 1) * 4));
        HIPCHK(hipHostMalloc(&S.hOffsets, (reads + 1) * 8, hipHostMallocDefault));
        HIPCHK(hipHostMalloc(&S.hLengths, (reads + 1) * 4, hipHostMallocDefault));
        HIPCHK(hipHostMalloc(&S.hOut, (reads + 1) * sizeof(snapgpu_result_t), hipHostMallocDefault));
    }
    HIPCHK(hipMalloc(&L.dDefer, 3 * (reads + 1) * 4));   // pass-1 / pass-2 defers, arena overflows
    HIPCHK(hipMalloc(&L.dOut, (reads + 1) * sizeof(snapgpu_result_t)));
    HIPCHK(hipMalloc(&L.dSeeds, (reads + 8) * SEEDS_PER_READ * sizeof(SeedRec)));
    L.capReads = reads;
    L.capBytes = bytes;
    return SNAPGPU_OK;
}

// The host tail of one chunk: wait for its records, account its kernel times, then MAPQ
// fix-ups, statistics and the copy into the caller's array (host threads, while the GPU
// already runs the next chunks).
static int finishChunk(snapgpu_aligner_t *a, ChunkSlot &L) {
    if (!L.pending) return SNAPGPU_OK;
    snapgpu_result_t *out = L.chunkOut;
    L.pending = false;
    int rc = waitEvent(a, L.done);
    if (rc) return rc;
    if ((rc = accountEvSet(a, a->evs[L.chunkEv]))) return rc;
    const auto t0 = std::chrono::steady_clock::now();
    const uint64_t n = L.chunkN;
    snapgpu_result_t *dst = out + L.chunkBegin;
    const unsigned nt = n >= 65536 ? snapgpu::hostThreads(4) : 1u;
    std::vector<snapgpu_aligner_stats_t> st(nt, snapgpu_aligner_stats_t{});
    std::vector<uint64_t> fixed(nt, 0), nul(nt, 0), unwritten(nt, 0), first(nt, 0);
    // per-thread sums in locals, stored once: the threads' slots of st / fixed / nul share cache
    // lines, and updating them per record made the lines bounce between cores -- 7.6-11.6 ms per
    // 1M-record chunk on the MI355X host, 1.3-1.5 ms without (the copy alone is ~0.9 ms,
    // tools/probe/pinned_read.cpp; profiles/r05/ab/host_tail_fs_r05t2.txt).  The last chunk's tail
    // is paid after the GPU is done, once per stream.
    auto work = [&](unsigned t) {
        const uint64_t b = n * t / nt, e = n * (t + 1) / nt;
        memcpy(dst + b, L.hOut + b, (e - b) * sizeof(snapgpu_result_t));
        uint64_t lk = 0, sc = 0, ig = 0, tm = 0, fx = 0, nu = 0, uw = 0, f0 = 0;
        for (uint64_t i = b; i < e; i++) {
            snapgpu_result_t &o = dst[i];
            if (o.result > SNAPGPU_UNKNOWN) { if (!uw++) f0 = L.chunkBegin + i; continue; }
            nu += (o.flags & SNAPGPU_FLAG_NUL_BYTE) ? 1 : 0;
            if (o.flags & SNAPGPU_FLAG_MAPQ_FIXED) {
                o.mapq = hostMapq(o.probabilityOfAllCandidates, o.probabilityOfBestCandidate, o.score, o.popularSeedsSkipped);
                o.result = o.mapq >= 10 ? SNAPGPU_SINGLE_HIT : SNAPGPU_MULTIPLE_HITS;
                fx++;
            }
            lk += o.nLookups;
            sc += o.nLocationsScored;
            ig += o.nHitsIgnored;
            tm += (o.flags & SNAPGPU_FLAG_TOO_MANY_NS) ? 1 : 0;
        }
        st[t].nHashTableLookups = lk;
        st[t].nLocationsScored = sc;
        st[t].nHitsIgnoredBecauseOfTooHighPopularity = ig;
        st[t].nReadsIgnoredBecauseOfTooManyNs = tm;
        fixed[t] = fx;
        nul[t] = nu;
        unwritten[t] = uw;
        first[t] = f0;
    };
    if (nt == 1) work(0);
    else {
        std::vector<std::thread> th;
        for (unsigned t = 0; t < nt; t++) th.emplace_back(work, t);
        for (auto &x : th) x.join();
    }
    for (unsigned t = 0; t < nt; t++) {
        a->stats.nHashTableLookups += st[t].nHashTableLookups;
        a->stats.nLocationsScored += st[t].nLocationsScored;
        a->stats.nHitsIgnoredBecauseOfTooHighPopularity += st[t].nHitsIgnoredBecauseOfTooHighPopularity;
        a->stats.nReadsIgnoredBecauseOfTooManyNs += st[t].nReadsIgnoredBecauseOfTooManyNs;
        a->timing.nMapqFixed += fixed[t];
        a->timing.nNulReads += nul[t];
    }
    a->stats.nReads += n;
    a->timing.fixupMs += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    uint64_t uw = 0, f0 = 0;
    for (unsigned t = 0; t < nt; t++) { if (unwritten[t] && !uw) f0 = first[t]; uw += unwritten[t]; }
    return checkRecords(a, uw, f0);
}

// The host tail of the oldest pipelined chunk still pending (any lane); false if none.
static int finishOldest(snapgpu_aligner_t *a, bool *any) {
    ChunkSlot *o = nullptr;
    for (auto &L : a->lane)
        for (ChunkSlot &S : L.slot)
            if (S.pending && (!o || S.seq < o->seq)) o = &S;
    *any = o != nullptr;
    return o ? finishChunk(a, *o) : SNAPGPU_OK;
}

static int finishAll(snapgpu_aligner_t *a) {
    for (bool any = true; any;) {
        const int rc = finishOldest(a, &any);
        if (rc) return rc;
    }
    return SNAPGPU_OK;
}

// After an error: nothing may stay in flight on the chunk buffers (unless a timeout made that impossible).
static void abandonChunks(snapgpu_aligner_t *a) {
    for (auto &L : a->lane) {
        for (ChunkSlot &S : L.slot) S.pending = false;
        if (!a->failed) waitLane(a, L);
    }
    if (!a->failed && a->copyStream) (void)hipStreamSynchronize(a->copyStream);
    a->streamOpen = false;
}

// Batched BaseAligner::AlignRead over host buffers (SURVEY.md 8(d) d1 boundary): the reads are
// cut into chunks that alternate over the two execution lanes -- H2D of the chunk's bytes,
// offsets and lengths, the three passes, D2H of its records into pinned staging -- and the
// host tail of chunk c-2 runs while chunks c-1 and c are on the GPU.  Submitting returns with
// the last two chunks in flight; the next submit continues the same pipeline (its first chunks
// overlap this batch's last kernels) and snapgpu_align_batch_wait drains it.
int snapgpu_align_batch_submit(snapgpu_aligner_t *a, const snapgpu_reads_t *reads, snapgpu_result_t *out) {
    if (!a || !reads || !out) return SNAPGPU_EINVAL;
    if (a->failed) { snapgpu::setError("aligner failed earlier (device timeout)"); return SNAPGPU_EDEVICE; }
    HIPCHK(hipSetDevice(a->device));
    int rc = SNAPGPU_OK;
    if (!a->streamOpen) {
        if (a->pendingTiming && (rc = snapgpu_synchronize(a))) return rc;   // a resident run still queued
        if ((rc = beginCall(a))) return rc;
        a->streamOpen = true;
        a->streamStart = std::chrono::steady_clock::now();
    }
    const uint64_t n = reads->n;
    if (n == 0) return SNAPGPU_OK;
    const uint64_t nChunks = (n + a->chunkReads - 1) / a->chunkReads;
    const uint64_t per = (n + nChunks - 1) / nChunks;
    // byte span of every chunk (reads are normally contiguous; any layout is accepted)
    std::vector<uint64_t> lo(nChunks, ~0ull), hi(nChunks, 0);
    uint64_t maxSpan = 0;
    for (uint64_t c = 0; c < nChunks; c++) {
        for (uint64_t i = c * per; i < std::min(n, (c + 1) * per); i++) {
            lo[c] = std::min(lo[c], reads->offsets[i]);
            hi[c] = std::max(hi[c], reads->offsets[i] + reads->lengths[i]);
        }
        if (hi[c] < lo[c]) lo[c] = hi[c] = 0;
        maxSpan = std::max(maxSpan, hi[c] - lo[c]);
    }
    const uint64_t hostEnd = reads->totalBytes + 64;   // allocated and zeroed past the last read
    bool grow = false;
    for (auto &L : a->lane) grow |= std::min(per, n) > L.capReads || maxSpan + 64 > L.capBytes;
    if (grow) {   // every pending chunk first (their buffers are reallocated)
        if ((rc = finishAll(a))) { abandonChunks(a); return rc; }
        for (auto &L : a->lane)
            if ((rc = ensureLaneCapacity(a, L, std::min(per, n), maxSpan + 64))) { abandonChunks(a); return rc; }
    }
    for (uint64_t c = 0; c < nChunks && rc == SNAPGPU_OK; c++) {
        const int li = (int)(a->nextLane++ & 1);
        ExecLane &L = a->lane[li];
        ChunkSlot &S = L.slot[L.nextSlot];
        L.nextSlot ^= 1u;
        // the chunk that last used this slot (4 chunks back) is finished first, oldest first
        for (bool any = true; S.pending && any;)
            if ((rc = finishOldest(a, &any))) break;
        if (rc) break;
        const uint64_t b = c * per, m = std::min(n, b + per) - b;
        uint32_t maxLen = 0;
        for (uint64_t i = 0; i < m; i++) {
            S.hOffsets[i] = reads->offsets[b + i] - lo[c];
            const uint32_t ln = reads->lengths[b + i];
            S.hLengths[i] = ln;
            maxLen = std::max(maxLen, ln);
        }
        const uint64_t span = std::min(hi[c] + 64, std::max(hostEnd, hi[c])) - lo[c];
        // inputs on the copy stream: they land while the lane's previous chunk is still running
        hipStream_t cs = a->copyStream, s = L.stream;
        HIPBRK(hipMemcpyAsync(S.dBases, reads->bases + lo[c], span, hipMemcpyHostToDevice, cs));
        HIPBRK(hipMemcpyAsync(S.dQuals, reads->quals + lo[c], span, hipMemcpyHostToDevice, cs));
        HIPBRK(hipMemcpyAsync(S.dOffsets, S.hOffsets, m * 8, hipMemcpyHostToDevice, cs));
        HIPBRK(hipMemcpyAsync(S.dLengths, S.hLengths, m * 4, hipMemcpyHostToDevice, cs));
        HIPBRK(hipEventRecord(S.h2d, cs));
        HIPBRK(hipStreamWaitEvent(s, S.h2d, 0));
        PassIO io{S.dBases, S.dQuals, S.dOffsets, S.dLengths, m, L.dOut, L.dDefer, L.dDefer + (L.capReads + 1),
                  L.dDefer + 2 * (L.capReads + 1), L.dSeeds, maxLen};
        EvSet *ev = nextEvSet(a);
        if (!ev) { rc = SNAPGPU_EDEVICE; break; }
        if ((rc = launch_passes(a, li, io, AlignExt(), *ev, a->nEvUsed >= 2 ? &a->evs[a->nEvUsed - 2] : nullptr))) break;
        HIPBRK(hipMemcpyAsync(S.hOut, L.dOut, m * sizeof(snapgpu_result_t), hipMemcpyDeviceToHost, s));
        HIPBRK(hipEventRecord(S.done, s));
        S.pending = true;
        S.seq = a->chunkSeq++;
        S.chunkBegin = b;
        S.chunkN = m;
        S.chunkEv = a->nEvUsed - 1;
        S.chunkOut = out;
    }
    if (rc) abandonChunks(a);
    return rc;
}

int snapgpu_align_batch_wait(snapgpu_aligner_t *a) {
    if (!a) return SNAPGPU_EINVAL;
    if (!a->streamOpen) return a->failed ? SNAPGPU_EDEVICE : SNAPGPU_OK;
    HIPCHK(hipSetDevice(a->device));
    int rc = finishAll(a);   // oldest first
    a->streamOpen = false;
    if (rc) {
        abandonChunks(a);
        return rc;
    }
    accountBusy(a);
    for (auto &L : a->lane) {   // lookup statistics of the whole stream
        HIPCHK(hipMemcpy(L.hLookupStats, L.lookupStats, 1024 * sizeof(unsigned long long), hipMemcpyDeviceToHost));
        addLookupStats(a->timing, L.hLookupStats);
    }
    rc = checkWatchdog(a);
    a->lastReads = nullptr;
    a->pendingTiming = false;
    a->timing.wallMs = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a->streamStart).count();
    return rc;
}

int snapgpu_align_batch(snapgpu_aligner_t *a, const snapgpu_reads_t *reads, snapgpu_result_t *out) {
    if (!a || !reads || !out) return SNAPGPU_EINVAL;
    int rc = snapgpu_align_batch_wait(a);   // a stream the caller left open
    if (rc) return rc;
    if ((rc = snapgpu_align_batch_submit(a, reads, out))) return rc;
    return snapgpu_align_batch_wait(a);
}

// The reads of a snapgpu_internal_align_batch_packed call in the aligner's own grow-only device
// reads (what snapgpu_reads_upload allocates per call), uploaded on the aligner's stream.  Several
// batches (the RNA path's two ends) go into one device batch, back to back: part p's reads follow
// part p-1's, their offsets moved past its bytes.
static snapgpu_device_reads_t *uploadCachedReads(snapgpu_aligner_t *a, const snapgpu_reads_t *const *parts, int np) {
    uint64_t n = 0, bytes = 0;
    uint32_t maxLen = 0;
    std::vector<uint64_t> span(np), base(np);
    for (int p = 0; p < np; p++) {
        const snapgpu_reads_t *r = parts[p];
        uint64_t b = 0;
        for (uint64_t i = 0; i < r->n; i++) {
            b = std::max<uint64_t>(b, r->offsets[i] + r->lengths[i]);
            maxLen = std::max(maxLen, r->lengths[i]);
        }
        span[p] = b;
        base[p] = bytes;
        bytes += (b + 63) & ~63ull;
        n += r->n;
    }
    bytes += 64;
    if (!a->exReads || n > a->exReadsCapN || bytes > a->exReadsCapBytes) {
        snapgpu_device_reads_free(a->exReads);
        a->exReads = nullptr;
        a->exReadsCapN = a->exReadsCapBytes = 0;
        auto *d = new snapgpu_device_reads_t();
        d->owner = a;
        d->device = a->device;
        const uint64_t capN = n + n / 4 + 64, capB = bytes + bytes / 4 + 4096;
        bool ok = hipMalloc(&d->dBases, capB) == hipSuccess && hipMalloc(&d->dQuals, capB) == hipSuccess &&
                  hipMalloc(&d->dOffsets, (capN + 1) * 8) == hipSuccess && hipMalloc(&d->dLengths, (capN + 1) * 4) == hipSuccess &&
                  hipMalloc(&d->dOut, (capN + 1) * sizeof(snapgpu_result_t)) == hipSuccess &&
                  hipMalloc(&d->dDefer, 3 * (capN + 1) * sizeof(uint32_t)) == hipSuccess &&
                  hipMalloc(&d->dSeeds, (capN + 8) * SEEDS_PER_READ * sizeof(SeedRec)) == hipSuccess;
        if (!ok) { snapgpu_device_reads_free(d); snapgpu::setError("reads_upload: hipMalloc"); return nullptr; }
        a->exReads = d;
        a->exReadsCapN = capN;
        a->exReadsCapBytes = capB;
    }
    snapgpu_device_reads_t *d = a->exReads;
    d->n = n;
    d->maxLen = maxLen;
    hipStream_t s = a->stream();
    // one part: its own offset / length arrays; several: concatenated, offsets moved (host copies
    // that outlive the asynchronous copies: the stream is synchronised below)
    std::vector<uint64_t> offs;
    std::vector<uint32_t> lens;
    const uint64_t *hOff = parts[0]->offsets;
    const uint32_t *hLen = parts[0]->lengths;
    if (np > 1) {
        offs.reserve(n);
        lens.reserve(n);
        for (int p = 0; p < np; p++)
            for (uint64_t i = 0; i < parts[p]->n; i++) {
                offs.push_back(parts[p]->offsets[i] + base[p]);
                lens.push_back(parts[p]->lengths[i]);
            }
        hOff = offs.data();
        hLen = lens.data();
    }
    bool ok = true;
    for (int p = 0; p < np && ok; p++) {
        const_cast<snapgpu_reads_t *>(parts[p])->nUploads++;   // clipping is refused from now on
        const uint64_t pad = (p + 1 < np ? base[p + 1] : bytes) - base[p] - span[p];   // zeroed up to the next part / end
        ok = hipMemcpyAsync(d->dBases + base[p], parts[p]->bases, span[p], hipMemcpyHostToDevice, s) == hipSuccess &&
             hipMemsetAsync(d->dBases + base[p] + span[p], 0, pad, s) == hipSuccess &&
             hipMemcpyAsync(d->dQuals + base[p], parts[p]->quals, span[p], hipMemcpyHostToDevice, s) == hipSuccess &&
             hipMemsetAsync(d->dQuals + base[p] + span[p], 0, pad, s) == hipSuccess;
    }
    // the deferred lists are laid out by the batch size (launch_resident): 3 * (n + 1) entries
    if (!ok || hipMemcpyAsync(d->dOffsets, hOff, n * 8, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(d->dLengths, hLen, n * 4, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess) {
        snapgpu::setError("reads_upload: copy");
        return nullptr;
    }
    return d;
}

// The extended AlignRead over a batch with the multi-hits returned packed: read i's hits are
// packed[off[i] .. off[i+1]) (off has n + 1 entries).  snapgpu_align_batch_ex scatters them into
// the caller's rows; the RNA path reads them packed (a row layout of 1000 hits per read would
// fault in ~8 KB of fresh host pages per read for a handful of hits).
static int alignPacked(snapgpu_aligner_t *a, const snapgpu_reads_t *const *parts, int np,
                       const snapgpu_search_t *search, uint32_t maxHitsToGet,
                       snapgpu_result_t *out, int32_t *multiHitsFound,
                       std::vector<uint64_t> &off, std::vector<snapgpu_multi_hit_t> &dense) {
    uint64_t nAll = 0;
    for (int p = 0; p < np; p++) nAll += parts[p]->n;
    if (maxHitsToGet > SNAPGPU_MAX_MULTI_HITS_TO_GET || (maxHitsToGet && !multiHitsFound)) {
        snapgpu::setError("align_batch_ex: maxHitsToGet must be <= 1024 and come with multiHitsFound/multiHits");
        return SNAPGPU_EINVAL;
    }
    // above 512 the reference's rows alias (record_hit); they must stay inside hitLocations
    if (maxHitsToGet > 512 && (a->p.maxK + a->p.extraSearchDepth) * 512u + maxHitsToGet > (uint32_t)MAX_K * 512u) {
        snapgpu::setError("align_batch_ex: maxHitsToGet > 512 needs (maxK + extraSearchDepth) * 512 + maxHitsToGet <= 15872");
        return SNAPGPU_EUNSUPPORTED;
    }
    if (search)
        for (uint64_t i = 0; i < nAll; i++)
            if (search[i].searchRadius && search[i].searchDirection > 1) {
                snapgpu::setError("align_batch_ex: searchDirection must be 0 (FORWARD) or 1 (RC)");
                return SNAPGPU_EINVAL;
            }
    if (nAll == 0) return SNAPGPU_OK;
    snapgpu_device_reads_t *d = uploadCachedReads(a, parts, np);
    if (!d) return SNAPGPU_EDEVICE;
    AlignExt x;
    // grow-only device buffers of the aligner (hipMalloc / hipFree of the hit rows, ~1 GB for
    // the RNA path's 1000 hits per read, cost more than the kernels)
    auto ensure = [a](snapgpu_aligner::ExBuf &b, uint64_t bytes) -> hipError_t {
        if (bytes <= b.cap) return hipSuccess;
        devFree(a, b.p);
        b.p = nullptr;
        b.cap = 0;
        const uint64_t want = bytes + bytes / 4 + 256;
        hipError_t e = hipMalloc(&b.p, want);
        if (e == hipSuccess) b.cap = want;
        return e;
    };
    auto cleanup = [&]() { a->lastReads = nullptr; };   // d stays the aligner's (grow-only)
    hipError_t e = hipSuccess;
    const uint64_t n = nAll;
    void *dScratch = nullptr, *dFound = nullptr, *dHits = nullptr;
    if (search) {
        if ((e = ensure(a->exSearch, n * sizeof(snapgpu_search_t))) == hipSuccess)
            e = hipMemcpyAsync(a->exSearch.p, search, n * sizeof(snapgpu_search_t), hipMemcpyHostToDevice, a->stream());
        x.search = (const snapgpu_search_t *)a->exSearch.p;
    }
    if (e == hipSuccess && maxHitsToGet) {
        const uint64_t blocks = (uint64_t)(a->grid > a->grid512 ? a->grid : a->grid512);
        const uint64_t stride = multiHitStride(maxHitsToGet);
        if ((e = ensure(a->exScratch, blocks * stride * 4)) == hipSuccess &&
            (e = ensure(a->exFound, n * sizeof(int32_t))) == hipSuccess)
            e = ensure(a->exHits, n * maxHitsToGet * sizeof(snapgpu_multi_hit_t));
        dScratch = a->exScratch.p; dFound = a->exFound.p; dHits = a->exHits.p;
        x.maxHitsToGet = maxHitsToGet;
        x.hitScratch = (uint32_t *)dScratch;
        x.multiFound = (int32_t *)dFound;
        x.multiHits = (snapgpu_multi_hit_t *)dHits;
    }
    if (e != hipSuccess) {
        snapgpu::setError(std::string("align_batch_ex: ") + hipGetErrorString(e));
        cleanup();
        return SNAPGPU_EDEVICE;
    }
    int rc = launch_resident(a, d, x);
    if (!rc) rc = snapgpu_results_download(a, d, out);
    if (!rc && maxHitsToGet) {
        // only the found hits cross PCIe: counts first, then the hits packed on the device
        void *dOff = nullptr, *dDense = nullptr;
        off.assign(n + 1, 0);
        e = hipStreamSynchronize(a->stream());
        dense.clear();
        if (e == hipSuccess) e = hipMemcpy(multiHitsFound, dFound, n * sizeof(int32_t), hipMemcpyDeviceToHost);
        if (e == hipSuccess) {
            for (uint64_t i = 0; i < n; i++) {
                const int32_t f = multiHitsFound[i];
                off[i + 1] = off[i] + (uint64_t)(f < 0 ? 0 : (f > (int32_t)maxHitsToGet ? (int32_t)maxHitsToGet : f));
            }
            const uint64_t total = off[n];
            if (total) {
                dense.resize(total);
                if ((e = ensure(a->exOff, (n + 1) * sizeof(uint64_t))) == hipSuccess &&
                    (e = ensure(a->exDense, total * sizeof(snapgpu_multi_hit_t))) == hipSuccess &&
                    ((dOff = a->exOff.p), (dDense = a->exDense.p), true) &&
                    (e = hipMemcpyAsync(dOff, off.data(), (n + 1) * sizeof(uint64_t), hipMemcpyHostToDevice,
                                        a->stream())) == hipSuccess) {
                    const uint64_t blocks = std::min<uint64_t>((n + 3) / 4, 8192);
                    hipLaunchKernelGGL(compact_hits_kernel, dim3((unsigned)blocks), dim3(256), 0, a->stream(),
                                       (const snapgpu_multi_hit_t *)dHits, (const int32_t *)dFound,
                                       (const uint64_t *)dOff, n, maxHitsToGet, (snapgpu_multi_hit_t *)dDense);
                    if ((e = hipGetLastError()) == hipSuccess &&
                        (e = hipMemcpyAsync(dense.data(), dDense, total * sizeof(snapgpu_multi_hit_t),
                                            hipMemcpyDeviceToHost, a->stream())) == hipSuccess)
                        e = hipStreamSynchronize(a->stream());
                }
            }
        }
        if (e != hipSuccess) {
            snapgpu::setError(std::string("align_batch_ex download: ") + hipGetErrorString(e));
            rc = SNAPGPU_EDEVICE;
        }
    }
    cleanup();
    return rc;
}

extern "C++" int snapgpu_internal_align_batch_packed(snapgpu_aligner_t *a, const snapgpu_reads_t *reads,
                                                     const snapgpu_search_t *search, uint32_t maxHitsToGet,
                                                     snapgpu_result_t *out, int32_t *multiHitsFound,
                                                     std::vector<uint64_t> &off, std::vector<snapgpu_multi_hit_t> &dense) {
    if (!a || !reads || !out) return SNAPGPU_EINVAL;
    return alignPacked(a, &reads, 1, search, maxHitsToGet, out, multiHitsFound, off, dense);
}

// Both ends of the RNA path's pairs in one call (one upload, one pass set: a single persistent-kernel
// tail instead of two): records and hit counts of r0's reads, then r1's; off / dense over all of them.
extern "C++" int snapgpu_internal_align_batch_packed2(snapgpu_aligner_t *a, const snapgpu_reads_t *r0,
                                                      const snapgpu_reads_t *r1, uint32_t maxHitsToGet,
                                                      snapgpu_result_t *out, int32_t *multiHitsFound,
                                                      std::vector<uint64_t> &off, std::vector<snapgpu_multi_hit_t> &dense) {
    if (!a || !r0 || !r1 || !out) return SNAPGPU_EINVAL;
    const snapgpu_reads_t *parts[2] = {r0, r1};
    return alignPacked(a, parts, 2, nullptr, maxHitsToGet, out, multiHitsFound, off, dense);
}

int snapgpu_align_batch_ex(snapgpu_aligner_t *a, const snapgpu_reads_t *reads, const snapgpu_search_t *search,
                           uint32_t maxHitsToGet, snapgpu_result_t *out, int32_t *multiHitsFound,
                           snapgpu_multi_hit_t *multiHits) {
    if (maxHitsToGet && (!multiHitsFound || !multiHits)) {
        snapgpu::setError("align_batch_ex: maxHitsToGet must be <= 1024 and come with multiHitsFound/multiHits");
        return SNAPGPU_EINVAL;
    }
    std::vector<uint64_t> off;
    std::vector<snapgpu_multi_hit_t> dense;
    const int rc = snapgpu_internal_align_batch_packed(a, reads, search, maxHitsToGet, out, multiHitsFound, off, dense);
    if (rc || !maxHitsToGet) return rc;
    for (uint64_t i = 0; i < reads->n; i++)
        if (off[i + 1] > off[i])
            memcpy(multiHits + i * maxHitsToGet, dense.data() + off[i], (off[i + 1] - off[i]) * sizeof(snapgpu_multi_hit_t));
    return SNAPGPU_OK;
}

// Diagnostic self-test of the timeout path (no GPU needed): an aligner whose event never
// completes must fail the wait with SNAPGPU_EDEVICE, mark itself failed, and from then on
// free nothing (a freed buffer could still be in use by the kernel that never finished).
int snapgpu_selftest_timeout_path(void) {
    snapgpu_aligner_t fake;
    fake.timeoutSec = 0.02;
    fake.eventQuery = [](hipEvent_t) { return hipErrorNotReady; };
    hipEvent_t never = reinterpret_cast<hipEvent_t>(0x10);
    if (waitEvent(&fake, never) != SNAPGPU_EDEVICE || !fake.failed) return 1;
    if (waitEvent(&fake, never) != SNAPGPU_EDEVICE) return 2;   // stays failed
    auto *d = new snapgpu_device_reads_t();
    d->owner = &fake;
    d->dBases = reinterpret_cast<char *>(0x1000);   // never dereferenced or freed
    d->dOut = reinterpret_cast<snapgpu_result_t *>(0x2000);
    const uint64_t before = g_devFrees.load();
    snapgpu_device_reads_free(d);
    if (g_devFrees.load() != before) return 3;
    return 0;
}

int snapgpu_last_timing(snapgpu_aligner_t *a, snapgpu_timing_t *t) {
    if (!a || !t) return SNAPGPU_EINVAL;
    *t = a->timing;
    return SNAPGPU_OK;
}

int snapgpu_aligner_get_stats(const snapgpu_aligner_t *a, snapgpu_aligner_stats_t *s) {
    if (!a || !s) return SNAPGPU_EINVAL;
    *s = a->stats;
    return SNAPGPU_OK;
}
int snapgpu_phase_cycles(snapgpu_aligner_t *a, uint64_t *out, uint32_t len, int reset) {
    if (!a || !out) return SNAPGPU_EINVAL;
    const uint32_t m = len < (uint32_t)PH_SLOTS ? len : (uint32_t)PH_SLOTS;   // the caller's buffer length
    memset(out, 0, m * sizeof(uint64_t));
#if !SNAPGPU_PHASE_TIMERS
    snapgpu::setError("library built without phase timers (make PHASE_TIMERS=1)");
    return SNAPGPU_EUNSUPPORTED;
#endif
    if (!a->dPhase) { snapgpu::setError("phase diagnostics off (set SNAPGPU_PHASES=1 before aligner_create)"); return SNAPGPU_EINVAL; }
    HIPCHK(hipSetDevice(a->device));
    for (auto &L : a->lane) HIPCHK(hipStreamSynchronize(L.stream));   // both lanes' pass sets add to it
    std::vector<uint64_t> buf((size_t)a->grid * PH_SLOTS);
    hipStream_t s0 = a->stream();
    HIPCHK(hipMemcpyAsync(buf.data(), a->dPhase, buf.size() * sizeof(uint64_t), hipMemcpyDeviceToHost, s0));
    // zeroed on lane 0's stream; the sync below orders it before any later pass set of either lane
    if (reset) HIPCHK(hipMemsetAsync(a->dPhase, 0, buf.size() * sizeof(uint64_t), s0));
    HIPCHK(hipStreamSynchronize(s0));
    for (size_t i = 0; i < buf.size(); i++)
        if (i % PH_SLOTS < m) out[i % PH_SLOTS] += buf[i];
    return SNAPGPU_OK;
}
const snapgpu_index_t *snapgpu_aligner_index(const snapgpu_aligner_t *a) { return a ? a->idx : nullptr; }
int snapgpu_aligner_get_params(const snapgpu_aligner_t *a, snapgpu_aligner_params_t *p) {
    if (!a || !p) return SNAPGPU_EINVAL;
    *p = a->p;
    return SNAPGPU_OK;
}
int snapgpu_aligner_set_overlap(snapgpu_aligner_t *a, int overlap) {
    if (!a) return SNAPGPU_EINVAL;
    a->overlapKernels = overlap != 0;
    return SNAPGPU_OK;
}
int snapgpu_aligner_debug_trip(snapgpu_aligner_t *a, uint32_t read_index) {
    if (!a) return SNAPGPU_EINVAL;
    a->tripRead = read_index;
    return SNAPGPU_OK;
}
int snapgpu_aligner_max_k(const snapgpu_aligner_t *a) { return a ? (int)a->p.maxK : -1; }
const char *snapgpu_aligner_name(const snapgpu_aligner_t *) { return "Base Aligner (MI355X)"; }

int snapgpu_lv_batch(int device, int direction, uint32_t n, const char *texts, const uint64_t *textOff,
                     const uint32_t *textLen, const char *patterns, const char *quals, const uint64_t *patOff,
                     const uint32_t *patLen, const int32_t *k, int32_t *outScore, int32_t *outNetIndel,
                     double *outProb) {
    if (n == 0) return SNAPGPU_OK;
    int ndev = snapgpu_device_count();
    if (ndev <= 0 || device >= ndev) { snapgpu::setError("no such HIP device"); return SNAPGPU_EDEVICE; }
    HIPCHK(hipSetDevice(device));
    HIPCHK(ensureDeviceTables(device));
    std::vector<LvTask> tasks(n);
    std::vector<char> rbuf, qbuf, gbuf;
    const int PADG = 512;
    for (uint32_t i = 0; i < n; i++) {
        int pl = (int)patLen[i], tl = (int)textLen[i];
        if (pl > 500) { snapgpu::setError("lv_batch: pattern longer than 500"); return SNAPGPU_EINVAL; }
        LvTask &T = tasks[i];
        T.readOff = rbuf.size();
        // "read" in read coordinates: forward = pattern, reverse = reversed pattern
        for (int j = 0; j < pl; j++) {
            int src = direction > 0 ? j : pl - 1 - j;
            rbuf.push_back(patterns[patOff[i] + src]);
            qbuf.push_back(quals[patOff[i] + src]);
        }
        for (int j = 0; j < 64; j++) { rbuf.push_back(0); qbuf.push_back(0); }
        // virtual genome: 'n' * PADG + text + 'n' * PADG (the reference harness pads with 'n')
        uint64_t gstart = gbuf.size();
        gbuf.insert(gbuf.end(), PADG, 'n');
        gbuf.insert(gbuf.end(), texts + textOff[i], texts + textOff[i] + tl);
        gbuf.insert(gbuf.end(), PADG, 'n');
        while (gbuf.size() % 4) gbuf.push_back('n');
        T.n = pl;
        T.patternLen = pl;
        T.textLen = tl;
        T.k = k[i];
        T.dir = direction > 0 ? 1 : -1;
        if (direction > 0) { T.p0 = 0; T.g = PADG; }
        else { T.p0 = pl - 1; T.g = PADG + tl - pl; }
        T.genOff = gstart;
    }
    LvTask *dT; char *dR, *dQ, *dG; DevTables *dTab; int32_t *dS, *dN; double *dP;
    DevTables t;
    fillTables(t, 20);
    HIPCHK(hipMalloc(&dT, n * sizeof(LvTask)));
    HIPCHK(hipMalloc(&dR, rbuf.size() + 64));
    HIPCHK(hipMalloc(&dQ, qbuf.size() + 64));
    HIPCHK(hipMalloc(&dG, gbuf.size() + 64));
    HIPCHK(hipMalloc(&dTab, sizeof(DevTables)));
    HIPCHK(hipMalloc(&dS, n * 4));
    HIPCHK(hipMalloc(&dN, n * 4));
    HIPCHK(hipMalloc(&dP, n * 8));
    hipMemcpy(dT, tasks.data(), n * sizeof(LvTask), hipMemcpyHostToDevice);
    hipMemcpy(dR, rbuf.data(), rbuf.size(), hipMemcpyHostToDevice);
    hipMemcpy(dQ, qbuf.data(), qbuf.size(), hipMemcpyHostToDevice);
    hipMemcpy(dG, gbuf.data(), gbuf.size(), hipMemcpyHostToDevice);
    hipMemcpy(dTab, &t, sizeof(t), hipMemcpyHostToDevice);
    hipLaunchKernelGGL(lv_kernel, dim3(n), dim3(64), 0, 0, dT, dR, dQ, dG, dTab, dS, dN, dP);
    HIPCHK(hipGetLastError());
    HIPCHK(hipDeviceSynchronize());
    hipMemcpy(outScore, dS, n * 4, hipMemcpyDeviceToHost);
    hipMemcpy(outNetIndel, dN, n * 4, hipMemcpyDeviceToHost);
    hipMemcpy(outProb, dP, n * 8, hipMemcpyDeviceToHost);
    hipFree(dT); hipFree(dR); hipFree(dQ); hipFree(dG); hipFree(dTab); hipFree(dS); hipFree(dN); hipFree(dP);
    return SNAPGPU_OK;
}

// The production bit-plane LV (lv_group + lv_prob_pair) on explicit tasks: unit parity for
// LandauVishkin<dir>::computeEditDistance as align_kernel<128> runs it (patterns <= 127 bases:
// 128-bit masks) and as align_kernel<256> runs it (a batch with a longer pattern, <= 253 bases:
// 256-bit masks).
int snapgpu_lv_group_batch(int device, int direction, uint32_t n, const char *texts, const uint64_t *textOff,
                           const uint32_t *textLen, const char *patterns, const char *quals, const uint64_t *patOff,
                           const uint32_t *patLen, const int32_t *k, int32_t *outScore, int32_t *outNetIndel,
                           double *outProb) {
    if (n == 0) return SNAPGPU_OK;
    int ndev = snapgpu_device_count();
    if (ndev <= 0 || device >= ndev) { snapgpu::setError("no such HIP device"); return SNAPGPU_EDEVICE; }
    HIPCHK(hipSetDevice(device));
    HIPCHK(ensureDeviceTables(device));
    std::vector<LvgTask> tasks(n);
    uint64_t pBytes = 0, tBytes = 0;
    bool wide = false;
    for (uint32_t i = 0; i < n; i++) {
        if (patLen[i] == 0 || patLen[i] > 253 || k[i] < 0) {
            snapgpu::setError("lv_group_batch: pattern length must be 1..253 and k >= 0");
            return SNAPGPU_EINVAL;
        }
        wide |= patLen[i] > 127;
        pBytes = std::max<uint64_t>(pBytes, patOff[i] + patLen[i]);
        tBytes = std::max<uint64_t>(tBytes, textOff[i] + textLen[i]);
        tasks[i] = LvgTask{patOff[i], textOff[i], (int32_t)patLen[i], (int32_t)textLen[i], k[i], direction > 0 ? 1 : -1};
    }
    LvgTask *dT = nullptr; char *dP = nullptr, *dQ = nullptr, *dX = nullptr;
    int32_t *dS = nullptr, *dN = nullptr; double *dPr = nullptr;
    int rc = SNAPGPU_OK;
    if (hipMalloc(&dT, n * sizeof(LvgTask)) != hipSuccess || hipMalloc(&dP, pBytes + 64) != hipSuccess ||
        hipMalloc(&dQ, pBytes + 64) != hipSuccess || hipMalloc(&dX, tBytes + 64) != hipSuccess ||
        hipMalloc(&dS, n * 4) != hipSuccess || hipMalloc(&dN, n * 4) != hipSuccess || hipMalloc(&dPr, n * 8) != hipSuccess) {
        snapgpu::setError("lv_group_batch: hipMalloc");
        rc = SNAPGPU_ENOMEM;
    }
    if (!rc) {
        hipMemcpy(dT, tasks.data(), n * sizeof(LvgTask), hipMemcpyHostToDevice);
        hipMemcpy(dP, patterns, pBytes, hipMemcpyHostToDevice);
        hipMemcpy(dQ, quals, pBytes, hipMemcpyHostToDevice);
        hipMemcpy(dX, texts, tBytes, hipMemcpyHostToDevice);
        if (wide) hipLaunchKernelGGL(lv_group_kernel<4>, dim3(n), dim3(64), 0, 0, dT, dP, dQ, dX, dS, dN, dPr);
        else hipLaunchKernelGGL(lv_group_kernel<2>, dim3(n), dim3(64), 0, 0, dT, dP, dQ, dX, dS, dN, dPr);
        if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
            snapgpu::setError("lv_group_kernel failed");
            rc = SNAPGPU_EDEVICE;
        } else {
            hipMemcpy(outScore, dS, n * 4, hipMemcpyDeviceToHost);
            hipMemcpy(outNetIndel, dN, n * 4, hipMemcpyDeviceToHost);
            hipMemcpy(outProb, dPr, n * 8, hipMemcpyDeviceToHost);
        }
    }
    hipFree(dT); hipFree(dP); hipFree(dQ); hipFree(dX); hipFree(dS); hipFree(dN); hipFree(dPr);
    return rc;
}

// ------------------------------------------------------ CIGAR / SAM records
static CigarArgs cigar_args(snapgpu_aligner_t *a, snapgpu_device_reads_t *d, int useM) {
    CigarArgs C;
    memset(&C, 0, sizeof(C));
    const snapgpu_index_t *idx = a->idx;
    C.genome = a->dGenome; C.pieces = a->dPieces; C.nPieces = (int32_t)idx->genome->pieceOffsets.size();
    C.nBases = idx->genome->nBases; C.padding = idx->genome->chromosomePadding;
    C.bases = d->dBases; C.offsets = d->dOffsets; C.lengths = d->dLengths; C.nReads = (uint32_t)d->n;
    C.useM = useM ? 1 : 0;
    return C;
}

// cigar_kernel over n reads on the aligner's side stream (timing events around it)
static int cigar_kernel_launch(snapgpu_aligner_t *a, const CigarArgs &C, uint64_t n) {
    if (!a->cigarGrid) {
        hipDeviceProp_t prop;
        HIPCHK(hipGetDeviceProperties(&prop, a->device));
        int perCU = 0;
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&perCU, (const void *)cigar_kernel, 64, 0);
        a->cigarGrid = prop.multiProcessorCount * (perCU > 0 ? perCU : 8);
    }
    int grid = a->cigarGrid;
    if ((uint64_t)grid > n) grid = (int)n;
    if (grid == 0) return SNAPGPU_OK;
    HIPCHK(hipEventRecord(a->cev[0], a->sideStream));
    hipLaunchKernelGGL(cigar_kernel, dim3(grid), dim3(64), 0, a->sideStream, C);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(a->cev[1], a->sideStream));
    return SNAPGPU_OK;
}

static int cigar_launch(snapgpu_aligner_t *a, snapgpu_device_reads_t *d, CigarArgs C) {
    if (d->maxLen > (uint32_t)CIG_MAXLEN) { snapgpu::setError("cigar: read longer than 512 bases"); return SNAPGPU_EINVAL; }
    if (d->n > 0xffffffffull) { snapgpu::setError("batch too large"); return SNAPGPU_EINVAL; }
    if (!d->dCigEd) {
        HIPCHK(hipMalloc(&d->dCigEd, (d->n + 1) * 4));
        HIPCHK(hipMalloc(&d->dCigN, (d->n + 1) * 4));
        HIPCHK(hipMalloc(&d->dCigOps, (d->n + 1) * CIG_MAX_OPS * 4));
    }
    C.outEd = d->dCigEd; C.outNOps = d->dCigN; C.outOps = d->dCigOps;
    return cigar_kernel_launch(a, C, d->n);
}

int snapgpu_cigar_resident(snapgpu_aligner_t *a, snapgpu_device_reads_t *d, int useM) {
    if (!a || !d) return SNAPGPU_EINVAL;
    HIPCHK(hipSetDevice(a->device));
    if (a->failed) { snapgpu::setError("aligner failed earlier (device timeout)"); return SNAPGPU_EDEVICE; }
    // the records may come from pass sets on both lanes: the side stream waits for both
    for (auto &L : a->lane) {
        HIPCHK(hipEventRecord(L.done, L.stream));
        HIPCHK(hipStreamWaitEvent(a->sideStream, L.done, 0));
    }
    CigarArgs C = cigar_args(a, d, useM);
    C.records = d->dOut;
    const int rc = cigar_launch(a, d, C);
    if (rc) return rc;
    HIPCHK(hipEventRecord(a->residentSideDone, a->sideStream));
    a->residentSidePending = true;
    return SNAPGPU_OK;
}

int snapgpu_cigar_download(snapgpu_aligner_t *a, snapgpu_device_reads_t *d, int32_t *editDistance, uint32_t *nOps,
                           uint32_t *ops) {
    if (!a || !d || !editDistance || !nOps || !ops || !d->dCigEd) return SNAPGPU_EINVAL;
    HIPCHK(hipSetDevice(a->device));
    HIPCHK(hipStreamSynchronize(a->sideStream));
    HIPCHK(hipMemcpy(editDistance, d->dCigEd, d->n * 4, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(nOps, d->dCigN, d->n * 4, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(ops, d->dCigOps, d->n * CIG_MAX_OPS * 4, hipMemcpyDeviceToHost));
    return SNAPGPU_OK;
}

int snapgpu_cigar_last_ms(snapgpu_aligner_t *a, double *ms) {
    if (!a || !ms) return SNAPGPU_EINVAL;
    HIPCHK(hipSetDevice(a->device));
    HIPCHK(hipEventSynchronize(a->cev[1]));
    float f = 0;
    HIPCHK(hipEventElapsedTime(&f, a->cev[0], a->cev[1]));
    *ms = f;
    return SNAPGPU_OK;
}

int snapgpu_cigar_batch(snapgpu_aligner_t *a, const snapgpu_reads_t *reads, const uint32_t *locations,
                        const uint8_t *directions, int useM, int32_t *editDistance, uint32_t *nOps, uint32_t *ops) {
    if (!a || !reads || !locations || !directions || !editDistance || !nOps || !ops) return SNAPGPU_EINVAL;
    const char *const base[2] = {reads->bases, reads->bases};
    return snapgpu_internal_cigar_view(a, base, nullptr, reads->offsets, reads->lengths, reads->n, locations, directions,
                                       useM, editDistance, nOps, ops);
}

// snapgpu_cigar_batch over read i = base[mate[i]][offsets[i] .. + lengths[i]) (the product paths pass
// both ends of a pair batch at once: two buffers, each row tagged with its end), without a batch copy
// The CIGAR call itself; its results stay in the aligner's pinned output buffer: *outEd / *outNOps
// (n entries) and *outOps (n rows of CIG_MAX_OPS, each row's first nOps written), valid until the
// aligner's next CIGAR call.
static int cigarPinned(snapgpu_aligner_t *a, const char *const base[2], const uint8_t *mate, const uint64_t *offsets,
                       const uint32_t *lengths, uint64_t n, const uint32_t *locations, const uint8_t *directions,
                       int useM, const int32_t **outEd, const uint32_t **outNOps, const uint32_t **outOps) {
    if (a->failed) { snapgpu::setError("aligner failed earlier (device timeout)"); return SNAPGPU_EDEVICE; }
    *outEd = nullptr; *outNOps = nullptr; *outOps = nullptr;
    if (n == 0) return SNAPGPU_OK;
    if (n > 0xffffffffull) { snapgpu::setError("batch too large"); return SNAPGPU_EINVAL; }
    HIPCHK(hipSetDevice(a->device));
    // one packed upload: the reads' bases back to back (the caller's batch view may point into a
    // much larger buffer), offsets, lengths, locations, directions; no qualities (CIGARs use none)
    uint64_t total = 0;
    uint32_t maxLen = 0;
    for (uint64_t i = 0; i < n; i++) {
        total += lengths[i];
        maxLen = std::max(maxLen, lengths[i]);
    }
    if (maxLen > (uint32_t)CIG_MAXLEN) { snapgpu::setError("cigar: read longer than 512 bases"); return SNAPGPU_EINVAL; }
    auto al8 = [](uint64_t x) { return (x + 7) & ~7ull; };
    const uint64_t oOff = 0, oLen = al8(oOff + (n + 1) * 8), oLoc = al8(oLen + (n + 1) * 4), oDir = al8(oLoc + (n + 1) * 4),
                   oBases = al8(oDir + n + 1), inBytes = al8(oBases + total + 64);
    const uint64_t rEd = 0, rN = al8((n + 1) * 4), rOps = al8(rN + (n + 1) * 4), outBytes = rOps + (n + 1) * CIG_MAX_OPS * 4;
    auto ensure = [a](snapgpu_aligner::ExBuf &b, uint64_t bytes) -> hipError_t {
        if (bytes <= b.cap) return hipSuccess;
        devFree(a, b.p);
        b.p = nullptr;
        b.cap = 0;
        const uint64_t want = bytes + bytes / 4 + 256;
        hipError_t e = hipMalloc(&b.p, want);
        if (e == hipSuccess) b.cap = want;
        return e;
    };
    HIPCHK(ensure(a->cgIn, inBytes));
    HIPCHK(ensure(a->cgOut, outBytes));
    auto pinned = [](void *&p, uint64_t &cap, uint64_t bytes) -> hipError_t {
        if (bytes <= cap) return hipSuccess;
        hostPinnedFree(p);
        p = nullptr;
        cap = 0;
        const uint64_t want = bytes + bytes / 4 + 256;
        hipError_t e = hipHostMalloc(&p, want, hipHostMallocDefault);
        if (e == hipSuccess) cap = want;
        return e;
    };
    HIPCHK(pinned(a->cgPin, a->cgPinCap, inBytes));
    HIPCHK(pinned(a->cgPinOut, a->cgPinOutCap, outBytes));
    char *h = (char *)a->cgPin;
    uint64_t *hOff = (uint64_t *)(h + oOff);
    uint64_t at = 0;
    for (uint64_t i = 0; i < n; i++) { hOff[i] = at; at += lengths[i]; }
    hOff[n] = at;
    memcpy(h + oLen, lengths, n * 4);
    memcpy(h + oLoc, locations, n * 4);
    memcpy(h + oDir, directions, n);
    {
        // pack the bases (several threads for big batches: the copy is the host's part of the call)
        const unsigned nt = n < 16384 ? 1u : snapgpu::hostThreads(8);
        auto pack = [&](uint64_t b, uint64_t e) {
            for (uint64_t i = b; i < e; i++) memcpy(h + oBases + hOff[i], base[mate ? mate[i] & 1 : 0] + offsets[i], lengths[i]);
        };
        std::vector<std::thread> th;
        for (unsigned t = 1; t < nt; t++) th.emplace_back(pack, n * t / nt, n * (t + 1) / nt);
        pack(0, n / nt);
        for (auto &x : th) x.join();
        memset(h + oBases + total, 0, inBytes - oBases - total);
    }
    hipStream_t st = a->sideStream;
    char *dIn = (char *)a->cgIn.p, *dOut = (char *)a->cgOut.p;
    HIPCHK(hipMemcpyAsync(dIn, h, inBytes, hipMemcpyHostToDevice, st));
    CigarArgs C;
    memset(&C, 0, sizeof(C));
    const snapgpu_index_t *idx = a->idx;
    C.genome = a->dGenome; C.pieces = a->dPieces; C.nPieces = (int32_t)idx->genome->pieceOffsets.size();
    C.nBases = idx->genome->nBases; C.padding = idx->genome->chromosomePadding;
    C.bases = dIn + oBases; C.offsets = (const uint64_t *)(dIn + oOff); C.lengths = (const uint32_t *)(dIn + oLen);
    C.nReads = (uint32_t)n;
    C.locations = (const uint32_t *)(dIn + oLoc);
    C.directions = (const uint8_t *)(dIn + oDir);
    C.useM = useM ? 1 : 0;
    C.outEd = (int32_t *)(dOut + rEd); C.outNOps = (uint32_t *)(dOut + rN); C.outOps = (uint32_t *)(dOut + rOps);
    int rc = cigar_kernel_launch(a, C, n);
    if (rc) return rc;
    // outputs through pinned memory (one D2H), then only each row's nOps ops to the caller (rows hold
    // a few of their 64 slots; a pageable D2H of every full row was most of the call)
    char *ho = (char *)a->cgPinOut;
    HIPCHK(hipMemcpyAsync(ho, dOut, outBytes, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    *outEd = (const int32_t *)(ho + rEd);
    *outNOps = (const uint32_t *)(ho + rN);
    *outOps = (const uint32_t *)(ho + rOps);
    return SNAPGPU_OK;
}

int snapgpu_internal_cigar_pinned(snapgpu_aligner_t *a, const char *const base[2], const uint8_t *mate,
                                  const uint64_t *offsets, const uint32_t *lengths, uint64_t n,
                                  const uint32_t *locations, const uint8_t *directions, int useM,
                                  const int32_t **editDistance, const uint32_t **nOps, const uint32_t **ops) {
    if (!a || !base || !offsets || !lengths || !locations || !directions || !editDistance || !nOps || !ops)
        return SNAPGPU_EINVAL;
    return cigarPinned(a, base, mate, offsets, lengths, n, locations, directions, useM, editDistance, nOps, ops);
}

int snapgpu_internal_cigar_view(snapgpu_aligner_t *a, const char *const base[2], const uint8_t *mate,
                                const uint64_t *offsets, const uint32_t *lengths,
                                uint64_t n, const uint32_t *locations, const uint8_t *directions, int useM,
                                int32_t *editDistance, uint32_t *nOps, uint32_t *ops) {
    const int32_t *ed = nullptr;
    const uint32_t *no = nullptr, *hops = nullptr;
    const int rc = cigarPinned(a, base, mate, offsets, lengths, n, locations, directions, useM, &ed, &no, &hops);
    if (rc || n == 0) return rc;
    // only each row's nOps ops to the caller (rows hold a few of their 64 slots), on host threads
    const unsigned nt = n < 65536 ? 1u : snapgpu::hostThreads(8);
    auto copy = [&](uint64_t b, uint64_t e) {
        memcpy(editDistance + b, ed + b, (e - b) * 4);
        memcpy(nOps + b, no + b, (e - b) * 4);
        for (uint64_t i = b; i < e; i++) {
            const uint32_t k = std::min<uint32_t>(no[i], (uint32_t)CIG_MAX_OPS);
            memcpy(ops + i * CIG_MAX_OPS, hops + i * CIG_MAX_OPS, k * 4);
        }
    };
    std::vector<std::thread> th;
    for (unsigned t = 1; t < nt; t++) th.emplace_back(copy, n * t / nt, n * (t + 1) / nt);
    copy(0, n / nt);
    for (auto &x : th) x.join();
    return SNAPGPU_OK;
}

int snapgpu_aligner_lookup_seeds(snapgpu_aligner_t *a, const char *seedBases, uint64_t n, int mode, uint64_t *out,
                                 uint32_t *lines) {
    if (!a || (n && (!seedBases || !out || !lines)) || mode < 0 || mode > 2) return SNAPGPU_EINVAL;
    if (n == 0) return SNAPGPU_OK;
    if (n >= (1ull << 31)) { snapgpu::setError("lookup_seeds: too many seeds"); return SNAPGPU_EINVAL; }
    if (a->failed) return SNAPGPU_EDEVICE;
    const uint32_t L = a->idx->seedLen;
    for (uint64_t i = 0; i < n * L; i++) {   // GenomeIndex::lookupSeed takes ACGT seeds only
        const char c = seedBases[i];
        if (c != 'A' && c != 'C' && c != 'G' && c != 'T') { snapgpu::setError("lookup_seeds: non-ACGT base"); return SNAPGPU_EINVAL; }
    }
    HIPCHK(hipSetDevice(a->device));
    KArgs A;
    if (int rc = snapgpu_internal_index_args(a, &A, nullptr)) return rc;
    char *dS = nullptr;
    unsigned long long *dO = nullptr;
    uint32_t *dL = nullptr;
    int rc = SNAPGPU_OK;
    hipStream_t st = a->stream();
    if (hipMalloc(&dS, n * L) != hipSuccess || hipMalloc(&dO, n * 48) != hipSuccess || hipMalloc(&dL, n * 4) != hipSuccess) {
        snapgpu::setError("lookup_seeds: hipMalloc");
        rc = SNAPGPU_ENOMEM;
    } else if (hipMemcpyAsync(dS, seedBases, n * L, hipMemcpyHostToDevice, st) != hipSuccess) {
        rc = SNAPGPU_EDEVICE;
    } else {
        const unsigned grid = (unsigned)std::min<uint64_t>((n + 63) / 64, 4096);
        hipLaunchKernelGGL(lookup_seeds_kernel, dim3(grid), dim3(64), 0, st, A, dS, (uint32_t)n, mode, dO, dL);
        if (hipGetLastError() != hipSuccess || hipMemcpyAsync(out, dO, n * 48, hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipMemcpyAsync(lines, dL, n * 4, hipMemcpyDeviceToHost, st) != hipSuccess || hipStreamSynchronize(st) != hipSuccess) {
            snapgpu::setError("lookup_seeds: kernel");
            rc = SNAPGPU_EDEVICE;
        }
    }
    devFree(a, dS); devFree(a, dO); devFree(a, dL);
    return rc;
}

int snapgpu_aligner_bucket_info(const snapgpu_aligner_t *a, snapgpu_bucket_info_t *info) {
    if (!a || !info) return SNAPGPU_EINVAL;
    *info = a->bucketInfo;
    return SNAPGPU_OK;
}

int snapgpu_gather_peak(snapgpu_aligner_t *a, uint32_t nLoads, double *ms) {
    if (!a || !ms || nLoads == 0) return SNAPGPU_EINVAL;
    HIPCHK(hipSetDevice(a->device));
    const uint64_t nBk = a->bucketInfo.nBuckets;
    if (nBk == 0 || nBk >= (1ull << 32)) { snapgpu::setError("gather_peak: bucket count"); return SNAPGPU_EINVAL; }
    const unsigned grid = (nLoads + 1023) / 1024;
    float best = 0;
    for (int rep = 0; rep < 3; rep++) {
        HIPCHK(hipEventRecord(a->cev[0], a->stream()));
        hipLaunchKernelGGL(gather_peak_kernel, dim3(grid), dim3(256), 0, a->stream(), a->dBuckets, (uint32_t)nBk, nLoads,
                           0x5bd1e995u * (rep + 1), a->lane[0].counter + 8);
        HIPCHK(hipGetLastError());
        HIPCHK(hipEventRecord(a->cev[1], a->stream()));
        HIPCHK(hipEventSynchronize(a->cev[1]));
        float f = 0;
        HIPCHK(hipEventElapsedTime(&f, a->cev[0], a->cev[1]));
        if (rep == 0 || f < best) best = f;
    }
    *ms = best;
    return SNAPGPU_OK;
}

// Streaming-copy ceiling (copy_peak_kernel): best of 3 over `bytes` read + `bytes` written.
int snapgpu_copy_peak(snapgpu_aligner_t *a, uint64_t bytes, double *ms) {
    if (!a || !ms || bytes < 4096) return SNAPGPU_EINVAL;
    if (a->failed) return SNAPGPU_EDEVICE;
    HIPCHK(hipSetDevice(a->device));
    const uint64_t nw = bytes / 16 / 1024 * 1024;
    void *src = nullptr, *dst = nullptr;
    HIPCHK(hipMalloc(&src, nw * 16));
    if (hipMalloc(&dst, nw * 16) != hipSuccess) { devFree(a, src); snapgpu::setError("copy_peak: hipMalloc"); return SNAPGPU_ENOMEM; }
    hipDeviceProp_t prop;
    HIPCHK(hipGetDeviceProperties(&prop, a->device));
    const unsigned grid = (unsigned)prop.multiProcessorCount * 16;
    float best = 0;
    int rc = SNAPGPU_OK;
    HIPCHK(hipMemsetAsync(src, 1, nw * 16, a->stream()));
    for (int rep = 0; rep < 4 && rc == SNAPGPU_OK; rep++) {   // first run warms up
        hipEventRecord(a->cev[0], a->stream());
        hipLaunchKernelGGL(copy_peak_kernel, dim3(grid), dim3(256), 0, a->stream(), (const uint4 *)src, (uint4 *)dst, nw);
        hipEventRecord(a->cev[1], a->stream());
        if (hipEventSynchronize(a->cev[1]) != hipSuccess) { rc = SNAPGPU_EDEVICE; break; }
        float f = 0;
        hipEventElapsedTime(&f, a->cev[0], a->cev[1]);
        if (rep == 1 || (rep > 1 && f < best)) best = f;
    }
    devFree(a, src);
    devFree(a, dst);
    *ms = best;
    return rc;
}

}  // extern "C"

// ------------------------------------------------- internal hand-off to paired.hip
// The paired-end aligner (paired.hip) runs over the index one snapgpu_aligner uploaded (the one
// its chimeric fallback uses): the index, genome and table arguments of its kernels.
int snapgpu_internal_devbuf(snapgpu_aligner_t *a, int slot, uint64_t bytes, void **p) {
    if (!a || slot < 0 || slot >= 8 || !p) return SNAPGPU_EINVAL;
    if (a->failed) return SNAPGPU_EDEVICE;
    auto &b = a->aux[slot];
    if (bytes > b.cap) {
        devFree(a, b.p);
        b.p = nullptr;
        b.cap = 0;
        const uint64_t want = bytes + bytes / 4 + 256;
        if (hipMalloc(&b.p, want) != hipSuccess) return SNAPGPU_ENOMEM;
        b.cap = want;
    }
    *p = b.p;
    return SNAPGPU_OK;
}
hipStream_t snapgpu_internal_stream(snapgpu_aligner_t *a) { return a->sideStream; }   // charseeds.hip

int snapgpu_internal_index_args(const snapgpu_aligner_t *a, sgk::KArgs *A, int *device) {
    if (!a || !A) return SNAPGPU_EINVAL;
    memset(A, 0, sizeof(*A));
    const snapgpu_index_t *idx = a->idx;
    A->buckets = a->dBuckets; A->bucketBase = a->dBucketBase; A->bucketCount = a->dBucketCount; A->overflow = a->dOverflow;
    A->genome = a->dGenome; A->pieces = a->dPieces; A->nPieces = (int32_t)idx->genome->pieceOffsets.size();
    A->gpl = a->dGPlanes; A->hasIupac = idx->hasIupac ? 1u : 0u;
    A->nBases = idx->genome->nBases; A->seedLen = idx->seedLen; A->nTables = idx->nTables;
    A->padding = idx->genome->chromosomePadding;
    A->tab = a->dTab;
    A->kRows = 31;
    if (device) *device = a->device;
    return a->failed ? SNAPGPU_EDEVICE : SNAPGPU_OK;
}

void snapgpu_internal_fill_tables(sgk::DevTables *t, uint32_t seedLen) { fillTables(*t, seedLen); }
bool snapgpu_internal_aligner_failed(const snapgpu_aligner_t *a) { return a && a->failed; }
