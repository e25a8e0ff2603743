// lv_lane.h -- Landau-Vishkin distance of one candidate per LANE (no path), for the forced-mode
// prefilter of align_kernel<128> (align_score.h, forced_filter).
//
// The group scorer (align_score.h lv_group) runs one candidate per group of GS = 8..64 lanes, lane
// = diagonal: 4 candidates per pass at the usual k of 4..7.  In forced mode a repeat-rich read pops
// hundreds of elements with one unscored candidate each, and 87 % of the LV calls fail, so most
// passes only establish "distance > k".  Here one lane takes one candidate and runs the same
// recurrence (LandauVishkin.h:211-455 as lv_group restates it, B = L + 2 arithmetic, X / D / I
// preference irrelevant for the value) over its own diagonals, held as 128-bit mismatch masks in
// registers: 64 candidates per pass.  Only the distance comes out; a candidate whose distances can
// still succeed goes through lv_group for its path (the match probability and netIndel).
//
// Exactness: lv_group's row e reads row e-1 only, so a lane evaluating row e's diagonals from its
// own copy of row e-1 computes the same values; the first row in which a diagonal reaches
// patternLen is the distance in both.  KM bounds k at compile time (register arrays, no dynamic
// indexing); callers use it only for k <= KM.  The kernel runs the distance split over a lane pair
// (limits <= 5) or a lane quad (limits 6 and 7), below; lv_lane_dist is the single-lane reference form.
#pragma once
#include <stdint.h>

namespace sgk {

// first set position >= m0 of a 128-bit mask (w0 = positions 0..63), 128 if none; m0 in [0, 128]
// (mk_first<2> of align_score.h with the suffix answer computed inline).  Written as selects, not
// early returns: inlined into lv_pair_dist's row loop, returns become exec-mask branches whose
// live ranges (the clamped start across both sides) spilled to scratch in align_kernel<128>.
__host__ __device__ __forceinline__ int ll_first_from(uint64_t w0, uint64_t w1, int m0) {
    const bool hw = m0 >= 64;
    const uint64_t x = (hw ? w1 : w0) >> (m0 & 63);   // m0 = 128: m0 & 63 = 0, cleared below
    const int inWord = m0 + (x ? __builtin_ctzll(x) : 0);
    const int inHigh = !hw && w1 ? 64 + __builtin_ctzll(w1) : 128;
    const int r = x ? inWord : inHigh;
    return m0 >= 128 ? 128 : r;
}

// last set position <= m1 of a 128-bit mask, -1 if none; m1 in [-1, 127] (selects, as above)
__host__ __device__ __forceinline__ int ll_last_upto(uint64_t w0, uint64_t w1, int m1) {
    const bool hw = m1 >= 64;
    const uint64_t x = (hw ? w1 : w0) << (63 - (m1 & 63));   // m1's bit at 63; m1 = -1: cleared below
    const int inWord = m1 - (x ? __builtin_clzll(x) : 0);
    const int inLow = hw && w0 ? 63 - __builtin_clzll(w0) : -1;
    const int r = x ? inWord : inLow;
    return m1 < 0 ? -1 : r;
}

// "first set position >= p" of the direction's mask of diagonal d.  DIR = 1: the forward mask
// M[d].  DIR = -1: the bit-reversed mask of forward diagonal -d (R[p] = F[127 - p], as lv_pass's
// mk_reverse builds it), read from the forward mask by a "last set <= 127 - p" query, so no reversed
// copy is held.  p in [0, 128]; 128 if none.
template <int KM, int DIR>
__host__ __device__ __forceinline__ int ll_first_dir(const uint64_t (&M)[2 * KM + 1][2], int d, int p) {
    if (DIR > 0) return ll_first_from(M[d + KM][0], M[d + KM][1], p);
    return 127 - ll_last_upto(M[KM - d][0], M[KM - d][1], 127 - p);
}

// Distance of pattern mask positions q0 .. q0 + patternLen against the text (diagonal d of the
// lane's masks, d in [-KM, KM], through ll_first_dir<KM, DIR>: for DIR = -1 the positions are those
// of the reversed masks, q0 = 127 - (first pattern base's forward position)), limit k <= KM; -1 when
// above k.  `act` false: -1.
// Mirrors lv_group<1, GS, 2>: end0 / exact prefix (LandauVishkin.h:290-305), then rows 1..k with
// best = max(L[d-1], L[d] + 1, L[d+1] + 1), the slide capped at endd = min(patternLen, textLen - d),
// and the `best >= endd` case as there.
template <int KM, int DIR = 1>
__host__ __device__ __forceinline__ int lv_lane_dist(const uint64_t (&M)[2 * KM + 1][2], bool act, int q0, int patternLen,
                                                    int textLen, int k) {
    constexpr int NBITS = 128;
    if (!act) return -1;
    if (k > KM) k = KM;
    const int end0 = patternLen < textLen ? patternLen : textLen;
    {
        const int fm = ll_first_dir<KM, DIR>(M, 0, q0) - q0;
        const int v0 = fm < end0 ? fm : end0;
        if (v0 == end0) {
            const int result = patternLen > end0 ? patternLen - end0 : 0;
            return result > k ? -1 : result;
        }
        // rows 1..k over B = L + 2 (0: no value), diagonals -KM-1 .. KM+1 (the outer two stay 0)
        int B[2 * KM + 3];
#pragma unroll
        for (int i = 0; i < 2 * KM + 3; i++) B[i] = 0;
        B[KM + 1] = v0 + 2;
        const int patB = patternLen + 2, q0m2 = q0 - 2;
#pragma unroll
        for (int e = 1; e <= KM; e++) {
            if (e > k) break;
            // row e from row e-1 in place: `left` carries the old value of the diagonal below
            bool hit = false;
            int left = B[KM - e];   // old B[d - 1] of the band's first diagonal d = -e
#pragma unroll
            for (int d = -KM; d <= KM; d++) {
                if (d < -e || d > e) continue;   // compile-time: the band of row e
                const int i = d + KM + 1;
                const int old = B[i];
                const int leftB = left, rightB = B[i + 1] + 1, x1B = old + 1;
                left = old;
                const int bxdB = leftB > x1B ? leftB : x1B;
                const int bestB = rightB > bxdB ? rightB : bxdB;
                const int endd = patternLen < textLen - d ? patternLen : textLen - d;
                const int enddB = endd + 2;
                const int mpos = q0m2 + bestB;
                const int mposc = mpos < NBITS ? mpos : NBITS;
                const int fa = ll_first_dir<KM, DIR>(M, d, mposc);
                const int fB = fa - q0m2;
                const int slidB = fB < enddB ? fB : enddB;
                const int bnewB = bestB < enddB ? slidB : (fa == mposc ? bestB : enddB);
                B[i] = bnewB;
                hit = hit || bnewB == patB;
            }
            if (hit) return e;
        }
    }
    return -1;
}

// ------------------------------------------------------------ two lanes per candidate
// lv_lane_dist with a candidate's diagonals split over a lane pair (lanes 2c, 2c + 1): half h holds
// forward diagonals x = 0, -1, .., -KM (h = 0) or 0, 1, .., KM (h = 1) at local index i = |x|, so
// each lane keeps KM + 1 masks instead of 2 KM + 1 (the registers a 64-candidate pass cannot spare
// inside align_kernel<128>) and the row loop runs over i = 0 .. e in both halves.  Diagonal 0 is
// computed by both; the one value a row needs across the pair -- the partner's diagonal +-1, the far
// neighbour of diagonal 0 -- and the row's "reached patternLen" flag cross by a DPP lane swap.  Both
// lanes of a pair must call it together with the same act / k (their element is the same); the
// distance comes out in both.  For DIR = -1 reverse diagonal d reads forward diagonal -d (the same
// mask index i; ll_first_dir's reversed view), so the halves swap roles.
__device__ __forceinline__ int ll_pair_swap(int v) {
    return __builtin_amdgcn_mov_dpp(v, 0xB1, 0xf, 0xf, false);   // quad_perm [1, 0, 3, 2]: lane ^ 1
}

template <int KM, int DIR>
__device__ __forceinline__ int lv_pair_dist(const uint64_t (&M)[KM + 1][2], int h, bool act, int q0, int patternLen,
                                            int textLen, int k) {
    constexpr int NBITS = 128;
    if (!act) return -1;
    if (k > KM) k = KM;
    const bool up = DIR > 0 ? h != 0 : h == 0;   // local i is diagonal +i (else -i)
    auto first = [&](int i, int p) -> int {
        if (DIR > 0) return ll_first_from(M[i][0], M[i][1], p);
        return 127 - ll_last_upto(M[i][0], M[i][1], 127 - p);
    };
    const int end0 = patternLen < textLen ? patternLen : textLen;
    const int fm = first(0, q0) - q0;
    const int v0 = fm < end0 ? fm : end0;
    if (v0 == end0) {
        const int result = patternLen > end0 ? patternLen - end0 : 0;
        return result > k ? -1 : result;
    }
    // B[i + 1] = local i (B = L + 2, 0: no value); B[0] = the partner's local 1; B[KM + 2] stays 0
    int B[KM + 3];
#pragma unroll
    for (int i = 0; i < KM + 3; i++) B[i] = 0;
    B[1] = v0 + 2;
    const int patB = patternLen + 2, q0m2 = q0 - 2;
#pragma unroll
    for (int e = 1; e <= KM; e++) {
        if (e > k) break;
        B[0] = ll_pair_swap(B[2]);
        bool hit = false;
        int prev = B[0];   // old value of local i - 1
#pragma unroll
        for (int i = 0; i <= KM; i++) {
            if (i > e) continue;   // compile-time: |d| <= e
            const int d = up ? i : -i;
            const int old = B[i + 1], lo = prev, hi = B[i + 2];
            prev = old;
            const int leftB = up ? lo : hi;              // B[d - 1]
            const int rightB = (up ? hi : lo) + 1;       // B[d + 1] + 1
            const int x1B = old + 1;
            const int bxdB = leftB > x1B ? leftB : x1B;
            const int bestB = rightB > bxdB ? rightB : bxdB;
            const int endd = patternLen < textLen - d ? patternLen : textLen - d;
            const int enddB = endd + 2;
            const int mpos = q0m2 + bestB;
            const int mposc = mpos < NBITS ? mpos : NBITS;
            const int fa = first(i, mposc);
            const int fB = fa - q0m2;
            const int slidB = fB < enddB ? fB : enddB;
            const int bnewB = bestB < enddB ? slidB : (fa == mposc ? bestB : enddB);
            B[i + 1] = bnewB;
            hit = hit || bnewB == patB;
        }
        // (the swap is evaluated by both lanes: under a short-circuit `||` a lane that already hit
        // would skip it, and its partner's DPP would read a lane outside EXEC)
        const int partnerHit = ll_pair_swap(hit ? 1 : 0);
        if (hit || partnerHit != 0) return e;
    }
    return -1;
}

// ------------------------------------------------------------ four lanes per candidate
// The same distance with a candidate's 2 KQ + 1 = 15 diagonals over a lane quad (lanes 4c .. 4c + 3),
// for limits 6 and 7, where a lane pair would hold 8 masks per lane (the registers spill).  Lane q holds
// slots s = 4q + j (j = 0..3), forward diagonal x = s - KQ (x = -7 .. 8; slot x = 8 is never in a row's
// band), 4 masks per lane.  A row reads its neighbours x - 1 / x + 1 of the previous row: inside the lane,
// or -- for j = 0 / j = 3 -- the neighbour lane's j = 3 / j = 0, moved by a DPP quad permute.  DIR = -1:
// reverse diagonal d = -x reads forward diagonal x's mask through the "last set <= 127 - p" view (as the
// pair form does), so its d - 1 / d + 1 are slots s + 1 / s - 1.
//
// quad_row: row e of lane q, every slot from the previous row's values (Bl[0]: the lower neighbour lane's
// slot 3, 0 for q = 0; Bl[1..4]: own slots; Bl[5]: the upper neighbour's slot 0, 0 for q = 3), in place.
// Out-of-band slots (|x| > e) keep their value.  Returns whether a slot reached patternLen.  The per-slot
// arithmetic is lv_lane_dist's.  Shared by lv_quad_dist and the host lockstep emulation
// (tests/c/lv_lane_test.cpp).
constexpr int LQ_K = 7;
template <int DIR>
__host__ __device__ __forceinline__ bool quad_row(const uint64_t (&M)[4][2], int q, int e, int (&Bl)[6], int q0m2, int patB,
                                                  int patternLen, int textLen) {
    constexpr int NBITS = 128;
    int nb[4];
    bool hit = false;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const int x = 4 * q + j - LQ_K;
        const int ax = x < 0 ? -x : x;
        const int d = DIR > 0 ? x : -x;
        const int old = Bl[j + 1], lowB = Bl[j], highB = Bl[j + 2];   // slots x - 1, x + 1
        const int leftB = DIR > 0 ? lowB : highB;                      // B[d - 1]
        const int rightB = (DIR > 0 ? highB : lowB) + 1;               // B[d + 1] + 1
        const int x1B = old + 1;
        const int bxdB = leftB > x1B ? leftB : x1B;
        const int bestB = rightB > bxdB ? rightB : bxdB;
        const int endd = patternLen < textLen - d ? patternLen : textLen - d;
        const int enddB = endd + 2;
        const int mpos = q0m2 + bestB;
        const int mposc = mpos < NBITS ? mpos : NBITS;
        const int fa = DIR > 0 ? ll_first_from(M[j][0], M[j][1], mposc) : 127 - ll_last_upto(M[j][0], M[j][1], 127 - mposc);
        const int fB = fa - q0m2;
        const int slidB = fB < enddB ? fB : enddB;
        const int bnewB = bestB < enddB ? slidB : (fa == mposc ? bestB : enddB);
        const bool in = ax <= e;
        nb[j] = in ? bnewB : old;
        hit = hit || (in && bnewB == patB);
    }
#pragma unroll
    for (int j = 0; j < 4; j++) Bl[j + 1] = nb[j];
    return hit;
}
// first set position >= p of lane-local slot j in the direction's view (see ll_first_dir)
template <int DIR>
__host__ __device__ __forceinline__ int quad_first(const uint64_t (&M)[4][2], int j, int p) {
    return DIR > 0 ? ll_first_from(M[j][0], M[j][1], p) : 127 - ll_last_upto(M[j][0], M[j][1], 127 - p);
}

// All four lanes of a quad call it together with the same act / k (one candidate); the distance (or -1
// above k) comes out in all four.  Divergence between quads is fine: every DPP stays inside the quad.
template <int DIR>
__device__ __forceinline__ int lv_quad_dist(const uint64_t (&M)[4][2], int q, bool act, int q0, int patternLen, int textLen,
                                            int k) {
    if (!act) return -1;
    if (k > LQ_K) k = LQ_K;
    const int end0 = patternLen < textLen ? patternLen : textLen;
    // diagonal 0 is slot 7: lane 1, j = 3 (broadcast over the quad: quad_perm [1, 1, 1, 1])
    const int f0 = __builtin_amdgcn_mov_dpp(quad_first<DIR>(M, 3, q0), 0x55, 0xf, 0xf, false);
    const int fm = f0 - q0;
    const int v0 = fm < end0 ? fm : end0;
    if (v0 == end0) {
        const int result = patternLen > end0 ? patternLen - end0 : 0;
        return result > k ? -1 : result;
    }
    int Bl[6] = {0, 0, 0, 0, 0, 0};
    if (q == 1) Bl[4] = v0 + 2;
    const int patB = patternLen + 2, q0m2 = q0 - 2;
#pragma unroll
    for (int e = 1; e <= LQ_K; e++) {
        if (e > k) break;
        const int lo = __builtin_amdgcn_mov_dpp(Bl[4], 0x90, 0xf, 0xf, false);   // quad_perm [0, 0, 1, 2]: lane q - 1's slot 3
        const int hi = __builtin_amdgcn_mov_dpp(Bl[1], 0xF9, 0xf, 0xf, false);   // quad_perm [1, 2, 3, 3]: lane q + 1's slot 0
        Bl[0] = q == 0 ? 0 : lo;
        Bl[5] = q == 3 ? 0 : hi;
        int h = quad_row<DIR>(M, q, e, Bl, q0m2, patB, patternLen, textLen) ? 1 : 0;
        h |= __builtin_amdgcn_mov_dpp(h, 0xB1, 0xf, 0xf, false);   // quad_perm [1, 0, 3, 2]
        h |= __builtin_amdgcn_mov_dpp(h, 0x4E, 0xf, 0xf, false);   // quad_perm [2, 3, 0, 1]
        if (h) return e;
    }
    return -1;
}

}  // namespace sgk
