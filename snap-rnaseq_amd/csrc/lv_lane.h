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
// indexing); callers use it only for k <= KM.
#pragma once
#include <stdint.h>

namespace sgk {

// first set position >= m0 of a 128-bit mask (w0 = positions 0..63), 128 if none; m0 in [0, 128]
// (mk_first<2> of align_score.h with the suffix answer computed inline)
__host__ __device__ __forceinline__ int ll_first_from(uint64_t w0, uint64_t w1, int m0) {
    if (m0 >= 128) return 128;
    const bool hw = m0 >= 64;
    const uint64_t x = (hw ? w1 : w0) >> (m0 & 63);
    if (x) return m0 + __builtin_ctzll(x);
    if (hw || !w1) return 128;
    return 64 + __builtin_ctzll(w1);
}

__host__ __device__ __forceinline__ uint64_t ll_brev64(uint64_t x) {
    return ((uint64_t)__builtin_bitreverse32((uint32_t)x) << 32) | __builtin_bitreverse32((uint32_t)(x >> 32));
}

// Distance of pattern mask positions q0 .. q0 + patternLen against the text (diagonal d of the
// lane's mask M[d + KM], d in [-KM, KM]), limit k <= KM; -1 when above k.  `act` false: -1.
// Mirrors lv_group<1, GS, 2>: end0 / exact prefix (LandauVishkin.h:290-305), then rows 1..k with
// best = max(L[d-1], L[d] + 1, L[d+1] + 1), the slide capped at endd = min(patternLen, textLen - d),
// and the `best >= endd` case as there.
template <int KM>
__host__ __device__ __forceinline__ int lv_lane_dist(const uint64_t (&M)[2 * KM + 1][2], bool act, int q0, int patternLen,
                                                    int textLen, int k) {
    constexpr int NBITS = 128;
    if (!act) return -1;
    if (k > KM) k = KM;
    const int end0 = patternLen < textLen ? patternLen : textLen;
    {
        const int fm = ll_first_from(M[KM][0], M[KM][1], q0) - q0;
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
            int Bn[2 * KM + 3];
#pragma unroll
            for (int i = 0; i < 2 * KM + 3; i++) Bn[i] = B[i];
            bool hit = false;
#pragma unroll
            for (int d = -KM; d <= KM; d++) {
                if (d < -e || d > e) continue;   // compile-time: the band of row e
                const int i = d + KM + 1;
                const int leftB = B[i - 1], rightB = B[i + 1] + 1, x1B = B[i] + 1;
                const int bxdB = leftB > x1B ? leftB : x1B;
                const int bestB = rightB > bxdB ? rightB : bxdB;
                const int endd = patternLen < textLen - d ? patternLen : textLen - d;
                const int enddB = endd + 2;
                const int mpos = q0m2 + bestB;
                const int mposc = mpos < NBITS ? mpos : NBITS;
                const int fa = ll_first_from(M[d + KM][0], M[d + KM][1], mposc);
                const int fB = fa - q0m2;
                const int slidB = fB < enddB ? fB : enddB;
                const int bnewB = bestB < enddB ? slidB : (fa == mposc ? bestB : enddB);
                Bn[i] = bnewB;
                hit = hit || bnewB == patB;
            }
            if (hit) return e;
#pragma unroll
            for (int i = 0; i < 2 * KM + 3; i++) B[i] = Bn[i];
        }
    }
    return -1;
}

// The reverse LV's masks from the forward ones: reverse diagonal d reads the forward mask of
// x = -d, bit-reversed (lv_pass: mk_reverse, lane li holds x = li - c, d = -x).
template <int KM>
__host__ __device__ __forceinline__ void lv_lane_reverse(uint64_t (&M)[2 * KM + 1][2]) {
    uint64_t R[2 * KM + 1][2];
#pragma unroll
    for (int d = -KM; d <= KM; d++) {
        R[d + KM][0] = ll_brev64(M[-d + KM][1]);
        R[d + KM][1] = ll_brev64(M[-d + KM][0]);
    }
#pragma unroll
    for (int i = 0; i < 2 * KM + 1; i++) { M[i][0] = R[i][0]; M[i][1] = R[i][1]; }
}

}  // namespace sgk
