// align_grouped.h -- batched, lane-grouped scoring for align_kernel<128>.
//
// BaseAligner::score (BaseAligner.cpp:977-1399) scores candidates one at a time
// with scoreLimit shrinking as better hits appear.  Landau-Vishkin with limit k'
// returns exactly what it returns with limit k >= k' when the answer is <= k', and
// -1 otherwise (the row loop is identical up to the answer; LandauVishkin.h:307-449).
// So a batch of candidates can be scored *speculatively* with the scoreLimit current
// at the start of the batch and then applied in the reference's order, clamping each
// result to the scoreLimit in force at that point: bit-exact, and 87% of the LV calls
// of the C2 workload are failures that then never need a backtrace.
//
// One pass scores G = 64/GS candidates at once, one lane group of GS lanes each
// (GS = 16 when k <= 7, 32 when k <= 15, else 64).  Lane `li` of a group holds the
// mismatch bitmap F_x, x = li - (GS/2-1), built from the 2-bit packed genome with
// funnel shifts (16 bases per dword, non-ACGT bases flagged in a spaced mask so a
// byte-exact comparison is kept; reads containing bytes other than ACGTN on a genome
// containing IUPAC codes take the byte path of align_device.h instead).
#pragma once
#include "align_device.h"

namespace sgk {

__device__ __forceinline__ uint32_t packed_code(uint32_t c) {
    return c == 'A' ? 0u : c == 'C' ? 1u : c == 'G' ? 2u : c == 'T' ? 3u : 4u;
}

template <int GS>
__device__ __forceinline__ int from_lower(int v) {   // lane i <- lane i-1 of its group, -2 at the group start
    if constexpr (GS == 16) return __builtin_amdgcn_update_dpp(-2, v, 0x111, 0xf, 0xf, false);   // row_shr:1
    else {
        int r = __shfl_up(v, 1);
        return ((lane_id() & (GS - 1)) == 0) ? -2 : r;
    }
}
template <int GS>
__device__ __forceinline__ int from_upper(int v) {   // lane i <- lane i+1 of its group, -2 at the group end
    if constexpr (GS == 16) return __builtin_amdgcn_update_dpp(-2, v, 0x101, 0xf, 0xf, false);   // row_shl:1
    else {
        int r = __shfl_down(v, 1);
        return ((lane_id() & (GS - 1)) == GS - 1) ? -2 : r;
    }
}

// first mismatch position >= m0 (positions outside [0, 128) count as mismatches); fb: spaced words
__device__ __forceinline__ int fb_first(const uint32_t *fb, int m0) {
    if (m0 >= 128 || m0 < 0) return m0;
    int w = m0 >> 4;
    uint32_t x = fb[w] & (~0u << (2 * (m0 & 15)));
    while (x == 0) {
        if (++w >= 8) return 128;
        x = fb[w];
    }
    return 16 * w + (__builtin_ctz(x) >> 1);
}
// last mismatch position <= m0 (positions outside [0, 128) count as mismatches)
__device__ __forceinline__ int fb_last(const uint32_t *fb, int m0) {
    if (m0 < 0 || m0 >= 128) return m0;
    int w = m0 >> 4;
    uint32_t sh = 2 * (m0 & 15);
    uint32_t x = fb[w] & (sh == 30 ? 0x7fffffffu : ((2u << sh) - 1));
    while (x == 0) {
        if (--w < 0) return -1;
        x = fb[w];
    }
    return 16 * w + ((31 - __builtin_clz(x)) >> 1);
}
__device__ __forceinline__ bool fb_bit(const uint32_t *fb, int m) {
    if (m < 0 || m >= 128) return true;
    return (fb[m >> 4] >> (2 * (m & 15))) & 1;
}

// LandauVishkin<DIR>::computeEditDistance for every active group at once.
// Group-uniform outputs (every lane of a group holds its group's answer).
template <int DIR, int GS>
__device__ __forceinline__ void lv_group(GroupLds &G, bool gact, int p0, int patternLen, int textLen, int k,
                                         int kmaxAll, const char *qual, uint16_t (*rows)[WAVE],
                                         const DevTables *tab, int &outE, double &outP, int &outNet) {
    const int lane = lane_id();
    const int li = lane & (GS - 1), gi = lane / GS, c = GS / 2 - 1;
    const int d = DIR > 0 ? li - c : c - li;
    const uint32_t *fb = G.fb + lane * FBS;
    if (k > MAX_K - 1) k = MAX_K - 1;
    outE = -1; outP = 1.0; outNet = 0;
    bool done = !gact;
    const int end0 = patternLen < textLen ? patternLen : textLen;
    int fm = DIR > 0 ? fb_first(fb, p0) - p0 : p0 - fb_last(fb, p0);
    int v0 = fm < end0 ? fm : end0;
    const int L0 = __shfl(v0, gi * GS + c);
    if (!done && L0 == end0) {   // exact match (LandauVishkin.h:290-305)
        int result = patternLen > end0 ? patternLen - end0 : 0;
        outP = tab->perfect[patternLen];
        outE = result > k ? -1 : result;
        done = true;
    }
    int Lp = (li == c) ? L0 : -2;
    const int endd = patternLen < textLen - d ? patternLen : textLen - d;
    for (int e = 1; e <= kmaxAll; e++) {
        if (!done && e > k) done = true;              // limit reached: -1
        if (ballot(!done) == 0) break;
        const int lower = from_lower<GS>(Lp), upper = from_upper<GS>(Lp);
        const int left = DIR > 0 ? lower : upper;     // L[e-1][d-1]
        const int right = (DIR > 0 ? upper : lower) + 1;   // L[e-1][d+1] + 1
        int best = Lp + 1, act = 0;
        if (left > best) { best = left; act = 1; }
        if (right > best) { best = right; act = 2; }
        const bool active = !done && d <= e && d >= -e;
        if (active) {
            const int mpos = p0 + DIR * best;
            if (best < endd) {
                int f = DIR > 0 ? fb_first(fb, mpos) - p0 : p0 - fb_last(fb, mpos);
                best = f < endd ? f : endd;
            } else if (!fb_bit(fb, mpos)) {
                best = endd;
            }
            rows[e][lane] = (uint16_t)((best + 2) | (act << 12));
        }
        const int Ln = active ? best : Lp;
        const uint64_t hit = ballot(active && Ln == patternLen);
        uint64_t gm;
        if constexpr (GS == 64) gm = hit;
        else gm = (hit >> (gi * GS)) & ((1ull << GS) - 1);
        if (gm != 0 && !done) {
            // first diagonal in the order 0, 1, -1, 2, -2, ... (LandauVishkin.h:180-182)
            int wd = 0;
            for (int j = 0; j <= e; j++) {
                int lp = DIR > 0 ? c + j : c - j, ln = DIR > 0 ? c - j : c + j;
                if ((gm >> lp) & 1) { wd = j; break; }
                if (j > 0 && ((gm >> ln) & 1)) { wd = -j; break; }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            // backtrace (LandauVishkin.h:376-431), group-uniform
            int curD = wd;
            for (int ce = e; ce >= 1; ce--) {
                int ln = gi * GS + (DIR > 0 ? c + curD : c - curD);
                uint32_t cell = rows[ce][ln];
                int a = (int)(cell >> 12);
                int Lcur = (int)(cell & 0xfff) - 2;
                int src = a == 2 ? curD + 1 : (a == 1 ? curD - 1 : curD);
                int ls = gi * GS + (DIR > 0 ? c + src : c - src);
                int Lsrc = (ce - 1 == 0) ? (src == 0 ? L0 : -2) : ((int)(rows[ce - 1][ls] & 0xfff) - 2);
                G.btA[gi][ce] = (int16_t)a;
                G.btM[gi][ce] = (int16_t)(a == 1 ? Lcur - Lsrc : Lcur - Lsrc - 1);
                curD = src;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            double p = 1.0;
            int ce = 1, offset = L0, net = 0;
            while (ce <= e) {
                int a = G.btA[gi][ce];
                int cnt = 1;
                while (ce + 1 <= e && G.btM[gi][ce] == 0 && G.btA[gi][ce + 1] == a) { cnt++; ce++; }
                if (a == 2) { p *= tab->indel[cnt]; offset += cnt; net += cnt; }
                else if (a == 1) { p *= tab->indel[cnt]; offset -= cnt; net -= cnt; }
                else {
                    for (int q = 0; q < cnt; q++) {
                        int qi = offset < 0 ? 0 : offset;
                        if (qi > patternLen - 1) qi = patternLen - 1;
                        p *= tab->phred[(uint8_t)qual[p0 + DIR * qi]];
                        offset++;
                    }
                }
                offset += G.btM[gi][ce];
                ce++;
            }
            p *= tab->perfect[patternLen - e];
            outE = e; outP = p; outNet = net;
            done = true;
        }
        Lp = Ln;
    }
}

}  // namespace sgk
