// align_score.h -- BaseAligner::score (BaseAligner.cpp:977-1399) for the bit-plane kernels
// align_kernel<128> (reads <= 128 bases) and align_kernel<256> (129..256 bases).
//
// Batching.  The reference scores one candidate at a time and scoreLimit shrinks as
// better hits appear.  Landau-Vishkin with limit k' returns exactly what it returns
// with a limit k >= k' when the answer is <= k', and -1 otherwise (the row loop is
// the same up to the answer; LandauVishkin.h:307-449).  So candidates are scored
// speculatively, several per pass, with the scoreLimit current at the start of the
// pass, and then applied in the reference's order, each result clamped to the
// scoreLimit in force at that candidate: bit-exact.
//
// Order.  In forced mode the reference pops the head of the highest non-empty weight
// list until all lists are empty (BaseAligner.cpp:1071-1396); no insertion happens
// meanwhile and scoring never relinks an element, so the pop order is fixed when
// forced mode starts.  A batch pops up to EB elements (selection touches only the
// LDS sort keys), fetches them from the HBM arena in one round trip, lists their
// unscored candidates (element order, then ascending bit, BaseAligner.cpp:1133) and
// scores the list in passes.
//
// One pass scores G = 64/GS candidates, one lane group of GS lanes each (GS = 16
// for k <= 7, 32 for k <= 15, else 64).  Lane `li` of a group holds diagonal
// x = li - (GS/2-1) as a 64*NW-bit mismatch mask in registers (NW = 2 or 4),
//   F_x[m] = read[dir][m] != genome[loc + x + m],
// built from the genome's bit planes (hi, lo, notACGT; 32 bases per dword) with
// funnel shifts; both the forward and the reverse LV read it.  Byte-exact: a base
// that is not ACGT never matches, which equals the byte comparison unless read and
// genome both hold IUPAC codes -- such reads are deferred to align_kernel<512>.
#pragma once
#include "align_device.h"
#include "lv_lane.h"

namespace sgk {

// ------------------------------------------------------------ read-length masks
// Bit m of a mask = mismatch at read position m (NW 64-bit words: 128 positions for
// align_kernel<128>, 256 for align_kernel<256>).  The reverse LV scans the read
// backwards, so it runs on the bit-reversed mask R[m'] = F[NBITS-1 - m'] and both
// directions only need "first set bit at or after m0" (positions >= NBITS count as
// set, which is "before position 0" for R).
template <int NW>
struct MaskW { uint64_t w[NW]; };
using Mask128 = MaskW<2>;

__device__ __forceinline__ uint64_t brev64(uint64_t x) {
    return ((uint64_t)__builtin_bitreverse32((uint32_t)x) << 32) | __builtin_bitreverse32((uint32_t)(x >> 32));
}
template <int NW>
__device__ __forceinline__ MaskW<NW> mk_reverse(const MaskW<NW> &F) {
    MaskW<NW> R;
#pragma unroll
    for (int j = 0; j < NW; j++) R.w[j] = brev64(F.w[NW - 1 - j]);
    return R;
}
// v_ffbl_b32: index of the lowest set bit, 0xffffffff for 0
__device__ __forceinline__ uint32_t ffbl(uint32_t x) {
    uint32_t r;
    asm("v_ffbl_b32 %0, %1" : "=v"(r) : "v"(x));
    return r;
}
// lowest set bit of a 64-bit word, >= 64 (not exactly 64) for 0
__device__ __forceinline__ uint32_t ffb64(uint64_t x) {
    const uint32_t a = ffbl((uint32_t)x), b = ffbl((uint32_t)(x >> 32)) | 32u;
    return a < b ? a : b;
}
// "Not in the word holding m0" answers of mk_first: sfx.s[j] = first set position in words
// j..NW-1 (NBITS if none), for j = 1..NW-1.
template <int NW>
struct MaskSfx { int s[NW]; };
template <int NW>
__device__ __forceinline__ MaskSfx<NW> mk_suffix(const MaskW<NW> &F) {
    MaskSfx<NW> x;
    int acc = 64 * NW;
#pragma unroll
    for (int j = NW - 1; j >= 1; j--) {
        const uint32_t r = ffb64(F.w[j]);
        acc = r < 64u ? 64 * j + (int)r : acc;
        x.s[j] = acc;
    }
    x.s[0] = 0;
    return x;
}
// first set position >= m0, m0 in [0, NBITS]; NBITS if none.  Branch-free: one 64-bit shift of
// the word holding m0 (OR-ing 32 keeps ffbl's 0xffffffff "none").
template <int NW>
__device__ __forceinline__ int mk_first(const MaskW<NW> &F, const MaskSfx<NW> &sf, int m0) {
    constexpr int NBITS = 64 * NW;
    if constexpr (NW == 2) {
        const bool hw = m0 >= 64;
        const uint64_t x = (hw ? F.w[1] : F.w[0]) >> (m0 & 63);
        const uint32_t a = ffbl((uint32_t)x), b = ffbl((uint32_t)(x >> 32)) | 32u;
        const int v = x != 0 ? m0 + (int)(a < b ? a : b) : (hw ? NBITS : sf.s[1]);
        return v < NBITS ? v : NBITS;
    } else {
        const int wi = m0 >> 6;
        uint64_t x = F.w[0];
        int nxt = sf.s[1];
#pragma unroll
        for (int j = 1; j < NW; j++) {
            x = wi >= j ? F.w[j] : x;
            nxt = wi >= j ? (j + 1 < NW ? sf.s[j + 1 < NW ? j + 1 : j] : NBITS) : nxt;
        }
        x >>= (m0 & 63);
        const int v = x != 0 ? m0 + (int)ffb64(x) : nxt;
        return v < NBITS ? v : NBITS;
    }
}

// ------------------------------------------------------------ group shifts
// Biased shifts (value + 2, so the "-2" of a missing neighbour is 0): bound_ctrl makes
// DPP write 0 where the source lane is outside the row, no old-value moves needed.
template <int GS>
__device__ __forceinline__ int from_lower_b(int v, bool gfirst) {
    if constexpr (GS == 16) return __builtin_amdgcn_mov_dpp(v, 0x111, 0xf, 0xf, true);   // row_shr:1
    else if constexpr (GS == 8) {
        const int r = __builtin_amdgcn_mov_dpp(v, 0x111, 0xf, 0xf, true);
        return gfirst ? 0 : r;
    } else {
        const int r = __builtin_amdgcn_mov_dpp(v, 0x138, 0xf, 0xf, true);                 // wave_shr:1
        return gfirst ? 0 : r;
    }
}
template <int GS>
__device__ __forceinline__ int from_upper_b(int v, bool glast) {
    if constexpr (GS == 16) return __builtin_amdgcn_mov_dpp(v, 0x101, 0xf, 0xf, true);   // row_shl:1
    else if constexpr (GS == 8) {
        const int r = __builtin_amdgcn_mov_dpp(v, 0x101, 0xf, 0xf, true);
        return glast ? 0 : r;
    } else {
        const int r = __builtin_amdgcn_mov_dpp(v, 0x130, 0xf, 0xf, true);                 // wave_shl:1
        return glast ? 0 : r;
    }
}

// ------------------------------------------------------------ LV per group
// LandauVishkin<DIR>::computeEditDistance (LandauVishkin.h:211-455) for every active
// group at once, in "forward" coordinates: pattern index i is mask position q0 + i
// (M = F for DIR = 1, M = R with q0 = 127 - p0 for DIR = -1).  Lane li holds
// diagonal d = DIR * (li - c).  Returns the rows run; outE (group-uniform) is the
// distance or -1.  A group that succeeds records its backtrace (LandauVishkin.h:
// 376-431) in G.pa / G.pm / G.pL0 / G.plen[dx]; the match probability is formed
// later, only for candidates the scorer applies (lv_prob).
// UNIFORM_K: every lane's limit k equals the row bound kmaxAll (the forward call), so the
// per-row "limit reached" test is the loop bound.
template <int DIR, int GS, int NW, bool UNIFORM_K = false>
__device__ __forceinline__ int lv_group(GroupLdsT<NW> &G, uint8_t (*rows8)[WAVE], const MaskW<NW> &M, bool gact, int q0,
                                        int patternLen, int textLen, int k, int kmaxAll, int &outE) {
    constexpr int NBITS = 64 * NW;
    constexpr int dx = DIR > 0 ? 0 : 1;
    const int lane = lane_id();
    const int li = lane & (GS - 1), gi = lane / GS, c = GS / 2 - 1;
    const bool gfirst = li == 0, glast = li == GS - 1;   // group boundaries of the row shifts
    const int d = DIR > 0 ? li - c : c - li;
    const int ad = d < 0 ? -d : d;                      // diagonal d is in row e's band iff |d| <= e
    const int pbase = gi * (GS / 2);                     // this group's path slots: rows 1..k, k < GS / 2
    if (k > MAX_K - 1) k = MAX_K - 1;
    outE = -1;
    uint32_t done = gact ? 0u : 1u;   // a VGPR flag: ballot(done == 0) is one v_cmp
    const int end0 = patternLen < textLen ? patternLen : textLen;
    const MaskSfx<NW> hf = mk_suffix(M);
    const int fm = mk_first(M, hf, q0) - q0;
    const int v0 = fm < end0 ? fm : end0;
    const int L0 = shfl_idx(v0, gi * GS + c);           // exact prefix on diagonal 0
    if (!done && L0 == end0) {                          // LandauVishkin.h:290-305
        const int result = patternLen > end0 ? patternLen - end0 : 0;
        outE = result > k ? -1 : result;
        if (li == 0) { G.plen[dx][gi] = 0; G.pL0[dx][gi] = (int16_t)L0; }
        done = 1u;
    }
    // the row loop keeps B = L + 2 (B = 0 for "no value")
    int Bp = (li == c) ? L0 + 2 : 0;
    const int endd = patternLen < textLen - d ? patternLen : textLen - d;
    const int enddB = endd + 2, patB = patternLen + 2, q0m2 = q0 - 2;
    int rowsRun = 0;
    for (int e = 1; e <= kmaxAll; e++) {
        if constexpr (!UNIFORM_K) done = e > k ? 1u : done;   // limit reached: -1
        if (ballot(done == 0u) == 0) break;
        rowsRun = e;
        const int lowerB = from_lower_b<GS>(Bp, gfirst), upperB = from_upper_b<GS>(Bp, glast);
        const int leftB = DIR > 0 ? lowerB : upperB;    // L[e-1][d-1] + 2
        const int rightB = (DIR > 0 ? upperB : lowerB) + 1;   // L[e-1][d+1] + 1 + 2
        const int x1B = Bp + 1;
        // X, then D if strictly greater, then I if strictly greater (only the value is needed here)
        const int bxdB = leftB > x1B ? leftB : x1B;
        const int bestB = rightB > bxdB ? rightB : bxdB;
        const bool active = !done && ad <= e;
        // slide along the diagonal (LandauVishkin.h:325-354)
        const int mpos = q0m2 + bestB;
        const int mposc = mpos < NBITS ? mpos : NBITS;
        const int fa = mk_first(M, hf, mposc);             // fa == mposc <=> mismatch at mpos (or past NBITS-1)
        const int fB = fa - q0m2;
        const int slidB = fB < enddB ? fB : enddB;
        const int bnewB = bestB < enddB ? slidB : (fa == mposc ? bestB : enddB);
        const int LnB = active ? bnewB : Bp;
        if (active) rows8[e][lane] = (uint8_t)bnewB;
        const uint64_t hit = ballot(active && LnB == patB);
        if (hit) {
            const uint64_t gm = GS == 64 ? hit : (hit >> (gi * GS)) & ((1ull << (GS & 63)) - 1);
            if (gm != 0) {
                // first diagonal in the order 0, 1, -1, 2, -2, ... (LandauVishkin.h:180-182)
                int wd = 0;
                for (int j = 0; j <= e; j++) {
                    const int lp = DIR > 0 ? c + j : c - j, ln = DIR > 0 ? c - j : c + j;
                    if ((gm >> lp) & 1) { wd = j; break; }
                    if (j > 0 && ((gm >> ln) & 1)) { wd = -j; break; }
                }
                __asm__ volatile("" ::: "memory");   // the row stores before the backtrace reads (wave_sync)
                // backtrace; the action of a cell is recomputed from the previous row exactly
                // as the row step chose it (X, then D, then I if strictly greater).  L of the
                // current cell is carried (patternLen at the hit); the three cells of row
                // ce-1 around it are adjacent bytes of the row, read with one ds_read2_b32.
                int curD = wd;
                int Lcur = patternLen;
                for (int ce = e; ce >= 1; ce--) {
                    const int r = ce - 1;
                    int vm, v0, vp;   // L[r][curD-1], L[r][curD], L[r][curD+1] as the row step saw them
                    if (r == 0) {
                        vm = curD == 1 ? L0 : -2;
                        v0 = curD == 0 ? L0 : -2;
                        vp = curD == -1 ? L0 : -2;
                    } else {
                        const int i0 = gi * GS + (DIR > 0 ? c + curD - 1 : c - curD - 1);   // lowest byte
                        // the two dwords holding bytes i0..i0+2 of row r, indexed off the row base (an
                        // address rounded through an integer loses its LDS address space: a flat load)
                        const uint32_t *row4 = reinterpret_cast<const uint32_t *>(&rows8[r][0]);
                        const uint64_t w = ((uint64_t)row4[(i0 >> 2) + 1] << 32) | row4[i0 >> 2];   // ds_read2_b32
                        const uint32_t sh = 8u * (uint32_t)(i0 & 3);
                        const int b0 = (int)((w >> sh) & 0xff) - 2, b1 = (int)((w >> (sh + 8)) & 0xff) - 2;
                        const int b2 = (int)((w >> (sh + 16)) & 0xff) - 2;
                        vm = DIR > 0 ? b0 : b2;
                        v0 = b1;
                        vp = DIR > 0 ? b2 : b0;
                        if (curD - 1 < -r || curD - 1 > r) vm = -2;
                        if (curD < -r || curD > r) v0 = -2;
                        if (curD + 1 < -r || curD + 1 > r) vp = -2;
                    }
                    const int x1 = v0 + 1, left = vm;
                    const int right = vp + 1;
                    const int bxd = left > x1 ? left : x1;
                    const int a = right > bxd ? 2 : (left > x1 ? 1 : 0);
                    const int src = a == 2 ? curD + 1 : (a == 1 ? curD - 1 : curD);
                    const int Lsrc = a == 2 ? right - 1 : (a == 1 ? left : x1 - 1);
                    if (li == 0) {
                        G.pa[dx][pbase + ce] = (int8_t)a;
                        G.pm[dx][pbase + ce] = (uint8_t)(a == 1 ? Lcur - Lsrc : Lcur - Lsrc - 1);
                    }
                    curD = src;
                    Lcur = Lsrc;
                }
                if (li == 0) { G.plen[dx][gi] = (int8_t)e; G.pL0[dx][gi] = (int16_t)L0; }
                outE = e;
                done = 1u;
            }
        }
        Bp = LnB;
    }
    return rowsRun;
}

// Match probabilities of the recorded forward and reverse LV paths of group g
// (LandauVishkin.h:376-431), lane-parallel: lanes 0..30 take forward path steps
// 1..31, lanes 32..62 reverse steps.  The reference merges runs of one action
// (continuing while the matched run between them is empty); an indel run gives one
// factor indel[cnt], X steps one phred factor each at offset L0 + sum of earlier
// steps' (+-1 + matched).  Factors are fetched in parallel and multiplied in the
// reference's order (x * 1.0 == x, so steps without a factor multiply by 1.0).
template <int NW>
__device__ __forceinline__ void lv_prob_pair(const DevTables *tab, const GroupLdsT<NW> &G, int g, int pbase, int n, int s0,
                                             int t0, const char *fwdQ, uint32_t rcRead, double &p1, double &p2, int &net2) {
    const int lane = lane_id();
    const int dx = lane >> 5, j = (lane & 31) + 1;               // step j of direction dx
    const int e = G.plen[dx][g];
    const int L0 = G.pL0[dx][g];
    const bool valid = j <= e;
    const int a = valid ? G.pa[dx][pbase + j] : -1;
    const int pmv = valid ? G.pm[dx][pbase + j] : 0;
    const int an = j + 1 <= e ? G.pa[dx][pbase + j + 1] : -2;
    const bool runEnd = valid && (j == e || pmv != 0 || an != a);
    // offset before step j: inclusive scan of delta over the half-wave, minus own delta
    const int delta = valid ? (a == 1 ? -1 : 1) + pmv : 0;
    // inclusive scan over each half-wave in DPP, no LDS round trips: Hillis-Steele inside each
    // 16-lane row, then rows 1 and 3 add the last lane of rows 0 and 2 (row_bcast:15)
    int incl = delta;
    incl += __builtin_amdgcn_update_dpp(0, incl, 0x111, 0xf, 0xf, true);   // row_shr:1
    incl += __builtin_amdgcn_update_dpp(0, incl, 0x112, 0xf, 0xf, true);   // row_shr:2
    incl += __builtin_amdgcn_update_dpp(0, incl, 0x114, 0xf, 0xf, true);   // row_shr:4
    incl += __builtin_amdgcn_update_dpp(0, incl, 0x118, 0xf, 0xf, true);   // row_shr:8
    incl += __builtin_amdgcn_update_dpp(0, incl, 0x142, 0xa, 0xf, false);  // row_bcast:15 into rows 1, 3
    const int offset = L0 + incl - delta;
    // indel run length = distance to the previous run end of this direction
    const uint64_t ends = ballot(runEnd);
    const uint64_t below = (ends >> (lane & 32)) & ((1ull << (lane & 31)) - 1);
    const int prevEnd = below ? 63 - __builtin_clzll(below) : -1;   // lane index within the half
    const int cnt = (lane & 31) - prevEnd;
    const int patternLen = dx ? s0 : n - t0;
    const int p0 = dx ? s0 - 1 : t0;
    int qi = offset < 0 ? 0 : offset;
    if (qi > patternLen - 1) qi = patternLen - 1;
    const int DIR = dx ? -1 : 1;
    double f = 1.0;
    if (valid && a == 0) {   // quality of read[dir] position p: the forward read's, reversed for RC
        const int p = p0 + DIR * qi;
        f = g_tab.phred[(uint8_t)fwdQ[rcRead ? n - 1 - p : p]];
    }
    else if (runEnd) f = g_tab.indel[cnt];
    const double perf = lane == 0 || lane == 32 ? g_tab.perfect[patternLen - e] : 1.0;
    const int e1 = G.plen[0][g], e2 = G.plen[1][g];
    double q = 1.0;
    for (int i = 0; i < e1; i++) q *= readlaned(f, i);
    p1 = q * readlaned(perf, 0);
    q = 1.0;
    for (int i = 0; i < e2; i++) q *= readlaned(f, 32 + i);
    p2 = q * readlaned(perf, 32);
    const uint64_t ins = ballot(valid && dx == 1 && a == 2), del = ballot(valid && dx == 1 && a == 1);
    net2 = __popcll(ins) - __popcll(del);
}

// The same match probabilities for every group of a pass at once, right after its LV calls (verdict
// r5 #2: the factor loads of all the pass's possible successes are issued together, before the
// in-order apply, instead of one success at a time inside it).  Lane l: direction dx = l >> 5, path
// slot sl = l & 31 of group g = sl / S (S = GS / 2 slots per group, G.pa / G.pm layout), step j = sl % S
// (steps 1..e; the slot j = 0 is never a step and its lane leads the segment).  Per segment the
// arithmetic of lv_prob_pair: offsets from a segmented inclusive scan of the step deltas, indel run
// lengths back to the segment's previous run end, one factor per step, multiplied in step order at the
// leader (after i wave_shl:1 moves it holds step i's factor), then the perfect-match factor.  gok: the
// lane's group succeeded in both directions (its paths are recorded); s0 / rcRead: its seed offset and
// direction.  -> leader lanes: qv = product * perfect (lane g*S forward, 32 + g*S reverse); reverse
// leaders: netv = insertions - deletions of the reverse path.
template <int GS, int NW>
__device__ __forceinline__ void lv_prob_groups(const GroupLdsT<NW> &G, bool gok, int n, int s0, int seedLen,
                                               uint32_t rcRead, const char *fwdQ, double &qv, int &netv) {
    constexpr int S = GS / 2;
    const int lane = lane_id();
    const int dx = lane >> 5, sl = lane & 31, g = sl / S, j = sl % S;
    const int e = gok ? (int)G.plen[dx][g] : 0;
    const int L0 = G.pL0[dx][g];
    const bool valid = j >= 1 && j <= e;
    const int a = valid ? G.pa[dx][sl] : -1;
    const int pmv = valid ? G.pm[dx][sl] : 0;
    const int an = valid && j + 1 <= e ? G.pa[dx][sl + 1] : -2;
    const bool runEnd = valid && (j == e || pmv != 0 || an != a);
    const int delta = valid ? (a == 1 ? -1 : 1) + pmv : 0;
    int incl = delta;   // segmented inclusive scan: row shifts masked at the segment start
    { const int t = __builtin_amdgcn_update_dpp(0, incl, 0x111, 0xf, 0xf, true); incl += j >= 1 ? t : 0; }   // row_shr:1
    if constexpr (S > 2) { const int t = __builtin_amdgcn_update_dpp(0, incl, 0x112, 0xf, 0xf, true); incl += j >= 2 ? t : 0; }
    if constexpr (S > 4) { const int t = __builtin_amdgcn_update_dpp(0, incl, 0x114, 0xf, 0xf, true); incl += j >= 4 ? t : 0; }
    if constexpr (S > 8) { const int t = __builtin_amdgcn_update_dpp(0, incl, 0x118, 0xf, 0xf, true); incl += j >= 8 ? t : 0; }
    if constexpr (S > 16) incl += __builtin_amdgcn_update_dpp(0, incl, 0x142, 0xa, 0xf, false);   // row_bcast:15 into rows 1, 3
    const int offset = L0 + incl - delta;
    const uint64_t ends = ballot(runEnd);
    const uint64_t below = (ends >> (lane - j)) & ((1ull << j) - 1) & ~1ull;   // run ends at steps 1..j-1
    const int cnt = j - (below ? 63 - (int)__builtin_clzll(below) : 0);
    const int t0 = s0 + seedLen;
    const int patternLen = dx ? s0 : n - t0;
    const int p0 = dx ? s0 - 1 : t0;
    int qi = offset < 0 ? 0 : offset;
    if (qi > patternLen - 1) qi = patternLen - 1;
    const int DIR = dx ? -1 : 1;
    double f = 1.0;
    if (valid && a == 0) {
        const int p = p0 + DIR * qi;
        f = g_tab.phred[(uint8_t)fwdQ[rcRead ? n - 1 - p : p]];
    } else if (runEnd) f = g_tab.indel[cnt];
    const double perf = j == 0 && gok ? g_tab.perfect[patternLen - e] : 1.0;
    const int emax = (int)max_reduce32((uint32_t)e);
    double q = 1.0;
    uint64_t fb = (uint64_t)__double_as_longlong(f);
    for (int i = 1; i <= emax; i++) {
        const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)fb, 0x130, 0xf, 0xf, false);          // wave_shl:1
        const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(fb >> 32), 0x130, 0xf, 0xf, false);
        fb = ((uint64_t)hi << 32) | lo;
        if (i <= e) q *= __longlong_as_double((long long)fb);
    }
    qv = q * perf;
    constexpr uint64_t SEG = S >= 64 ? ~0ull : (1ull << S) - 1;
    const uint64_t ins = ballot(valid && dx == 1 && a == 2), del = ballot(valid && dx == 1 && a == 1);
    netv = __popcll((ins >> lane) & SEG) - __popcll((del >> lane) & SEG);
}

// Terminal branch of score() (BaseAligner.cpp:1081-1103) + computeMAPQ (mapq.h:32-65).
__device__ __forceinline__ void finalize_read(const KArgs &A, ReadState &st, int *result, uint32_t *flags) {
    st.outScore = (int32_t)st.bestScore;
    if (st.bestScore <= A.maxK) {
        st.outLoc = st.bestLoc;
        const int mq = mapq_dev(A.tab, st.pAll, st.pBest, st.bestScore, sv_get(st, SV_POPULAR), flags);
        st.outMapq = mq;
        *result = mq >= 10 ? SNAPGPU_SINGLE_HIT : SNAPGPU_MULTIPLE_HITS;
    } else {
        *result = (st.nSeedsApplied[0] == 0 && st.nSeedsApplied[1] == 0) ? SNAPGPU_MULTIPLE_HITS : SNAPGPU_NOT_FOUND;
        st.outMapq = 0;
    }
}

// Per-lane pass inputs: this lane's group candidate and its mismatch mask.
struct PassLane {
    uint32_t loc;      // genome location of the candidate (element base + bit)
    int s;             // seed offset
    int glen;          // genome bytes available (BaseAligner.cpp:1161-1185)
    bool act;          // group holds a candidate whose genome window is servable
    int dir;
    uint32_t cw;       // candidate list entry (slot << 8 | bit)
};

// One speculative pass over up to G = 64/GS candidates of the list: group gi takes cand[lvIdx[gi]].
template <int GS, int MAXLEN>
__device__ __forceinline__ void lv_pass(const KArgs &A, Lds<MAXLEN> &S, const Elem64 *ar, const uint16_t *lvIdx, int m, int k,
                                        uint32_t n, PassLane &P, int &e1, int &e2) {
    constexpr int NW = Lds<MAXLEN>::NW;
    GroupLdsT<NW> &G = S.grp[0];
    const int lane = lane_id();
    const int gi = lane / GS, li = lane & (GS - 1), c = GS / 2 - 1;
    PH_T(A, tst);
    P.act = gi < m;
    P.loc = 0; P.s = 0; P.glen = (int)n; P.dir = 0; P.cw = 0;
    if (P.act) {
        const uint32_t cw = G.cand[lvIdx[gi]];
        const uint32_t sl = cand_slot(cw), bit = cand_bit(cw);
        const uint32_t *ec = G.ecache[sl];
        const uint32_t key = ec[6], sp = spill_index(ec[11]);
        P.cw = cw;
        P.loc = (key >> 1) * ELEM + bit;
        P.dir = (int)(key & 1);
        // the candidate's seed offset: the element's inline slots, or its spill block
        P.s = (int)(sp ? (uint32_t)reinterpret_cast<const uint8_t *>(ar + sp)[bit]
                       : slot_offset(ec[12], ec[13], ec[14], ec[15], bit));
        uint32_t glen = n + MAX_K;
        bool ok = substring_ok(A, P.loc, glen);
        if (!ok) {   // BaseAligner.cpp:1163-1185
            uint32_t endOffset = 0;
            bool have = false;
            if ((uint64_t)P.loc + n + MAX_K >= A.nBases) { endOffset = A.nBases; have = true; }
            else {
                const int np = next_piece_after(A, P.loc);
                if (np >= 0) { endOffset = A.pieces[np]; have = true; }
            }
            if (have) {
                glen = endOffset - P.loc - 1;
                if (glen >= n - (uint32_t)MAX_K) ok = substring_ok(A, P.loc, glen);
            }
        }
        P.glen = (int)glen;
        P.act = ok;
    }
    // F_x from the genome bit planes: positions loc + x + [0, 64*NW)
    MaskW<NW> F;
    {
        const int64_t gp = (int64_t)P.loc + (li - c) + PACK_GUARD;
        const GPlane *src = A.gpl + (gp >> 5);
        const uint32_t sh = (uint32_t)gp & 31;
        GPlane w[2 * NW + 1];
#pragma unroll
        for (int j = 0; j < 2 * NW + 1; j++) w[j] = src[j];
        const uint64_t *rp = &G.rpl[P.dir][0][0];
        uint64_t RHw[NW], RLw[NW], RMw[NW];
#pragma unroll
        for (int j = 0; j < NW; j++) { RHw[j] = rp[j]; RLw[j] = rp[NW + j]; RMw[j] = rp[2 * NW + j]; }
        uint32_t f[2 * NW];
#pragma unroll
        for (int j = 0; j < 2 * NW; j++) {
            const uint32_t gh = __builtin_amdgcn_alignbit(w[j + 1].hi, w[j].hi, sh);
            const uint32_t gl = __builtin_amdgcn_alignbit(w[j + 1].lo, w[j].lo, sh);
            const uint32_t gm = __builtin_amdgcn_alignbit(w[j + 1].nm, w[j].nm, sh);
            const uint64_t RH = RHw[j / 2], RL = RLw[j / 2], RM = RMw[j / 2];
            const uint32_t sft = 32 * (j & 1);
            f[j] = (gh ^ (uint32_t)(RH >> sft)) | (gl ^ (uint32_t)(RL >> sft)) | gm | (uint32_t)(RM >> sft);
        }
#pragma unroll
        for (int j = 0; j < NW; j++) F.w[j] = ((uint64_t)f[2 * j + 1] << 32) | f[2 * j];
    }
    PH_ADD(A, S, PH_STAGE, tst);
    PH_T(A, tf);
    const int t = P.s + (int)A.seedLen;
    const int rf = lv_group<1, GS, NW, true>(G, lv_rows(S), F, P.act, t, (int)n - t, P.glen - t, k, k, e1);
    PH_ADD(A, S, PH_LVF, tf);
    PH_CNT(A, S, PH_ROWSF, rf);
    PH_CNT(A, S, GS <= 16 ? PH_NPASS16 : (GS == 32 ? PH_NPASS32 : PH_NPASS64), 1);
    PH_T(A, tr);
    const int k2 = k - e1;
    const bool ract = P.act && e1 >= 0;
    const int kmax2 = (int)max_reduce32(ract ? (uint32_t)(k2 + 1) : 0u) - 1;   // largest reverse limit
    e2 = -1;
    if (kmax2 >= 0) {
        // reverse LV: pattern = read[s-1 .. 0], text = genome backwards from loc+s-1 (BaseAligner.cpp:1216-1220)
        const MaskW<NW> R = mk_reverse(F);
        const int rr = lv_group<-1, GS, NW>(G, lv_rows(S), R, ract, 64 * NW - 1 - (P.s - 1), P.s, P.s + MAX_K, k2,
                                            kmax2, e2);
        PH_CNT(A, S, PH_ROWSR, rr);
    }
    PH_ADD(A, S, PH_LVR, tr);
}

// One LV pass over the candidates that need it and the in-order application of every candidate in
// [i0, iEnd) of the batch's list (BaseAligner.cpp:1129-1384).  lvIdx[0..m) are the positions that
// need LV -- those of unknown distances and those whose filter distances can still succeed at limit
// k -- in list order, and [i0, iEnd) holds exactly those m of them; every other candidate of the
// range has filter distances that fail at any limit <= k (align_score.h forced_filter).  Lane l of a
// 64-position chunk applies position c0 + l with the limit in force at it.  Returns true when the
// read is finished (stopOnFirstHit).  GS is a template parameter so group indexing is shifts and
// the per-group loops unroll.
constexpr int FETCH_NLD = (EB * Elem64::DWORDS + WAVE - 1) / WAVE;   // dwords per lane of a popped batch

// the candidates that need an LV pass at limit k (the test pass_apply and the list gather share)
__device__ __forceinline__ bool cand_needs_lv(uint32_t cw, int k) {
    if (!cand_known(cw)) return true;
    const int a = cand_e1(cw), b = cand_e2(cw);
    return a <= k && b <= k - a;
}

template <int GS, bool EXT, int MAXLEN>
__device__ __forceinline__ bool pass_apply(const KArgs &A, Lds<MAXLEN> &S, Elem64 *ar, ReadState &st, uint32_t i0,
                                           uint32_t iEnd, const uint16_t *lvIdx, int m, int k, uint32_t n, uint32_t nb,
                                           uint32_t &lastSlot, bool &lastSkip, int *result) {
    auto &G = S.grp[0];
    const DevTables *tab = A.tab;
    PassLane P;
    int e1 = -1, e2 = -1;
    P.act = false; P.s = 0;
    double qv = 1.0;   // the groups' match probabilities (lv_prob_groups), at their leader lanes
    int netv = 0;
    uint32_t nbv = NONE;   // lane g: the nearby element of group g's candidate
    if (m > 0) {
        lv_pass<GS, MAXLEN>(A, S, ar, lvIdx, m, k, n, P, e1, e2);
      if (ballot(P.act && e1 >= 0 && e2 >= 0) != 0) {   // (a pass whose LV calls all failed applies no success)
        PH_T(A, tpr);
        // this lane's segment's group: its distances, act, seed offset and direction in one ds_bpermute
        const int gsrc = ((lane_id() & 31) / (GS / 2)) * GS;
        const int gpk = shfl_idx((e1 + 1) | (e2 + 1) << 5 | (P.act ? 1 << 10 : 0) | P.dir << 11 | P.s << 12, gsrc);
        const bool gok = (gpk & 31) != 0 && ((gpk >> 5) & 31) != 0 && ((gpk >> 10) & 1) != 0;
        lv_prob_groups<GS, Lds<MAXLEN>::NW>(G, gok, (int)n, gpk >> 12, (int)A.seedLen, (uint32_t)(gpk >> 11) & 1u, S.fwdQ,
                                            qv, netv);
        PH_ADD(A, S, PH_PROB, tpr);
        PH_T(A, tnb);
        // the nearby element of every group's candidate (BaseAligner.cpp:1272-1331): lane g walks group g's
        // chain, all groups at once (no element is inserted while scoring, so the index stays valid; its
        // header is read at the success, where it may have changed)
        {
            const int gl = lane_id();
            const int src = (gl < 64 / GS ? gl : 0) * GS;
            const uint32_t gloc = (uint32_t)shfl_idx((int)P.loc, src);
            const int gk = shfl_idx((e1 >= 0 && e2 >= 0 && P.act ? 2 : 0) | P.dir, src);
            if (gl < 64 / GS && (gk & 2)) {
                const uint32_t nl = gloc + (2 * (gloc % ELEM / (ELEM / 2)) - 1) * (ELEM / 2);
                nbv = chain_find(A, S, ar, ((nl / ELEM) << 1) | (uint32_t)(gk & 1), (uint32_t)A.arenaElems);
            }
        }
        PH_ADD(A, S, PH_NEARBY, tnb);
      }
    }
    PH_T(A, tapp);
    // ---- apply in order with the limit in force at each candidate.  A failure only sets its scored
    // bit and, for an element's first scored candidate, bestLoc/bestScore/prob (BaseAligner.cpp:
    // 1253-1265 with score -1: nothing else changes), so the failures before the next success are
    // applied together, lane-parallel.
    uint32_t gBase = 0;   // LV groups of the earlier chunks
    for (uint32_t c0 = i0; c0 < iEnd; c0 += WAVE) {
        const int lane = lane_id();   // re-read per chunk: `lane == x` masks are not hoisted and spilled
        const uint32_t p = c0 + (uint32_t)lane;
        const bool have = p < iEnd;
        const uint32_t cw = have ? G.cand[p] : 0u;
        const uint32_t sl = cand_slot(cw), bit = cand_bit(cw);
        const bool lvd = have && cand_needs_lv(cw, k);
        const uint64_t lvm = ballot(lvd);
        const uint32_t g = gBase + (uint32_t)__popcll(lvm & ((1ull << lane) - 1));   // this position's LV group
        const int src = (int)((g * GS) & 63u);
        const int ge1 = shfl_idx(e1, src), ge2 = shfl_idx(e2, src), gact = shfl_idx(P.act ? 1 : 0, src);
        const int re1 = lvd ? ge1 : (cand_e1(cw) == 7 ? -1 : cand_e1(cw));
        const int re2 = lvd ? ge2 : (cand_e2(cw) == 7 ? -1 : cand_e2(cw));
        const bool ract = lvd ? gact != 0 : true;
        gBase += (uint32_t)__popcll(lvm);
        const uint32_t ew11 = have ? G.ecache[sl][11] : 0u;
        const int lastLane = (int)(iEnd - c0 < (uint32_t)WAVE ? iEnd - c0 : (uint32_t)WAVE) - 1;
        for (int g0 = 0; g0 <= lastLane;) {
            const int lane = lane_id();
            const int kNow = (int)(st.scoreLimit < (uint32_t)(MAX_K - 1) ? st.scoreLimit : MAX_K - 1);
            // element lps test, made once when the element's first candidate is reached
            // (BaseAligner.cpp:1129); candidates of one element are contiguous
            const bool skip = sl == lastSlot ? lastSkip : ((ew11 >> 8) & 0xff) > st.scoreLimit;
            const int lim2 = (int)st.scoreLimit - re1 > MAX_K - 1 ? MAX_K - 1 : (int)st.scoreLimit - re1;
            const bool succ = have && !skip && ract && re1 >= 0 && re1 <= kNow && re2 >= 0 && re2 <= lim2;
            const uint64_t sm = ballot(succ && lane >= g0);
            const int ls = sm ? (int)__builtin_ctzll(sm) : lastLane + 1;
            const bool fail = have && !skip && lane >= g0 && lane < ls;
            const uint64_t fm = ballot(fail);
            PH_T(A, tfl);
            if (fm) {
                // An element's candidates are contiguous in the list: its first failing candidate of
                // this step records score -1 if nothing of the element was scored before; every
                // failing candidate ORs its bit into candidatesScored (ds_or_b64).
                const uint32_t prevSl = (uint32_t)shfl_idx((int)sl, lane >= 1 ? lane - 1 : lane);
                uint32_t *ec = G.ecache[sl];
                const bool was0 = fail && (lane == g0 || prevSl != sl) && (ec[2] | ec[3]) == 0;
                if (fail) atomicOr(reinterpret_cast<unsigned long long *>(ec + 2), 1ull << bit);
                if (was0) {
                    ec[9] = (ec[6] >> 1) * ELEM + bit;
                    ec[8] = FAIL_SCORE;
                    ec[4] = 0u;
                    ec[5] = 0u;
                }
                sv_add(st, lane, SV_SCORED, (uint32_t)__popcll(fm));
                wave_sync();
                PH_ADD(A, S, PH_FAILS, tfl);
                PH_CNT(A, S, PH_NFAILSTEP, 1);
            }
            if (ls > lastLane) {
                lastSlot = readlaneu(sl, lastLane);
                lastSkip = readlane(skip ? 1 : 0, lastLane) != 0;
                break;
            }
            lastSlot = readlaneu(sl, ls);
            lastSkip = false;
            PH_T(A, tsu);
            // ---- the success at position lane ls (LV group gs): full bookkeeping (BaseAligner.cpp:1227-1384)
            const uint32_t csl = readlaneu(sl, ls), cbit = readlaneu(bit, ls);
            const int r1 = readlane(re1, ls), r2 = readlane(re2, ls);
            const int gs = readlane((int)g, ls);
            const uint32_t ev = lane < 12 ? G.ecache[csl][lane] : 0u;
            uint64_t cScored = rl64(ev, 2);
            const double cProb = rld(ev, 4);
            const uint32_t cKey = rl(ev, 6), cBest = rl(ev, 8);
            const uint32_t sc = (uint32_t)(r1 + r2);
            PH_CNT(A, S, PH_NSUCC, 1);
            const uint32_t dir = cKey & 1;
            const uint32_t ebase = (cKey >> 1) * ELEM;
            const uint32_t elemLoc = ebase + cbit;
            // the nearby element (BaseAligner.cpp:1272-1331) does not depend on the match probability:
            // found and loaded before lv_prob_pair, so its chain walk and load overlap the product
            uint32_t nbPre;
            int csPre = -1;
            uint32_t nvPre = 0;
            {
                nbPre = readlaneu(nbv, gs);   // (found for every group after the LV pass)
                if (nbPre != NONE) {
                    const uint64_t inb = ballot((uint32_t)lane < nb && G.eidx[lane < EB ? lane : 0] == nbPre);
                    csPre = inb ? (int)__builtin_ctzll(inb) : -1;
                    if (csPre >= 0) nvPre = lane < 12 ? G.ecache[csPre][lane] : 0u;
                    else if (nbPre < ELCAP) nvPre = lane < 12 ? S.eloc[nbPre][lane] : 0u;
                    else nvPre = lane < 12 ? ((const uint32_t *)(ar + nbPre))[lane] : 0u;
                }
            }
            const double q1 = readlaned(qv, gs * (GS / 2)), q2 = readlaned(qv, 32 + gs * (GS / 2));
            const int net2 = readlane(netv, 32 + gs * (GS / 2));
            const double prob = q1 * q2 * tab->seedProb;
            PH_T(A, twt);
            const uint32_t loc = elemLoc + (uint32_t)net2;
            const bool anyNearby0 = cScored != 0;
            cScored |= 1ull << cbit;
            record_hit<EXT>(A, loc, dir, sc);
            sv_add(st, lane, SV_SCORED, 1);
            g0 = ls + 1;
            const bool passA = !(anyNearby0 && (cBest < sc || (cBest == sc && prob <= cProb)));
            bool take = passA;
            uint32_t nb2 = NONE;
            int cs = -1;
            uint32_t nv = 0;
            if (take) { nb2 = nbPre; cs = csPre; nv = nvPre; }
            if (nb2 != NONE) {
                // the nearby element may be in this batch: its cache is authoritative (read above)
                if (rl64(nv, 2) == 0) nb2 = NONE;   // nearby element not scored yet
                if (nb2 != NONE) {
                    const uint32_t nbase = (rl(nv, 6) >> 1) * ELEM;
                    const uint32_t nbl = rl(nv, 9);
                    if (!((nbase > ebase && loc - nbl <= (uint32_t)ELEM) || (nbase < ebase && nbl <= (uint32_t)ELEM)))
                        nb2 = NONE;   // sic: BaseAligner.cpp:1311-1312
                }
                if (nb2 != NONE) {
                    const uint32_t nbs = rl(nv, 8);
                    const double np = rld(nv, 4);
                    if (nbs < sc || (nbs == sc && np >= prob)) take = false;
                    else {
                        st.pAll = st.pAll - np > 0.0 ? st.pAll - np : 0.0;
                        if (cs >= 0) { if (lane == 4 || lane == 5) G.ecache[cs][lane] = 0u; }
                        else if (nb2 < ELCAP) { if (lane == 4 || lane == 5) S.eloc[nb2][lane] = 0u; }
                        else if (lane == 4 || lane == 5) ((uint32_t *)(ar + nb2))[lane] = 0u;
                    }
                }
            }
            // write the element back (scored always; the rest only when taken)
            {
                const uint64_t pb = (uint64_t)__double_as_longlong(prob);
                uint32_t *ec = G.ecache[csl];
                if (lane == 2) ec[2] = (uint32_t)cScored;
                else if (lane == 3) ec[3] = (uint32_t)(cScored >> 32);
                // bestScoreGenomeLocation is set once the candidate passed the first check (:1266-1268)
                if (lane == 9 && passA) ec[9] = loc;
                if (take) {
                    if (lane == 4) ec[4] = (uint32_t)pb;
                    else if (lane == 5) ec[5] = (uint32_t)(pb >> 32);
                    else if (lane == 8) ec[8] = sc;
                }
                wave_sync();
            }
            PH_ADD(A, S, PH_SUCCWB, twt);
            if (!take) { PH_ADD(A, S, PH_SUCC, tsu); continue; }
            st.pAll = st.pAll - cProb > 0.0 ? st.pAll - cProb : 0.0;
            st.pAll += prob;
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
            PH_ADD(A, S, PH_SUCC, tsu);
        }
    }
    PH_ADD(A, S, PH_APPLY, tapp);
    return false;
}

// Forced-mode pop order of a read with many elements: every linked element's (sortkey << 32 |
// index), sorted ascending by an LSD radix sort (4 passes of 8-bit digits; the keys are unique)
// in the free tail of the wave's element arena, with an LDS histogram (the idle LV rows).  The
// pops then read it from the top.  O(n) per pass where the windowed ranks cost O(n^2) per
// 256-element window.  Returns false (rank path) when the arena tail cannot hold two buffers.
template <int MAXLEN>
__device__ __forceinline__ bool forced_sort(const KArgs &A, Lds<MAXLEN> &S, Elem64 *ar, uint32_t nE,
                                            const uint64_t *&sorted, uint32_t &nLinked) {
    // the free slots between the elements and the spill blocks at the arena's top
    if (((uint64_t)A.arenaElems - S.nSpill - nE) * sizeof(Elem64) < 16ull * nE + 64) return false;
    uint64_t *bufA = reinterpret_cast<uint64_t *>(ar + nE), *bufB = bufA + nE;
    uint32_t n = 0, kOr = 0, kAnd = 0xffffffffu;
    for (uint32_t e0 = 0; e0 < nE; e0 += WAVE) {   // linked elements, compacted in index order
        const int lane = lane_id();
        const uint32_t e = e0 + (uint32_t)lane;
        const uint32_t k = e < nE ? sk_get(A, S, ar, e) : 0u;
        const uint64_t m = ballot(k != 0u);
        if (k) bufA[n + (uint32_t)__popcll(m & ((1ull << lane) - 1))] = ((uint64_t)k << 32) | e;
        n += (uint32_t)__popcll(m);
        kOr |= k;
        kAnd &= k ? k : 0xffffffffu;
    }
    // a digit that is the same in every key leaves a stable pass's order unchanged: skip its pass
    // (the keys' timestamp bits above the read's hit count are all ones, and weights fit in 5 bits)
    const uint32_t varying = (uint32_t)or_reduce64(kOr) ^ ~(uint32_t)or_reduce64(~kAnd);   // OR ^ AND
    wave_sync();
    uint32_t *hist = reinterpret_cast<uint32_t *>(&S.u.sc.rows8[0][0]);
    for (int pass = 0; pass < 4; pass++) {
        if (((varying >> (8 * pass)) & 255u) == 0u) continue;
        const int lane = lane_id();
        const int sh = 32 + 8 * pass;
        for (int j = lane; j < 256; j += WAVE) hist[j] = 0u;
        wave_sync();
        for (uint32_t i0 = 0; i0 < n; i0 += WAVE) {
            const uint32_t i = i0 + (uint32_t)lane;
            if (i < n) atomicAdd(&hist[(uint32_t)(bufA[i] >> sh) & 255u], 1u);
        }
        wave_sync();
        // exclusive prefix over the 256 bins, four per lane
        const uint32_t h0 = hist[4 * lane], h1 = hist[4 * lane + 1], h2 = hist[4 * lane + 2], h3 = hist[4 * lane + 3];
        const uint32_t tot = h0 + h1 + h2 + h3;
        uint32_t incl = tot;
#pragma unroll
        for (int o = 1; o < WAVE; o <<= 1) {
            const uint32_t v = (uint32_t)shfl_idx((int)incl, lane >= o ? lane - o : lane);
            if (lane >= o) incl += v;
        }
        const uint32_t base = incl - tot;
        wave_sync();
        hist[4 * lane] = base;
        hist[4 * lane + 1] = base + h0;
        hist[4 * lane + 2] = base + h0 + h1;
        hist[4 * lane + 3] = base + h0 + h1 + h2;
        wave_sync();
        // stable scatter: a lane's place among the lanes of its digit from eight ballots
        for (uint32_t i0 = 0; i0 < n; i0 += WAVE) {
            const int ln = lane_id();
            const uint32_t i = i0 + (uint32_t)ln;
            const bool act = i < n;
            const uint64_t v = act ? bufA[i] : 0ull;
            const uint32_t d = (uint32_t)(v >> sh) & 255u;
            uint64_t peers = ballot(act);
#pragma unroll
            for (int b = 0; b < 8; b++) {
                const uint64_t bb = ballot(act && ((d >> b) & 1u));
                peers &= ((d >> b) & 1u) ? bb : ~bb;
            }
            const uint32_t before = (uint32_t)__popcll(peers & ((1ull << ln) - 1));
            const uint32_t at = act ? hist[d] : 0u;
            wave_sync();
            if (act) bufB[at + before] = v;
            if (act && before == 0) hist[d] = at + (uint32_t)__popcll(peers);
            wave_sync();
        }
        uint64_t *t = bufA; bufA = bufB; bufB = t;
    }
    sorted = bufA;
    nLinked = n;
    return true;
}

// ------------------------------------------------------------ forced-mode prefilter
// In forced mode the pop order is fixed (above) and a repeat-rich read pops hundreds of elements,
// most with one unscored candidate whose LV calls fail: lv_group would spend a pass per 4-8 of them
// just to establish "distance > k".  forced_filter takes the next 32 elements of the order, one per
// lane pair, and computes the distances of each one's first unscored candidate with lv_lane.h
// (lv_pair_dist: a pair's 11 diagonals as 128-bit masks in registers, 6 per lane) at the limit k of
// the moment; at limits 6 and 7 the next 16, one per lane quad (lv_quad_dist: 15 diagonals, 4 masks
// per lane; round 6: forced mode's LV calls at those limits were 5.0 per C2 read and 10.4 per C3 read).  The limit only shrinks, so a distance above it fails at every later limit too: those
// candidates are applied as failures without an LV pass (pass_apply); the rest -- possible successes,
// which need their LV path for the match probability -- still go through lv_group.  Result per lane:
// FRES_VALID | bit | e1 << 8 | e2 << 11 (7: above the limit), 0 when the lane's element has no
// candidate the filter can settle (none unscored, lps above the limit, or a window short of n + MAX_K
// bases at a contig end, whose text bound lv_group handles).
constexpr int FKM = 5;                     // lv_lane.h KM: the pair filter runs at limits k <= 5 (6 and 7 on pairs
                                           // spill more than they save: prefilter_range_r05m.txt); limits 6 and 7
                                           // take the quad form (LQ_K)
constexpr uint32_t FILTER_MIN = 2;         // elements left in the order for a filter pass to pay off
constexpr uint32_t FWIN = WAVE / 2;        // pop-order positions per pair filter pass (a lane pair each; quads: FWIN / 2)
constexpr uint32_t FRES_VALID = 1u << 31;

// QUAD: one candidate per lane quad (lv_quad_dist, limits 6 and 7: 16 positions per pass), else per lane
// pair (lv_pair_dist, limits <= 5: 32 positions).  Distances above the limit are encoded 7; at limit 7 a
// 7 is also an exact distance, which cand_needs_lv still sends through lv_group (7 <= k), so the
// encoding stays sound: a candidate it lets fail without LV has e1 > k or e2 > k - e1.
template <int MAXLEN, bool QUAD>
__device__ __forceinline__ uint32_t forced_filter(const KArgs &A, Lds<MAXLEN> &S, const Elem64 *ar, const ReadState &st,
                                                  uint32_t n, const uint64_t *fSorted, uint32_t fAvail,
                                                  const uint16_t *order, uint32_t ordBase, uint32_t pos0, uint32_t cnt,
                                                  int k) {
    static_assert(Lds<MAXLEN>::NW == 2, "forced_filter: 128-bit masks");
    constexpr int LPC = QUAD ? 4 : 2;          // lanes per candidate
    constexpr int NM = QUAD ? 4 : FKM + 1;     // masks per lane
    constexpr int KB = QUAD ? LQ_K : FKM;      // the window starts at loc - KB
    const int lane = lane_id();
    const int c = lane / LPC, h = lane % LPC;  // lanes LPC*c .. take pop-order position pos0 + c
    const uint32_t pos = pos0 + (uint32_t)c;
    bool act = (uint32_t)c < cnt;
    uint32_t e = 0;
    if (act) e = fSorted ? (uint32_t)fSorted[fAvail - 1 - pos] : (uint32_t)order[pos - ordBase];
    // the header words it needs: used, scored (dw 0-3), key (6), w11 (11), the slots (12-15)
    uint4 h0 = make_uint4(0u, 0u, 0u, 0u), h3 = h0;
    uint32_t key = 0, w11 = 0;
    if (act) {
        const uint32_t *hp = e < ELCAP ? S.eloc[e < ELCAP ? e : 0] : reinterpret_cast<const uint32_t *>(ar + e);
        h0 = reinterpret_cast<const uint4 *>(hp)[0];
        key = hp[6];
        w11 = hp[11];
        h3 = reinterpret_cast<const uint4 *>(hp)[3];
    }
    const uint64_t pend = (((uint64_t)h0.y << 32) | h0.x) & ~(((uint64_t)h0.w << 32) | h0.z);
    act = act && pend != 0 && ((w11 >> 8) & 0xffu) <= st.scoreLimit;
    const uint32_t bit = act ? (uint32_t)__builtin_ctzll(pend) : 0u;
    const uint32_t loc = (key >> 1) * ELEM + bit, dir = key & 1u;
    const uint32_t sp = spill_index(w11);
    int s = 0;
    if (act) s = (int)(sp ? (uint32_t)reinterpret_cast<const uint8_t *>(ar + sp)[bit] : slot_offset(h3.x, h3.y, h3.z, h3.w, bit));
    act = act && substring_ok(A, loc, n + MAX_K);
    // this lane's masks, F_x[m] = read[dir][m] != genome[loc + x + m] on the bit planes: pair half h holds
    // forward diagonal x = h ? i : -i at local i; quad lane h holds x = 4h + i - LQ_K at local i
    uint64_t F[NM][2];
    {
        const int64_t gp = (int64_t)loc - KB + PACK_GUARD;
        const GPlane *src = A.gpl + (act ? (gp >> 5) : 0);
        const uint32_t sh = (uint32_t)gp & 31;
        uint32_t wh[6], wl[6], wm[6];
#pragma unroll
        for (int j = 0; j < 6; j++) {
            const GPlane w = src[j];
            wh[j] = w.hi; wl[j] = w.lo; wm[j] = w.nm;
        }
        uint32_t ah[5], al[5], am[5];   // the genome planes from position loc - KB, 160 bits
#pragma unroll
        for (int j = 0; j < 5; j++) {
            ah[j] = __builtin_amdgcn_alignbit(wh[j + 1], wh[j], sh);
            al[j] = __builtin_amdgcn_alignbit(wl[j + 1], wl[j], sh);
            am[j] = __builtin_amdgcn_alignbit(wm[j + 1], wm[j], sh);
        }
        const uint64_t *rp = &S.grp[0].rpl[dir][0][0];
        uint32_t rh[4], rl_[4], rm[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            rh[j] = (uint32_t)(rp[j / 2] >> (32 * (j & 1)));
            rl_[j] = (uint32_t)(rp[2 + j / 2] >> (32 * (j & 1)));
            rm[j] = (uint32_t)(rp[4 + j / 2] >> (32 * (j & 1)));
        }
#pragma unroll
        for (int i = 0; i < NM; i++) {   // the window shifted by KB + x bits
            const uint32_t cs = QUAD ? (uint32_t)(4 * h + i) : (uint32_t)(h ? FKM + i : FKM - i);
            uint32_t f[4];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const uint32_t gh = __builtin_amdgcn_alignbit(ah[j + 1], ah[j], cs);
                const uint32_t gl = __builtin_amdgcn_alignbit(al[j + 1], al[j], cs);
                const uint32_t gm = __builtin_amdgcn_alignbit(am[j + 1], am[j], cs);
                f[j] = (gh ^ rh[j]) | (gl ^ rl_[j]) | gm | rm[j];
            }
            F[i][0] = ((uint64_t)f[1] << 32) | f[0];
            F[i][1] = ((uint64_t)f[3] << 32) | f[2];
        }
    }
    const int t = s + (int)A.seedLen;
    int e1, e2 = -1;
    if constexpr (QUAD) e1 = lv_quad_dist<1>(F, h, act, t, (int)n - t, (int)n + MAX_K - t, k);
    else e1 = lv_pair_dist<FKM, 1>(F, h, act, t, (int)n - t, (int)n + MAX_K - t, k);
    if (ballot(e1 >= 0)) {
        // reverse LV: pattern = read[s-1 .. 0], text = genome backwards from loc + s - 1 (BaseAligner.cpp:1216-1220)
        if constexpr (QUAD) e2 = lv_quad_dist<-1>(F, h, e1 >= 0, 127 - (s - 1), s, s + MAX_K, k - e1);
        else e2 = lv_pair_dist<FKM, -1>(F, h, e1 >= 0, 127 - (s - 1), s, s + MAX_K, k - e1);
    }
    return act ? FRES_VALID | bit | (uint32_t)(e1 < 0 ? 7 : e1) << 8 | (uint32_t)(e2 < 0 ? 7 : e2) << 11 : 0u;
}

// BaseAligner::score (BaseAligner.cpp:977-1399) over batches of popped elements.
template <bool EXT, int MAXLEN>
__device__ __forceinline__ bool score_batched(const KArgs &A, Lds<MAXLEN> &S, Elem64 *ar, ReadState &st, bool force,
                                           uint32_t n, int *result, uint32_t *flags) {
    const int lane = lane_id();
    auto &G = S.grp[0];
    const DevTables *tab = A.tab;
    for (int d = 0; d < 2; d++)
        if (st.mostSeeds[d]) {
            const uint32_t v = uni(st.nSeedsApplied[d] / st.mostSeeds[d]);   // (VALU division: back to an SGPR)
            if (v > st.lps[d]) st.lps[d] = v;
        }
    const uint32_t minLps = st.lps[0] < st.lps[1] ? st.lps[0] : st.lps[1];
    const bool forced = force || minLps > st.scoreLimit;
    PH_CNT(A, S, PH_NSCORECALL, 1);
    PH_CNT(A, S, PH_NFORCED, forced ? 1 : 0);
    // Forced mode pops every linked element in descending sort-key order and the read
    // ends with it, so the order is computed once (ranks, ORDCAP at a time) and the
    // elements are not unlinked one by one.
    uint16_t *order = S.u.sc.order;
    uint32_t fDone = 0, fAvail = 0, ordBase = 0;
    bool fMore = true;   // a ranking window came back full: elements of lower rank may remain
    const uint64_t *fSorted = nullptr;   // radix-sorted pop order (reads with >= A.radixMin elements)
    // forced_filter's window over pop-order positions [wBase, wEnd): lanes j << fShift .. hold position wBase + j
    uint32_t fres = 0, wBase = 0, wEnd = 0, fShift = 1;   // fShift: log2 of the lanes per position (pairs 1, quads 2)
    for (uint32_t guard = 0;; guard++) {
        // lane id re-read per batch (volatile asm): masks and addresses derived from it are
        // recomputed in the batch instead of hoisted and kept live, spilled, across the pass loop
        const int lane = lane_id();
        if (guard > (uint32_t)A.arenaElems) {   // every batch unlinks >= 1 element
            if (lane == 0) diag_report(A.diag, DIAG_SCORE_LOOP, st.rid, S.nElems);
            st.abort = 1;
        }
        if (overdue(A, st, 1)) return true;
        PH_T(A, tpop);
        // ---- pop in weight-list order (head of the highest list first); LDS only
        uint32_t nb = 0, posb = 0;   // batch size, its first pop-order position (forced mode)
        if (!forced) {
            // sort keys are unique: reduce the 32-bit keys, then take the owner lane's index
            const uint64_t lm = S.laneMax[lane];
            const uint32_t kmax = max_reduce32((uint32_t)(lm >> 32));
            if (kmax != 0) {
                const int owner = (int)__builtin_ctzll(ballot((uint32_t)(lm >> 32) == kmax));
                const uint32_t e = readlaneu((uint32_t)lm, owner);
                sk_set(A, S, ar, e, 0);                       // unlink (BaseAligner.cpp:1391-1394)
                wave_sync();
                recompute_lane_max(A, S, ar, owner);
                if (lane == 0) G.eidx[0] = e;
                nb = 1;
                wave_sync();
            }
        } else {
            if (fDone == 0 && !fSorted && S.nElems >= A.radixMin) {
                PH_T(A, trs);
                uint32_t nl = 0;
                if (forced_sort<MAXLEN>(A, S, ar, S.nElems, fSorted, nl)) { fAvail = nl; fMore = false; }
                PH_ADD(A, S, PH_RANK, trs);
            }
            if (fDone == fAvail && fMore) {
                PH_T(A, trk);
                PH_CNT(A, S, PH_NELEMSF, fDone == 0 ? S.nElems : 0);
                // rank[e] = number of linked elements with a larger key (keys are unique).  The
                // keys of elements >= SKCAP are staged from the arena into LDS a block at a time
                // (the LV rows are idle here), so every lane compares against broadcast LDS reads.
                ordBase = fDone;
                const uint32_t nE = S.nElems;
                const uint32_t nL = nE < SKCAP ? nE : SKCAP;
                uint32_t *stage = reinterpret_cast<uint32_t *>(&S.u.sc.rows8[0][0]);
                uint32_t inRange = 0;
                for (uint32_t e0 = 0; e0 < nE; e0 += WAVE) {
                    const uint32_t e = e0 + lane;
                    const uint32_t ke = e < nE ? sk_get(A, S, ar, e) : 0u;
                    uint32_t rank = 0;
                    uint32_t f = 0;
                    for (; f + 4 <= nL; f += 4) {
                        const uint4 k4 = *reinterpret_cast<const uint4 *>(&S.sk[f]);
                        rank += (k4.x > ke) + (k4.y > ke) + (k4.z > ke) + (k4.w > ke);
                    }
                    for (; f < nL; f++) rank += S.sk[f] > ke;
                    for (uint32_t b0 = SKCAP; b0 < nE; b0 += SKCAP) {
                        const uint32_t nk = nE - b0 < SKCAP ? nE - b0 : SKCAP;
                        wave_sync();
                        for (uint32_t j = lane; j < ((nk + 3) & ~3u); j += WAVE) stage[j] = j < nk ? sk_get(A, S, ar, b0 + j) : 0u;
                        wave_sync();
                        for (uint32_t g = 0; g < nk; g += 4) {
                            const uint4 k4 = *reinterpret_cast<const uint4 *>(&stage[g]);
                            rank += (k4.x > ke) + (k4.y > ke) + (k4.z > ke) + (k4.w > ke);
                        }
                    }
                    const bool in = ke != 0 && rank >= ordBase && rank < ordBase + Lds<MAXLEN>::ORD;
                    if (in) order[rank - ordBase] = (uint16_t)e;
                    inRange += (uint32_t)__popcll(ballot(in));
                }
                fAvail = ordBase + inRange;
                fMore = inRange == Lds<MAXLEN>::ORD;
                wave_sync();
                PH_ADD(A, S, PH_RANK, trk);
            }
            if constexpr (Lds<MAXLEN>::NW == 2) {
                const int kf = st.scoreLimit < (uint32_t)(MAX_K - 1) ? (int)st.scoreLimit : MAX_K - 1;
                if (fDone >= wEnd && kf <= LQ_K && fAvail - fDone >= FILTER_MIN) {
                    const bool quad = kf > FKM;
                    const uint32_t fw = quad ? FWIN / 2 : FWIN;
                    const uint32_t cnt = fAvail - fDone < fw ? fAvail - fDone : fw;
                    if (quad) fres = forced_filter<MAXLEN, true>(A, S, ar, st, n, fSorted, fAvail, order, ordBase, fDone, cnt, kf);
                    else fres = forced_filter<MAXLEN, false>(A, S, ar, st, n, fSorted, fAvail, order, ordBase, fDone, cnt, kf);
                    fShift = quad ? 2u : 1u;
                    wBase = fDone;
                    wEnd = fDone + cnt;
                    PH_CNT(A, S, PH_NFILTER, 1);
#if SNAPGPU_PHASE_TIMERS
                    const uint32_t nfr = (uint32_t)__popcll(ballot((fres & FRES_VALID) != 0u)) >> fShift;
                    PH_CNT(A, S, PH_NFRES, nfr);
#endif
                }
            }
            posb = fDone;
            nb = fAvail - fDone < (uint32_t)EB ? fAvail - fDone : (uint32_t)EB;
            if ((uint32_t)lane < nb)
                G.eidx[lane] = fSorted ? (uint32_t)fSorted[fAvail - 1 - (fDone + (uint32_t)lane)]
                                       : (uint32_t)order[fDone - ordBase + lane];
            fDone += nb;
            wave_sync();
        }
        if (nb == 0) {
            PH_ADD(A, S, PH_POP, tpop);
            if (forced) { finalize_read(A, st, result, flags); return true; }
            return false;
        }
        PH_ADD(A, S, PH_SEL, tpop);
        PH_T(A, tfe);
        // ---- fetch the batch from the arena in one round trip.  (Loading the next forced batch
        // during this one's passes measured 1% slower: the 9 VGPRs it holds across the pass loop,
        // profiles/r03/ab/micro_opts_ab.txt.)
        {
            constexpr int ED = Elem64::DWORDS;
            const uint32_t tot = nb * ED;
            uint32_t v[FETCH_NLD];
#pragma unroll
            for (int j = 0; j < FETCH_NLD; j++) {
                const uint32_t idx = (uint32_t)(j * WAVE + lane);
                const uint32_t e = idx < tot ? G.eidx[idx / ED] : 0u;
                v[j] = idx >= tot ? 0u : (e < ELCAP ? S.eloc[e][idx % ED] : ((const uint32_t *)(ar + e))[idx % ED]);
            }
#pragma unroll
            for (int j = 0; j < FETCH_NLD; j++) {
                const uint32_t idx = (uint32_t)(j * WAVE + lane);
                if (idx < tot) G.ecache[idx / ED][idx % ED] = v[j];
            }
            wave_sync();
        }
        PH_ADD(A, S, PH_FETCH, tfe);
        // ---- candidate list: elements in pop order, ascending bit; lane sl owns element sl
        PH_CNT(A, S, PH_NBATCH, 1);
        PH_T(A, tcl);
        uint32_t nc;
        {
            uint64_t pend = 0;
            if ((uint32_t)lane < nb) {
                const uint32_t *ec = G.ecache[lane];
                if (((ec[11] >> 8) & 0xff) <= st.scoreLimit)   // cannot be scored (the limit only shrinks)
                    pend = (((uint64_t)ec[1] << 32) | ec[0]) & ~(((uint64_t)ec[3] << 32) | ec[2]);
            }
            const uint32_t cnt = (uint32_t)__popcll(pend);
            // the filter's result for this element (pop-order position posb + lane), if in its window
            const uint32_t wl = posb + (uint32_t)lane - wBase;
            const uint32_t fr = (uint32_t)shfl_idx((int)fres, (int)((wl << fShift) & 63u));
            const bool inWin = forced && posb + (uint32_t)lane >= wBase && posb + (uint32_t)lane < wEnd &&
                               (uint32_t)lane < nb && (fr & FRES_VALID);
            const uint32_t known = inWin ? (1u << 9) | ((fr >> 8) & 7u) << 10 | ((fr >> 11) & 7u) << 13 : 0u;
            const uint32_t kbit = fr & 63u;
            // exclusive prefix sum over lanes 0..EB-1
            uint32_t pos = 0;
#pragma unroll
            for (int j = 0; j < EB; j++) {
                const uint32_t cj = (uint32_t)__builtin_amdgcn_readlane((int)cnt, j);
                if (j < lane) pos += cj;
            }
            nc = (uint32_t)__builtin_amdgcn_readlane((int)(pos + cnt), EB - 1);
            while (pend) {
                const int bit = __builtin_ctzll(pend);
                pend &= pend - 1;
                G.cand[pos++] = (uint16_t)((uint32_t)bit | (uint32_t)lane << 6 | ((uint32_t)bit == kbit ? known : 0u));
            }
            wave_sync();
        }
        PH_ADD(A, S, PH_CANDL, tcl);
        PH_ADD(A, S, PH_POP, tpop);
        PH_CNT(A, S, PH_NCAND, nc);
        PH_CNT(A, S, PH_NPOPPED, nb);
        PH_T(A, tpl);
        uint32_t lastSlot = NONE;   // element of the last candidate reached, and its lps decision
        bool lastSkip = false;
        // the LV list of a pass (positions into cand, list order) in an LV row the scorer never
        // reaches at the limits that fill it (k <= 15 uses rows 1..15)
        uint16_t *lvIdx = reinterpret_cast<uint16_t *>(&S.u.sc.rows8[MAX_K - 2][0]);
        for (uint32_t i0 = 0; i0 < nc;) {
            if (overdue(A, st, 2)) return true;
            const int k = st.scoreLimit < (uint32_t)(MAX_K - 1) ? (int)st.scoreLimit : MAX_K - 1;
            const int GS = k <= 3 ? 8 : (k <= 7 ? 16 : (k <= 15 ? 32 : 64));
            const int Gn = 64 / GS;
            // the next Gn candidates that need LV (unknown distances, or filter distances that can still
            // succeed at k); the pass applies everything up to the last of them (the end when fewer)
            int m = 0;
            for (uint32_t c0 = i0; c0 < nc && m < Gn; c0 += WAVE) {
                const int lane = lane_id();
                const uint32_t p = c0 + (uint32_t)lane;
                const bool need = p < nc && cand_needs_lv(G.cand[p], k);
                const uint64_t nm = ballot(need);
                const int r = m + __popcll(nm & ((1ull << lane) - 1));
                if (need && r < Gn) lvIdx[r] = (uint16_t)p;
                m += __popcll(nm);
                m = m < Gn ? m : Gn;
            }
            wave_sync();
            const uint32_t iEnd = m == Gn ? (uint32_t)lvIdx[Gn - 1] + 1u : nc;
            if (m > 0) {
                PH_CNT(A, S, PH_NPASS, 1);
                if (forced) PH_CNT(A, S, PH_NPASSF, 1);
#if SNAPGPU_PHASE_TIMERS
                if (forced) {   // LV'd candidates of forced passes, and those with filter distances (possible successes)
                    const int ln = lane_id();
                    const uint32_t lp = lvIdx[ln < m ? ln : 0];
                    const uint32_t cwl = G.cand[lp];
                    const bool second = lp > 0 && cand_slot(G.cand[lp - 1]) == cand_slot(cwl);
                    const uint32_t nk = (uint32_t)__popcll(ballot(ln < m && cand_known(cwl)));
                    const uint32_t nu = (uint32_t)__popcll(ballot(ln < m && !cand_known(cwl) && k <= FKM));
                    const uint32_t n2 = (uint32_t)__popcll(ballot(ln < m && !cand_known(cwl) && second));
                    PH_CNT(A, S, PH_NLVF, m);
                    PH_CNT(A, S, PH_NLVFK, nk);
                    PH_CNT(A, S, PH_NLVFU, nu);
                    PH_CNT(A, S, PH_NLVF2, n2);
                }
#endif
            }
            bool fin;
            if (GS == 8) fin = pass_apply<8, EXT>(A, S, ar, st, i0, iEnd, lvIdx, m, k, n, nb, lastSlot, lastSkip, result);
            else if (GS == 16) fin = pass_apply<16, EXT>(A, S, ar, st, i0, iEnd, lvIdx, m, k, n, nb, lastSlot, lastSkip, result);
            else if (GS == 32) fin = pass_apply<32, EXT>(A, S, ar, st, i0, iEnd, lvIdx, m, k, n, nb, lastSlot, lastSkip, result);
            else fin = pass_apply<64, EXT>(A, S, ar, st, i0, iEnd, lvIdx, m, k, n, nb, lastSlot, lastSkip, result);
            if (fin) return true;
            i0 = iEnd;
        }
        PH_ADD(A, S, PH_PASSLOOP, tpl);
        if (forced) { PH_ADD(A, S, PH_PASSLOOPF, tpl); PH_CNT(A, S, PH_NCANDF, nc); }
        PH_T(A, twb);
        // ---- write the batch back (scored, prob, bestScore, bestLoc, allScored = 1)
        for (uint32_t idx = lane; idx < nb * 8; idx += WAVE) {
            const uint32_t sl = idx >> 3, f = idx & 7;
            const uint32_t dw = f < 4 ? 2 + f : (f == 4 ? 8 : (f == 5 ? 9 : 11));
            if (f < 7) {
                uint32_t w = G.ecache[sl][dw];
                if (dw == 11) w |= W11_ALLSCORED;   // (the spill index above it stays)
                const uint32_t e = G.eidx[sl];
                if (e < ELCAP) S.eloc[e][dw] = w;
                else ((uint32_t *)(ar + e))[dw] = w;
            }
        }
        wave_sync();
        PH_ADD(A, S, PH_WB, twb);
        if (!forced) return false;
    }
}

}  // namespace sgk
