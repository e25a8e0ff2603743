// cigar.h -- CIGAR strings of aligned reads on the GPU.
//
// What the reference's SAM writer computes per aligned read on the host
// (SAMFormat::writeRead -> computeCigarString, SNAPLib/SAM.cpp:1007-1230):
// LandauVishkinWithCigar::computeEditDistance (SNAPLib/LandauVishkin.cpp:252-535)
// of the read -- reverse-complemented for RC alignments (getSAMData,
// SAM.cpp:866-883) -- against the genome substring at the alignment location,
// with k = MAX_K - 1.  Out: the edit distance (the SAM NM tag) and the CIGAR as
// BAM ops (count << 4 | code, code index into "MIDNSHP=X").
//
// One wave per read.  Lane l holds diagonal d = l - 31 (|d| <= 30 fits 61 lanes),
// so one LV row is computed in parallel: the reference visits diagonals in the
// order 0, -1, +1, -2, ... but a row only reads the previous row, so the parallel
// row is the same row; among the diagonals of the first row that reach the end
// of the read, the first one in the reference's order is taken.  Rows (L and the
// chosen action) are kept in LDS for the backtrace, which, like the emission of
// the ops (run merging, useM accumulation), is wave-uniform scalar code.  The read
// and a genome window [loc - 32, loc + len + 96) are staged in LDS; a diagonal's
// slide compares 4 bytes per step (two aligned LDS words + v_alignbyte).
#pragma once
#include "align_device.h"

namespace sgk {

constexpr int CIG_MAXLEN = 512;          // reads longer than this are rejected on the host
constexpr int CIG_MAX_OPS = 64;          // SNAPGPU_CIGAR_MAX_OPS: 2 * 30 + 1 ops at most
constexpr int CIG_K = MAX_K - 1;         // computeCigarString passes MAX_K - 1 (SAM.cpp:1185)

struct CigarArgs {
    // genome (HBM, >= 1 KiB guard each side) and its pieces, for Genome::getSubstring
    const char *genome;
    const uint32_t *pieces;
    int32_t nPieces;
    uint32_t nBases, padding;
    // reads
    const char *bases;
    const uint64_t *offsets;
    const uint32_t *lengths;
    uint32_t nReads;
    // per read: either AlignRead's records (SAM rules of getSAMData) or explicit
    // (location, pattern direction) pairs
    const snapgpu_result_t *records;
    const uint32_t *locations;
    const uint8_t *directions;
    int useM;
    int32_t *outEd;                      // [n]
    uint32_t *outNOps;                   // [n]
    uint32_t *outOps;                    // [n][CIG_MAX_OPS]
};

struct CigarLds {
    uint32_t pat[(CIG_MAXLEN + 16) / 4];     // oriented read, zero slack (the reference's 8-byte compares)
    uint32_t txt[(CIG_MAXLEN + 128) / 4];    // genome bytes [tStart, tStart + 4 * 160)
    int16_t L[MAX_K][WAVE];                  // LV rows 0..30, lane = diagonal + 31
    uint8_t A[MAX_K][WAVE];                  // action that produced L: 0 'X', 1 'D', 2 'I'
    uint64_t mm[CIG_MAXLEN / 64];            // diagonal-0 mismatch bits (straight alignment)
    int32_t btA[MAX_K + 1], btM[MAX_K + 1];  // backtraceAction / backtraceMatched
    uint32_t ops[CIG_MAX_OPS];
};

__device__ __forceinline__ uint32_t cig_ld4(const uint32_t *w, int i) {   // bytes [i, i+4) of a word array
    return __builtin_amdgcn_alignbyte(w[(i >> 2) + 1], w[i >> 2], (uint32_t)(i & 3));
}
__device__ __forceinline__ uint32_t cig_byte(const uint32_t *w, int i) { return (w[i >> 2] >> ((i & 3) * 8)) & 0xffu; }

// Read::init's TO_UPPER_CASE (Tables.cpp:74-80) then COMPLEMENT (Tables.cpp:22-30; 0 for other bytes)
__device__ __forceinline__ uint32_t cig_upper(uint32_t c) { return (c >= 'a' && c <= 'z') ? c - 0x20 : c; }
__device__ __forceinline__ uint32_t cig_comp(uint32_t c) {
    switch (c) {
        case 'A': return 'T';
        case 'C': return 'G';
        case 'G': return 'C';
        case 'T': return 'A';
        case 'N': return 'N';
        case 'n': return 'n';
        default: return 0;
    }
}

// next position >= i whose diagonal-0 mismatch bit equals `want`, or len
__device__ __forceinline__ int cig_next_bit(const CigarLds &S, int i, int len, bool want) {
    for (int c = i >> 6; c * 64 < len; c++) {
        uint64_t w = S.mm[c];
        if (!want) w = ~w;
        if (c == (i >> 6)) w &= ~0ull << (i & 63);
        if (w) {
            const int p = c * 64 + __builtin_ctzll(w);
            return p < len ? p : len;
        }
    }
    return len;
}

__global__ __launch_bounds__(64) void cigar_kernel(CigarArgs A) {
    __shared__ CigarLds S;
    const int l = lane_id();
    const int d = l - 31;                        // this lane's diagonal
    const uint32_t *pat = S.pat;
    for (uint32_t r = blockIdx.x; r < A.nReads; r += gridDim.x) {
        const uint32_t len = A.lengths[r];
        uint32_t loc;
        int rc;
        if (A.records) {
            // getSAMData (SAM.cpp:855-883): NotFound or no location -> FORWARD data; the
            // CIGAR is still computed at writeRead's own location (SAM.cpp:1041-1048)
            const snapgpu_result_t &rec = A.records[r];
            loc = rec.location;
            rc = (rec.result != SNAPGPU_NOT_FOUND && loc != 0xffffffffu) ? rec.direction : 0;
        } else {
            loc = A.locations[r];
            rc = A.directions[r];
        }
        uint32_t nOps = 0;
        int ed = -1;
        if (loc != 0xffffffffu && len <= (uint32_t)CIG_MAXLEN && substring_ok(A, loc, len)) {
            // ---- stage the oriented read and the genome window
            const char *rb = A.bases + A.offsets[r];
            for (int w = l; w < (CIG_MAXLEN + 16) / 4; w += WAVE) {
                uint32_t v = 0;
                for (int j = 0; j < 4; j++) {
                    const int i = 4 * w + j;
                    uint32_t c = 0;
                    if (i < (int)len) {
                        c = cig_upper((uint8_t)rb[rc ? len - 1 - i : i]);
                        if (rc) c = cig_comp(c);
                    }
                    v |= c << (8 * j);
                }
                S.pat[w] = v;
            }
            const int64_t t0 = (int64_t)loc - 32;
            const int64_t ta = t0 & ~(int64_t)3;
            const int tOff = (int)(t0 - ta) + 32;    // text position j lives at byte j + tOff
            const uint32_t *src = reinterpret_cast<const uint32_t *>(A.genome + ta);
            const int nw = ((int)len + 128) / 4;
            for (int w = l; w < nw && w < (CIG_MAXLEN + 128) / 4; w += WAVE) S.txt[w] = src[w];
            wave_sync();
            const uint32_t *txt = S.txt;
            // ---- diagonal 0: exact prefix (L[0][0]) and the straight mismatch count
            int L0 = (int)len, straight = 0;
            for (int c = 0; c * 64 < (int)len; c++) {
                const int i = c * 64 + l;
                const bool mis = i < (int)len && cig_byte(pat, i) != cig_byte(txt, i + tOff);
                const uint64_t b = ballot(mis);
                if (l == 0) S.mm[c] = b;
                straight += __builtin_popcountll(b);
                if (b && L0 == (int)len) L0 = c * 64 + __builtin_ctzll(b);
            }
            if (L0 == (int)len) {                // LandauVishkin.cpp:285-309
                ed = 0;
                S.ops[0] = (len << 4) | (A.useM ? 0u : 7u);
                nOps = len ? 1 : 0;
            } else {
                int Lp = d == 0 ? L0 : -2;
                S.L[0][l] = (int16_t)Lp;
                int eDone = 0, dDone = 0;
                for (int e = 1; e <= CIG_K; e++) {
                    const int left = shfl_idx(Lp, l == 0 ? 0 : l - 1);
                    const int right = shfl_idx(Lp, l == 63 ? 63 : l + 1) + 1;
                    const bool act = d >= -e && d <= e;
                    int best = Lp + 1, a = 0;
                    if (left > best) { best = left; a = 1; }
                    if (right > best) { best = right; a = 2; }
                    if (act && cig_byte(pat, best) == cig_byte(txt, d + best + tOff)) {
                        const int endd = d <= 0 ? (int)len : (int)len - d;
                        if (best >= endd) best = endd;
                        else {
                            int m = best;
                            for (;;) {
                                const uint32_t x = cig_ld4(pat, m) ^ cig_ld4(txt, m + d + tOff);
                                if (x) { m += __builtin_ctz(x) >> 3; break; }
                                m += 4;
                                if (m >= endd) break;
                            }
                            best = m < endd ? m : endd;
                        }
                    }
                    Lp = act ? best : -2;
                    S.L[e][l] = (int16_t)Lp;
                    S.A[e][l] = (uint8_t)a;
                    const uint64_t done = ballot(act && Lp == (int)len);
                    if (done) {
                        for (int k = 0; k <= 2 * e; k++) {     // order 0, -1, +1, -2, +2, ...
                            const int dd = k == 0 ? 0 : ((k & 1) ? -((k + 1) >> 1) : (k >> 1));
                            if ((done >> (dd + 31)) & 1) { dDone = dd; break; }
                        }
                        eDone = e;
                        break;
                    }
                }
                wave_sync();
                if (eDone) {
                    ed = eDone;
                    const uint32_t cEq = A.useM ? 0u : 7u;
                    auto put = [&](int cnt, uint32_t code) {
                        if (cnt > 0) {
                            if (l == 0) S.ops[nOps] = ((uint32_t)cnt << 4) | code;
                            nOps++;
                        }
                    };
                    if (straight == eDone) {     // LandauVishkin.cpp:341-393: no indels needed
                        if (A.useM) put((int)len, 0);
                        else {
                            bool matching = !(S.mm[0] & 1);
                            for (int i = 0; i < (int)len;) {
                                const int j = cig_next_bit(S, i, (int)len, matching);
                                put(j - i, matching ? 7u : 8u);
                                i = j;
                                matching = !matching;
                            }
                        }
                    } else {
                        // backtrace (LandauVishkin.cpp:420-440)
                        int curD = dDone;
                        for (int ce = eDone; ce >= 1; ce--) {
                            const int a = S.A[ce][curD + 31];
                            const int pd = a == 2 ? curD + 1 : a == 1 ? curD - 1 : curD;
                            const int m = S.L[ce][curD + 31] - S.L[ce - 1][pd + 31] - (a == 1 ? 0 : 1);
                            if (l == 0) { S.btA[ce] = a; S.btM[ce] = m; }
                            curD = pd;
                        }
                        wave_sync();
                        // emission (LandauVishkin.cpp:442-520)
                        int accM = 0;
                        const int l00 = S.L[0][31];
                        if (A.useM) accM = l00;
                        else put(l00, cEq);
                        for (int ce = 1; ce <= eDone; ce++) {
                            const int a = S.btA[ce];
                            int cnt = 1;
                            while (ce + 1 <= eDone && S.btM[ce] == 0 && S.btA[ce + 1] == a) { cnt++; ce++; }
                            const uint32_t code = a == 0 ? 8u : a == 1 ? 2u : 1u;
                            if (A.useM) {
                                if (a == 0) accM += cnt;
                                else { put(accM, 0); accM = 0; put(cnt, code); }
                            } else put(cnt, code);
                            const int m = S.btM[ce];
                            if (m > 0) {
                                if (A.useM) accM += m;
                                else put(m, 7);
                            }
                        }
                        if (A.useM) put(accM, 0);
                    }
                }
            }
            wave_sync();
        }
        if (l == 0) {
            A.outEd[r] = ed;
            A.outNOps[r] = nOps;
        }
        A.outOps[(uint64_t)r * CIG_MAX_OPS + l] = l < (int)nOps ? S.ops[l] : 0u;
        wave_sync();
    }
}

}  // namespace sgk
