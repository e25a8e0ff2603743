// Host check of the per-lane LV distance (snap-rnaseq_amd/csrc/lv_lane.h) against the oracle's
// LandauVishkin restatement (oracle/snap_oracle.c oracle_lv, pinned to the reference by
// tests/test_oracle_golden.py): random reads against mutated genome windows -- substitutions,
// insertions, deletions, N and non-ACGT bytes, seeds at both read ends -- forward and reverse, every k up
// to KM, exactly as BaseAligner::score calls them (BaseAligner.cpp:1199-1220).  Built with hipcc
// (the header's functions are __host__ __device__), run on the CPU.
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "lv_lane.h"

extern "C" int oracle_lv(int dir, const char *text, int textLen, const char *pattern, const char *qual, int patternLen,
                         int k, double *matchProbability, int *netIndel);

using namespace sgk;
constexpr int KM = 5, MAXK = 31, N = 128;

static uint64_t rng = 88172645463325252ull;
static uint32_t rnd() { rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17; return (uint32_t)rng; }
static bool acgt(char c) { return c == 'A' || c == 'C' || c == 'G' || c == 'T'; }


// Host lockstep emulation of lv_pair_dist (lv_lane.h, device-only: it swaps values across a lane
// pair by DPP): the same per-half arithmetic, both halves advanced row by row, the swaps done by
// hand.  Local i of half h is forward diagonal x = h ? i : -i.
template <int KM, int DIR>
static int pair_emul(const uint64_t (&F)[2 * KM + 1][2], int q0, int patternLen, int textLen, int k) {
    uint64_t M[2][KM + 1][2];
    for (int h = 0; h < 2; h++)
        for (int i = 0; i <= KM; i++) {
            const int x = h ? i : -i;
            M[h][i][0] = F[x + KM][0];
            M[h][i][1] = F[x + KM][1];
        }
    if (k > KM) k = KM;
    auto first = [&](int h, int i, int p) -> int {
        if (DIR > 0) return ll_first_from(M[h][i][0], M[h][i][1], p);
        return 127 - ll_last_upto(M[h][i][0], M[h][i][1], 127 - p);
    };
    const int end0 = patternLen < textLen ? patternLen : textLen;
    const int fm = first(0, 0, q0) - q0;
    const int v0 = fm < end0 ? fm : end0;
    if (v0 == end0) {
        const int result = patternLen > end0 ? patternLen - end0 : 0;
        return result > k ? -1 : result;
    }
    int B[2][KM + 3] = {};
    B[0][1] = B[1][1] = v0 + 2;
    const int patB = patternLen + 2, q0m2 = q0 - 2;
    for (int e = 1; e <= KM; e++) {
        if (e > k) break;
        const int s0 = B[1][2], s1 = B[0][2];
        B[0][0] = s0;
        B[1][0] = s1;
        bool hit[2] = {false, false};
        for (int h = 0; h < 2; h++) {
            const bool up = DIR > 0 ? h != 0 : h == 0;
            int prev = B[h][0];
            for (int i = 0; i <= e && i <= KM; i++) {
                const int d = up ? i : -i;
                const int old = B[h][i + 1], lo = prev, hi = B[h][i + 2];
                prev = old;
                const int leftB = up ? lo : hi, rightB = (up ? hi : lo) + 1, x1B = old + 1;
                const int bxdB = leftB > x1B ? leftB : x1B;
                const int bestB = rightB > bxdB ? rightB : bxdB;
                const int endd = patternLen < textLen - d ? patternLen : textLen - d;
                const int enddB = endd + 2;
                const int mpos = q0m2 + bestB;
                const int mposc = mpos < 128 ? mpos : 128;
                const int fa = first(h, i, mposc);
                const int fB = fa - q0m2;
                const int slidB = fB < enddB ? fB : enddB;
                const int bnewB = bestB < enddB ? slidB : (fa == mposc ? bestB : enddB);
                B[h][i + 1] = bnewB;
                hit[h] = hit[h] || bnewB == patB;
            }
        }
        if (hit[0] || hit[1]) return e;
    }
    return -1;
}

// Host lockstep emulation of lv_quad_dist (lv_lane.h, device-only: DPP quad permutes): four lane states,
// the neighbour slots moved by hand, every lane's row through the shared quad_row.  F16[s] is forward
// diagonal x = s - LQ_K (s = 0..15); lane q holds slots 4q .. 4q + 3.
template <int DIR>
static int quad_emul(const uint64_t (&F16)[16][2], int q0, int patternLen, int textLen, int k) {
    uint64_t M[4][4][2];
    for (int q = 0; q < 4; q++)
        for (int j = 0; j < 4; j++) { M[q][j][0] = F16[4 * q + j][0]; M[q][j][1] = F16[4 * q + j][1]; }
    if (k > LQ_K) k = LQ_K;
    const int end0 = patternLen < textLen ? patternLen : textLen;
    const int fm = quad_first<DIR>(M[1], 3, q0) - q0;
    const int v0 = fm < end0 ? fm : end0;
    if (v0 == end0) {
        const int result = patternLen > end0 ? patternLen - end0 : 0;
        return result > k ? -1 : result;
    }
    int Bl[4][6] = {};
    Bl[1][4] = v0 + 2;
    const int patB = patternLen + 2, q0m2 = q0 - 2;
    for (int e = 1; e <= LQ_K; e++) {
        if (e > k) break;
        int lo[4], hi[4];
        for (int q = 0; q < 4; q++) { lo[q] = q == 0 ? 0 : Bl[q - 1][4]; hi[q] = q == 3 ? 0 : Bl[q + 1][1]; }
        bool h = false;
        for (int q = 0; q < 4; q++) {
            Bl[q][0] = lo[q];
            Bl[q][5] = hi[q];
            h = quad_row<DIR>(M[q], q, e, Bl[q], q0m2, patB, patternLen, textLen) || h;
        }
        if (h) return e;
    }
    return -1;
}

// ll_first_from / ll_last_upto (select forms) against a plain bit scan, every start, sparse and
// dense masks (empty words, single bits at the word edges)
static long scanCheck() {
    long bad = 0;
    for (int c = 0; c < 4000; c++) {
        uint64_t w[2];
        for (int j = 0; j < 2; j++) {
            const uint32_t kind = rnd() % 5;
            w[j] = kind == 0 ? 0ull : kind == 1 ? 1ull << (rnd() % 64) : kind == 2 ? 1ull << (63 - (rnd() % 2) * 63)
                 : ((uint64_t)rnd() << 32 | rnd()) & ((uint64_t)rnd() << 32 | rnd());
        }
        auto bit = [&](int p) { return (w[p >> 6] >> (p & 63)) & 1; };
        for (int m = 0; m <= 128; m++) {
            int f = 128;
            for (int p = m; p < 128; p++) if (bit(p)) { f = p; break; }
            if (ll_first_from(w[0], w[1], m) != f) bad++;
        }
        for (int m = -1; m <= 127; m++) {
            int l = -1;
            for (int p = m; p >= 0; p--) if (bit(p)) { l = p; break; }
            if (ll_last_upto(w[0], w[1], m) != l) bad++;
        }
    }
    return bad;
}

int main(int argc, char **argv) {
    const int cases = argc > 1 ? atoi(argv[1]) : 200000;
    if (const long sb = scanCheck()) { printf("mask scans: %ld wrong\n", sb); return 1; }
    static const char B4[] = "ACGT";
    long bad = 0, checked = 0, succ = 0, qsucc = 0;
    for (int c = 0; c < cases; c++) {
        // genome window g[0 .. n + MAXK + KM) around loc = KM (so x = -KM .. KM stay inside)
        const int n = 40 + (int)(rnd() % 89);       // read length 40..128
        const int seedLen = 20;
        const int s = (int)(rnd() % (n - seedLen + 1));   // seed offset
        char g[N + 2 * MAXK + 64];
        for (int i = 0; i < (int)sizeof g; i++) g[i] = B4[rnd() & 3];
        if (rnd() % 16 == 0) for (int i = 0; i < 4; i++) g[rnd() % sizeof g] = 'n';   // N runs / padding
        const int loc = 2 * MAXK;
        // read = genome at loc with edits (the seed region kept intact)
        char read[N + 16] = {0};
        int gi = loc, ri = 0;
        const int rate = 1 + (int)(rnd() % 12);
        while (ri < n) {
            const bool inSeed = ri >= s && ri < s + seedLen;
            const uint32_t r = rnd() % 100;
            if (!inSeed && r < (uint32_t)rate) read[ri++] = B4[rnd() & 3];                  // substitution
            else if (!inSeed && r < (uint32_t)rate + 2 && ri > 0) { read[ri++] = B4[rnd() & 3]; }   // insertion
            else if (!inSeed && r < (uint32_t)rate + 4) gi++;                                   // deletion
            else { const char b = g[gi++]; read[ri++] = b == 'n' ? 'N' : b; }   // reads are upper case (Read::init)
            if (gi >= (int)sizeof g - 1) gi = (int)sizeof g - 2;
        }
        if (rnd() % 20 == 0) read[rnd() % n] = 'N';
        if (rnd() % 40 == 0) read[rnd() % n] = 'R';   // IUPAC: not ACGT, never matches on the bit planes
        // reads with IUPAC bytes go to the byte path only when the genome has IUPAC codes too; here
        // the genome has none, so bit-plane (mask) semantics = byte semantics
        // masks F_x[m] = read[m] != g[loc + x + m] (non-ACGT on either side never matches), m < 128
        uint64_t F[2 * KM + 1][2];
        for (int x = -KM; x <= KM; x++) {
            uint64_t w[2] = {0, 0};
            for (int m = 0; m < N; m++) {
                const char rc = m < n ? read[m] : 0;
                const int gp = loc + x + m;
                const char gc = gp >= 0 && gp < (int)sizeof g ? g[gp] : 'n';
                const bool mm = !acgt(rc) || !acgt(gc) || rc != gc;
                if (mm) w[m >> 6] |= 1ull << (m & 63);
            }
            F[x + KM][0] = w[0];
            F[x + KM][1] = w[1];
        }
        // the quad form's slots: forward diagonals x = -LQ_K .. LQ_K + 1
        uint64_t F16[16][2];
        for (int sl = 0; sl < 16; sl++) {
            const int x = sl - LQ_K;
            uint64_t w[2] = {0, 0};
            for (int m = 0; m < N; m++) {
                const char rc = m < n ? read[m] : 0;
                const int gp = loc + x + m;
                const char gc = gp >= 0 && gp < (int)sizeof g ? g[gp] : 'n';
                if (!acgt(rc) || !acgt(gc) || rc != gc) w[m >> 6] |= 1ull << (m & 63);
            }
            F16[sl][0] = w[0];
            F16[sl][1] = w[1];
        }
        // the genome substring of a full window (BaseAligner.cpp:1161-1162); the shorter windows of the
        // contig-end fallback (:1163-1185) never take the per-lane filter (forced_filter routes them to
        // lv_group, whose text bound there depends on bytes past the window)
        const int glen = n + MAXK;
        const int t = s + seedLen;
        char qual[N + 16];
        memset(qual, 'I', sizeof qual);
        for (int k = 0; k <= LQ_K; k++) {
            double p;
            int ni;
            const int want1 = oracle_lv(1, g + loc + t, glen - t, read + t, qual, n - t, k, &p, &ni);
            const int quad1 = quad_emul<1>(F16, t, n - t, glen - t, k);
            checked++;
            if (want1 != quad1) {
                if (bad++ < 10) printf("quad fwd n=%d s=%d k=%d: oracle %d quad %d\n", n, s, k, want1, quad1);
            }
            if (want1 < 0) continue;
            char rev[N + 16];
            for (int i = 0; i < s; i++) rev[i] = read[s - 1 - i];
            const int k2 = k - want1;
            const int want2 = oracle_lv(-1, g + loc + s, s + MAXK, rev, qual, s, k2, &p, &ni);
            const int quad2 = quad_emul<-1>(F16, 127 - (s - 1), s, s + MAXK, k2);
            checked++;
            if (want2 != quad2) {
                if (bad++ < 10) printf("quad rev n=%d s=%d k2=%d: oracle %d quad %d\n", n, s, k2, want2, quad2);
            }
            qsucc += want2 >= 0;
        }
        for (int k = 0; k <= KM; k++) {
            double p;
            int ni;
            const int want1 = oracle_lv(1, g + loc + t, glen - t, read + t, qual, n - t, k, &p, &ni);
            const int got1 = lv_lane_dist<KM>(F, true, t, n - t, glen - t, k);
            const int pair1 = pair_emul<KM, 1>(F, t, n - t, glen - t, k);
            checked++;
            if (want1 != got1 || want1 != pair1) {
                if (bad++ < 10) printf("fwd n=%d s=%d k=%d glen=%d: oracle %d lane %d pair %d\n", n, s, k, glen, want1, got1, pair1);
            }
            if (want1 < 0) continue;
            // reverse: pattern = read[s-1 .. 0], text = genome backwards from loc + s - 1, k2 = k - e1
            char rev[N + 16];
            for (int i = 0; i < s; i++) rev[i] = read[s - 1 - i];
            const int k2 = k - want1;
            const int want2 = oracle_lv(-1, g + loc + s, s + MAXK, rev, qual, s, k2, &p, &ni);
            const int got2 = lv_lane_dist<KM, -1>(F, true, 127 - (s - 1), s, s + MAXK, k2);
            const int pair2 = pair_emul<KM, -1>(F, 127 - (s - 1), s, s + MAXK, k2);
            checked++;
            if (want2 != got2 || want2 != pair2) {
                if (bad++ < 10) printf("rev n=%d s=%d k2=%d: oracle %d lane %d\n", n, s, k2, want2, got2);
            }
            succ += want2 >= 0;
        }
    }
    printf("lv_lane: %ld calls, %ld full successes (pair form, k <= %d), %ld (quad form, k <= %d), %ld mismatches\n", checked,
           succ, KM, qsucc, LQ_K, bad);
    return bad != 0;
}
