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

int main(int argc, char **argv) {
    const int cases = argc > 1 ? atoi(argv[1]) : 200000;
    static const char B4[] = "ACGT";
    long bad = 0, checked = 0, succ = 0;
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
        // the genome substring of a full window (BaseAligner.cpp:1161-1162); the shorter windows of the
        // contig-end fallback (:1163-1185) never take the per-lane filter (forced_filter routes them to
        // lv_group, whose text bound there depends on bytes past the window)
        const int glen = n + MAXK;
        const int t = s + seedLen;
        char qual[N + 16];
        memset(qual, 'I', sizeof qual);
        for (int k = 0; k <= KM; k++) {
            double p;
            int ni;
            const int want1 = oracle_lv(1, g + loc + t, glen - t, read + t, qual, n - t, k, &p, &ni);
            const int got1 = lv_lane_dist<KM>(F, true, t, n - t, glen - t, k);
            checked++;
            if (want1 != got1) {
                if (bad++ < 10) printf("fwd n=%d s=%d k=%d glen=%d: oracle %d lane %d\n", n, s, k, glen, want1, got1);
            }
            if (want1 < 0) continue;
            // reverse: pattern = read[s-1 .. 0], text = genome backwards from loc + s - 1, k2 = k - e1
            char rev[N + 16];
            for (int i = 0; i < s; i++) rev[i] = read[s - 1 - i];
            uint64_t R[2 * KM + 1][2];
            memcpy(R, F, sizeof R);
            lv_lane_reverse<KM>(R);
            const int k2 = k - want1;
            const int want2 = oracle_lv(-1, g + loc + s, s + MAXK, rev, qual, s, k2, &p, &ni);
            const int got2 = lv_lane_dist<KM>(R, true, 127 - (s - 1), s, s + MAXK, k2);
            checked++;
            if (want2 != got2) {
                if (bad++ < 10) printf("rev n=%d s=%d k2=%d: oracle %d lane %d\n", n, s, k2, want2, got2);
            }
            succ += want2 >= 0;
        }
    }
    printf("lv_lane: %ld calls, %ld full successes, %ld mismatches\n", checked, succ, bad);
    return bad != 0;
}
