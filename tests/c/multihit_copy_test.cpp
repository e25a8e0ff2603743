// GpuBaseAligner::AlignReadsMultiHit's copy-out (snap-rnaseq_amd/integration/multihit_copy.h):
// maxHitsToGet == 0 copies nothing whatever the caller's multiHitsFound holds, and a count above the
// row width (or negative) is clamped, so no row is read or written past maxHitsToGet.
#include <stdio.h>
#include <string.h>

#include "multihit_copy.h"

static int fails = 0;
#define CHECK(c) do { if (!(c)) { printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c); fails++; } } while (0)

int main() {
    const unsigned W = 3;   // row width (maxHitsToGet)
    snapgpu_multi_hit_t rows[2 * W];
    for (unsigned i = 0; i < 2 * W; i++) { rows[i].location = 100 + i; rows[i].direction = i & 1; rows[i].score = i; rows[i].reserved = 0; }
    unsigned loc[2 * W + 4];
    bool rc[2 * W + 4];
    int sc[2 * W + 4];
    memset(loc, 0xab, sizeof loc); memset(sc, 0xab, sizeof sc); memset(rc, 0, sizeof rc);
    // maxHitsToGet == 0: nothing, even with garbage in the caller's count
    CHECK(gpuMultiHitsToCopy(12345, 0) == 0);
    CHECK(gpuCopyMultiHits(rows, 0, 0, 12345, loc, rc, sc) == 0 && loc[0] == 0xabababab);
    // counts: negative -> 0, above the width -> the width
    CHECK(gpuMultiHitsToCopy(-7, W) == 0);
    CHECK(gpuMultiHitsToCopy(2, W) == 2);
    CHECK(gpuMultiHitsToCopy(1000, W) == (int)W);
    // a limit below the hit count: row 1 gets exactly W hits, nothing past its end
    CHECK(gpuCopyMultiHits(rows, 1, W, 1000, loc, rc, sc) == (int)W);
    for (unsigned j = 0; j < W; j++) CHECK(loc[W + j] == 100 + W + j && sc[W + j] == (int)(W + j) && rc[W + j] == (((W + j) & 1) != 0));
    CHECK(loc[2 * W] == 0xabababab && sc[2 * W] == (int)0xabababab);
    CHECK(loc[0] == 0xabababab);   // row 0 untouched
    printf(fails ? "multihit_copy: %d failures\n" : "multihit_copy: ok\n", fails);
    return fails != 0;
}
