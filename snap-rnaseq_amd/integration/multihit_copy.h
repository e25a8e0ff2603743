// multihit_copy.h -- the copy-out step of GpuBaseAligner::AlignReadsMultiHit, kept free of SNAPLib
// types so tests/c/multihit_copy_test.cpp can exercise it without the reference.
#pragma once
#include <stddef.h>

#include "snapgpu.h"

// Hits of read i that AlignReadsMultiHit copies: none when maxHitsToGet == 0 (then neither the
// library, aligner.hip, nor the reference, BaseAligner.cpp:587-590 and 956, writes
// multiHitsFound[i], so whatever the caller left there is not a count), else the library's count
// clamped to [0, maxHitsToGet] -- the rows hold maxHitsToGet entries.
inline int gpuMultiHitsToCopy(int found, unsigned maxHitsToGet) {
    if (maxHitsToGet == 0 || found <= 0) return 0;
    return found > (int)maxHitsToGet ? (int)maxHitsToGet : found;
}

// Row i of the library's hits -> the caller's arrays (AlignReadsMultiHit's multiHitLocations /
// RCs / Scores, BaseAligner.h:72-86), each row maxHitsToGet wide.  Returns the count copied.
template <typename BoolT>
inline int gpuCopyMultiHits(const snapgpu_multi_hit_t *rows, size_t i, unsigned maxHitsToGet, int found,
                            unsigned *locations, BoolT *rcs, int *scores) {
    const int k = gpuMultiHitsToCopy(found, maxHitsToGet);
    for (int j = 0; j < k; j++) {
        const snapgpu_multi_hit_t &m = rows[i * maxHitsToGet + j];
        locations[i * maxHitsToGet + j] = m.location;
        rcs[i * maxHitsToGet + j] = m.direction != 0;
        scores[i * maxHitsToGet + j] = m.score;
    }
    return k;
}
