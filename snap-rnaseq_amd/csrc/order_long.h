// order_long.h -- longest-first order of the persistent kernels' work lists (the tail of the
// heaviest read).  The RNA aligners (maxHits 16000) meet reads whose seeds hit a multi-isoform
// gene's shared exons: one wave scores thousands of candidates for one of them, and when such a read
// comes late in a persistent kernel's list that wave finishes alone after the rest of the grid has
// drained (~40 % of the transcriptome and intersecting kernels' time at 100k pairs, DESIGN.md
// section 8).  The list builders weigh each entry by the summed hit counts of its first seeds
// (seed_lookup_kernel for single reads, pair_weight_kernel for pairs) and this kernel sorts the list
// by the weight's log2 class, heaviest first.  Each read or pair is aligned by one wave on its own
// arena, so the order changes no result.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sgk {

constexpr uint32_t ORDER_CLASS_SHIFT = 28;   // list entry = index | class << 28 (index < 2^28)

// log2 class of a weight, 0 .. 15
__device__ __forceinline__ uint32_t order_class(uint32_t w) {
    const uint32_t c = w ? (uint32_t)(32 - __builtin_clz(w)) : 0u;
    return c < 15u ? c : 15u;
}

// Pass 0's long reads onto pass 2's list (and the paired aligner's long pairs onto pass 1b's),
// heaviest weight class first: a counting sort of the order list (index | class << 28, *count
// entries) by class, descending, into list[0, *count).  One block: the list is the batch's long
// reads or pairs (a few hundred thousand at most), two reads of it from L2.  Within a class the order is the atomics' (results do not depend on it).
static __global__ __launch_bounds__(1024) void order_long_kernel(const uint32_t *tmp, const uint32_t *count, uint32_t *list) {
    __shared__ uint32_t hist[16], cur[16];
    const uint32_t n = *count;
    if (threadIdx.x < 16) hist[threadIdx.x] = 0;
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) atomicAdd(&hist[tmp[i] >> ORDER_CLASS_SHIFT], 1u);
    __syncthreads();
    if (threadIdx.x < 16) {
        uint32_t s = 0;
        for (uint32_t c = threadIdx.x + 1; c < 16; c++) s += hist[c];
        cur[threadIdx.x] = s;
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
        const uint32_t v = tmp[i];
        list[atomicAdd(&cur[v >> ORDER_CLASS_SHIFT], 1u)] = v & ((1u << ORDER_CLASS_SHIFT) - 1u);
    }
}

}  // namespace sgk
