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
// entries) by class, descending, into list[0, *count), stable (input order within a class).  One
// block of 256 threads, thread t taking a contiguous slice: per-thread class counts in registers,
// per class an exclusive scan over the threads in LDS, then each thread scatters its slice from its
// offsets -- no atomics (a first version with LDS atomics on 16 counters took 0.27 ms per 100k
// entries, contended; profiles/r05/rna/kernel_stats.csv).
static __global__ __launch_bounds__(256) void order_long_kernel(const uint32_t *tmp, const uint32_t *count, uint32_t *list) {
    constexpr int NT = 256, NC = 16;
    __shared__ uint32_t cnt[NC][NT];
    __shared__ uint32_t base[NC];
    const uint32_t n = *count, t = threadIdx.x;
    const uint32_t per = (n + NT - 1) / NT;
    const uint32_t b = t * per < n ? t * per : n, e = b + per < n ? b + per : n;
    uint32_t c[NC];
#pragma unroll
    for (int q = 0; q < NC; q++) c[q] = 0;
    for (uint32_t i = b; i < e; i++) {
        const uint32_t k = tmp[i] >> ORDER_CLASS_SHIFT;
#pragma unroll
        for (int q = 0; q < NC; q++) c[q] += k == (uint32_t)q ? 1u : 0u;
    }
#pragma unroll
    for (int q = 0; q < NC; q++) cnt[q][t] = c[q];
    __syncthreads();
    if (t < NC) {   // class t: exclusive scan over the threads, its total in base[t]
        uint32_t sum = 0;
        for (int j = 0; j < NT; j++) {
            const uint32_t v = cnt[t][j];
            cnt[t][j] = sum;
            sum += v;
        }
        base[t] = sum;
    }
    __syncthreads();
    if (t == 0) {   // heaviest class first
        uint32_t at = 0;
        for (int q = NC - 1; q >= 0; q--) {
            const uint32_t tot = base[q];
            base[q] = at;
            at += tot;
        }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < NC; q++) c[q] = base[q] + cnt[q][t];
    for (uint32_t i = b; i < e; i++) {
        const uint32_t v = tmp[i], k = v >> ORDER_CLASS_SHIFT;
        uint32_t pos = 0;
#pragma unroll
        for (int q = 0; q < NC; q++)
            if (k == (uint32_t)q) pos = c[q]++;
        list[pos] = v & ((1u << ORDER_CLASS_SHIFT) - 1u);
    }
}

}  // namespace sgk
