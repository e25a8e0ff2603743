// bucket_table.h -- the device image of the seed index, laid out for coalesced bucket probes.
//
// GenomeIndex::lookupSeed (GenomeIndex.cpp:971-1011) needs one thing from SNAPHashTable: the map
// key -> (value1, value2) that SNAPHashTable::Lookup (HashTable.h:74-105) defines.  The on-disk
// table answers it with 12-byte slots and a quadratic-then-linear probe sequence (+1, +4, +9, +16
// slots, then linear), so a lookup that misses its home slot touches two to four different 64-B
// lines, one dependent round trip each.  At aligner creation the device re-lays that map into
// 64-byte buckets -- one HBM line, four 16-byte entries:
//
//     entry = {key, value1, value2, aux}
//     aux   = [31] occupied | [30] (entry 0) overflow | [29:15] count(value2) | [14:0] count(value1)
//
// A key lives in its home bucket `home(key)` or, when that was full, in the first later bucket
// (wrapping) with room; every bucket passed over is flagged `overflow`.  A lookup loads the home
// line: the key is there, or the line proves it absent (no overflow flag) -- one line in the common
// case (C2: 2 keys per bucket on average, a few % of buckets overflow).  The counts are the lengths
// of the overflow lists the values point at (saturated at 0x7fff; a saturated count is re-read from
// the overflow table), so the list length needs no second dependent load either.
//
// Exactness: the builder (bucket_place_kernel / bucket_fill_kernel, aligner.hip) runs the
// reference's own probe sequence for every used slot and keeps exactly the slots that
// SNAPHashTable::Lookup of their key returns, so the bucket map answers every key as the reference
// table does (found or not, same values).  Which keys share a line is fixed too: placement is
// priority-ordered (a smaller key keeps its entry), which gives the layout of sequential insertion
// in key order on every build.  The per-read count of lines probed (snapgpu_result_t::nProbes) is
// therefore deterministic, but it is a device statistic, not a reference quantity.
#pragma once
#include "align_device.h"

namespace sgk {

constexpr uint32_t BK_OCC = 1u << 31;    // entry holds a key
constexpr uint32_t BK_OVF = 1u << 30;    // entry 0: a key homed at or before this bucket lives after it
constexpr uint32_t BK_CSAT = 0x7fffu;    // overflow-list count saturation (and field mask)
constexpr uint32_t BK_KEYS_PER_BUCKET = 2;   // sizing: buckets = ceil(keys / 2) per table (load 0.5)

// home bucket of `key` in a table of nB buckets: multiply-shift of a second 32-bit mixer (the
// slot hash fmix32 stays the reference's; this one only spreads keys over buckets)
__device__ __forceinline__ uint32_t bucket_home(uint32_t key, uint32_t nB) {
    uint32_t h = key * 0x9e3779b1u;
    h ^= h >> 15; h *= 0x2c1b3c6du; h ^= h >> 12; h *= 0x297a2d39u; h ^= h >> 15;
    return (uint32_t)(((uint64_t)h * nB) >> 32);
}
__device__ __forceinline__ uint32_t bucket_next(uint32_t b, uint32_t nB) { return b + 1 == nB ? 0u : b + 1; }

// overflow-list length of side value v (v >= nBases, v != UNUSED_SIDE) from its entry count
__device__ __forceinline__ uint32_t bucket_count(const KArgs &A, uint32_t cnt, uint32_t v) {
    return cnt < BK_CSAT ? cnt : A.overflow[v - A.nBases];
}

// One lane, one lookup: the whole 64-B line in four 16-B loads per bucket visited.
// -> found; v1/v2 as the slot holds them; aux of the entry (counts); lines = buckets loaded.
// (Named entries, not an array: an indexed uint4[4] went to scratch.)
__device__ __forceinline__ bool bucket_lookup_lane(const KArgs &A, uint32_t table, uint32_t key, uint32_t &v1,
                                                   uint32_t &v2, uint32_t &aux, uint32_t &lines) {
    const uint32_t nB = A.bucketCount[table];
    const uint4 *T = A.buckets + 4ull * A.bucketBase[table];
    uint32_t b = bucket_home(key, nB);
    for (lines = 1;; lines++) {
        const uint4 *p = T + 4ull * b;
        const uint4 e0 = p[0], e1 = p[1], e2 = p[2], e3 = p[3];
        const bool h0 = (e0.w & BK_OCC) && e0.x == key, h1 = (e1.w & BK_OCC) && e1.x == key;
        const bool h2 = (e2.w & BK_OCC) && e2.x == key, h3 = (e3.w & BK_OCC) && e3.x == key;
        if (h0 | h1 | h2 | h3) {
            const uint4 e = h0 ? e0 : (h1 ? e1 : (h2 ? e2 : e3));
            v1 = e.y; v2 = e.z; aux = e.w;
            return true;
        }
        if (!(e0.w & BK_OVF) || lines >= nB) return false;
        b = bucket_next(b, nB);
    }
}

// One lookup per lane, four lanes per line: in round t (0..3) lane 4i + p loads entry p of the home
// bucket of lane 16t + i's key, so each 16-B load instruction covers 16 whole 64-B lines where
// bucket_lookup_lane has every lane touch a different line (4x the line requests for the same
// bytes).  The entries found go back to their lanes by ds_bpermute.  A key absent from its home
// bucket whose home bucket is flagged overflow continues lane by lane from the next bucket, so
// the answer and `lines` equal bucket_lookup_lane's.  Every lane of the wave must call it.
__device__ __forceinline__ bool bucket_lookup_quad(const KArgs &A, bool act, uint32_t table, uint32_t key,
                                                   uint32_t &v1, uint32_t &v2, uint32_t &aux, uint32_t &lines) {
    const int lane = lane_id();
    uint32_t nB = 1;
    uint64_t tb = 0;
    if (act) { nB = A.bucketCount[table]; tb = A.bucketBase[table]; }
    const uint32_t hb = act ? bucket_home(key, nB) : 0u;
    const uint64_t line = tb + hb;   // bucket index in the whole image
    bool found = false, ovf = false;
    v1 = v2 = aux = 0;
#pragma unroll
    for (int t = 0; t < 4; t++) {
        const int src = 16 * t + (lane >> 2);
        const uint32_t lo = (uint32_t)shfl_idx((int)(uint32_t)line, src);
        const uint32_t hi = (uint32_t)shfl_idx((int)(uint32_t)(line >> 32), src);
        const uint32_t k = (uint32_t)shfl_idx((int)key, src);
        const bool a = shfl_idx(act ? 1 : 0, src) != 0;
        uint4 e = make_uint4(0u, 0u, 0u, 0u);
        if (a) e = A.buckets[4ull * (((uint64_t)hi << 32) | lo) + (uint32_t)(lane & 3)];
        const uint64_t hm = ballot(a && (e.w & BK_OCC) && e.x == k);
        const uint64_t om = ballot(a && (lane & 3) == 0 && (e.w & BK_OVF));
        const bool mine = (lane >> 4) == t;          // lanes 16t .. 16t+15 own this round's keys
        const int i = lane & 15;
        const uint32_t nib = (uint32_t)(hm >> (4 * i)) & 0xfu;
        const int from = 4 * i + (nib ? (int)__builtin_ctz(nib) : 0);
        const uint32_t y = (uint32_t)shfl_idx((int)e.y, from), z = (uint32_t)shfl_idx((int)e.z, from);
        const uint32_t w = (uint32_t)shfl_idx((int)e.w, from);
        if (mine) {
            found = nib != 0;
            ovf = ((om >> (4 * i)) & 1ull) != 0;
            if (found) { v1 = y; v2 = z; aux = w; }
        }
    }
    lines = 1;
    if (act && !found && ovf && nB > 1) {   // past the home bucket, as bucket_lookup_lane continues
        const uint4 *T = A.buckets + 4ull * tb;
        uint32_t b = bucket_next(hb, nB);
        for (lines = 2;; lines++) {   // (entry by entry: this rare path must not raise the kernel's VGPRs)
            const uint4 *p = T + 4ull * b;
            bool ovfB = false;
            for (int q = 0; q < 4 && !found; q++) {
                const uint4 e = p[q];
                if (q == 0) ovfB = (e.w & BK_OVF) != 0;
                if ((e.w & BK_OCC) && e.x == key) { v1 = e.y; v2 = e.z; aux = e.w; found = true; }
            }
            if (found || !ovfB || lines >= nB) break;
            b = bucket_next(b, nB);
        }
    }
    return found;
}

// The whole wave, one lookup (uniform key): lanes 0-3 load the four entries of bucket b, lanes 4-7
// those of bucket b+1 (the adjacent line: a key that spilled over is found without a further round
// trip).  Results are wave-uniform; lines = buckets a sequential lookup would have loaded.
__device__ __forceinline__ bool bucket_lookup_wave(const KArgs &A, uint32_t table, uint32_t key, int lane, uint32_t &v1,
                                                   uint32_t &v2, uint32_t &aux, uint32_t &lines) {
    const uint32_t nB = A.bucketCount[table];
    const uint4 *T = A.buckets + 4ull * A.bucketBase[table];
    uint32_t b = bucket_home(key, nB);
    for (uint32_t step = 0;; step += 2) {
        const uint32_t bl = (lane & 4) ? bucket_next(b, nB) : b;
        uint4 e = make_uint4(0u, 0u, 0u, 0u);
        if (lane < 8) e = T[4ull * bl + (lane & 3)];
        const uint64_t hit = ballot(lane < 8 && (e.w & BK_OCC) && e.x == key);
        const uint64_t ovf = ballot(lane < 8 && (lane & 3) == 0 && (e.w & BK_OVF));
        const uint64_t h0 = hit & 0xfull, h1 = hit & 0xf0ull;
        int src = -1;
        if (h0) { src = __builtin_ctzll(h0); lines = step + 1; }
        else if (!(ovf & 1ull) || step + 1 >= nB) { lines = step + 1; return false; }
        else if (h1) { src = __builtin_ctzll(h1); lines = step + 2; }
        else if (!(ovf & 0x10ull) || step + 2 >= nB) { lines = step + 2; return false; }
        if (src >= 0) {
            v1 = readlaneu(e.y, src); v2 = readlaneu(e.z, src); aux = readlaneu(e.w, src);
            return true;
        }
        b = bucket_next(bucket_next(b, nB), nB);
    }
}

}  // namespace sgk
