// align_device.h -- gfx950 device code for the batched BaseAligner::AlignRead.
//
// One wavefront (64 lanes) aligns one read at a time; waves pull reads from a
// device work counter (persistent grid).  Per wave:
//   * LDS: the read in both orientations + qualities, the genome window of the
//     candidate being scored, the Landau-Vishkin row history, the candidate
//     element hash buckets, insertion-batch scratch, per-lane selection maxima.
//   * HBM: a private element arena (worst-case sized: (maxSeeds+1)*maxHits
//     elements), 64-B Elem64 (reads <= 256 b; the first ELCAP in LDS) or 144-B Elem512 elements,
//     one read = one arena lifetime.
//
// Reference semantics restated (all citations SNAPLib/...):
//   AlignRead   BaseAligner.cpp:510-938   score  BaseAligner.cpp:977-1399
//   LV          LandauVishkin.h:211-455   lookup GenomeIndex.cpp:971-1086, HashTable.h:74-105
//   MAPQ        mapq.h:32-65
//
// Lane roles:
//   * hash-probe: lanes 0-7 load the 16-B entries of a key's home bucket and the next one
//     (bucket_table.h).
//   * hit insertion: lane i handles hit i of a 64-hit batch; duplicates inside
//     the batch are grouped through an LDS table and applied in hit order by
//     the group's first lane (so FIFO/weight semantics are exactly sequential).
//   * LV: lane 31+d (forward) / 31-d (reverse) holds diagonal d; the per-lane
//     mismatch bitmap F_x[m] = read[m] != genome[g+x+m] is built with one
//     compare+ballot per (x, 64-position block) and v_writelane.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "snapgpu.h"

namespace sgk {

constexpr int WAVE = 64;
constexpr int MAX_K = 31;                 // LandauVishkin.h:9
constexpr uint32_t INVALID = 0xffffffffu; // InvalidGenomeLocation
constexpr uint32_t UNUSED_SIDE = 0xfffffffeu;
constexpr uint32_t UNUSED_SCORE = 0xffffu;
constexpr uint32_t FAIL_SCORE = 0xffffffffu;
constexpr int ELEM = 48;                  // hashTableElementSize == maxMergeDist
constexpr uint32_t NPAD = 100;            // Genome::N_PADDING
constexpr int NBUCKET_LOG2 = 9;         // (512 u16 heads: C3 -2.2 %, C2 -0.9 % against 256; 128 was C3 +3.8 %,
                                         // profiles/r06/ab/hash_buckets_r06h9.txt)
constexpr int NBUCKET = 1 << NBUCKET_LOG2;  // element hash buckets (LDS)
constexpr uint32_t SKCAP = 192;           // selection keys kept in LDS (192 + 192 mirrors pay for the 512 heads)
constexpr uint32_t MIRCAP = 192;          // elements whose key / chain link are mirrored in LDS
constexpr int ELEM_DWORDS = 36;           // dwords of Elem512 (byte path)
constexpr int BT = 128;                   // insertion-batch dedupe table (LDS)
constexpr uint32_t NONE = 0xffffffffu;
constexpr uint32_t ELCAP = 6;             // Elem64 kernels: elements 0..ELCAP-1 of a read are kept in LDS
                                         // (32 fit 4 waves/SIMD; 6 keep <128> within the 8 KB of 5 waves/SIMD)

struct DevTables {
    double indel[64];
    double phred[256];
    double perfect[512];
    double seedProb;          // __powidf2(0.999, seedLen), BaseAligner.cpp:1227
    uint32_t wrap[32];        // GetWrappedNextSeedToTest order (SeedSequencer.h)
    double mapqT[72];         // mapqT[q] = 10^(-q/10) (glibc pow): MAPQ thresholds, no device log10
    uint32_t maxSeedsForLen[513];   // (int)(seedCoverage * n / seedLen) per read length n (BaseAligner.cpp:563-568)
    // The first 16 seed offsets of the seed sequence (BaseAligner.cpp:686-746) of a read of length n
    // whose bases are all ACGT: the sequence then depends on n and seedLen only (0xff: not reached)
    uint8_t seedSeq[129][16];
};
// The seedLen-independent tables (indel, phred, perfect, mapqT), one copy per device, set
// once by the host: a global's address is a constant the compiler rematerializes, where a
// table pointer argument is one more SGPR pair to keep live (and spill) in the scorer.
static __device__ DevTables g_tab;   // per translation unit (aligner.hip, paired.hip): each sets its own

// HashTableElement (BaseAligner.h:188-214) in the HBM arena: a 48-byte header of the fields the
// kernels read and write, then the per-candidate seed offsets.
//
// The byte path (reads > 256 bases) keeps every candidate's u16 offset in the element (Elem512,
// 144 B).  The bit-plane kernels (reads <= 256 bases, u8 offsets) keep an element in one 64-B
// line (Elem64): most elements use one or two of their 48 candidates, so the header is followed
// by eight (bit + 1, offset) byte pairs in first-use order; an element that uses a ninth
// candidate gets a spill block -- a 64-B slot taken from the top of the wave's arena, offsets by
// bit -- into which the eight are copied, and its offsets live there from then on (w11.spill).
// A read's elements then stay one line each (round 3: 96 B, two or three lines per pair).
template <typename OffT>
struct ElemT {
    uint64_t used;            // candidatesUsed
    uint64_t scored;          // candidatesScored
    double prob;              // matchProbabilityForBestScore
    uint32_t key;             // (base/48)<<1 | direction
    uint32_t next;            // hash chain
    uint32_t bestScore;
    uint32_t bestLoc;         // bestScoreGenomeLocation
    uint32_t sortkey;         // linked ? weight<<24 | (0xffffff - ts) : 0
    uint8_t weight, lps, allScored, pad;
    OffT seedOffset[ELEM];
    static constexpr int DWORDS = (48 + ELEM * (int)sizeof(OffT)) / 4;
};
using Elem512 = ElemT<uint16_t>;
struct Elem64 {
    uint64_t used;            // dw 0-1   candidatesUsed
    uint64_t scored;          // dw 2-3   candidatesScored
    double prob;              // dw 4-5   matchProbabilityForBestScore
    uint32_t key;             // dw 6     (base/48)<<1 | direction
    uint32_t next;            // dw 7     hash chain
    uint32_t bestScore;       // dw 8
    uint32_t bestLoc;         // dw 9     bestScoreGenomeLocation
    uint32_t sortkey;         // dw 10    linked ? weight<<24 | (0xffffff - ts) : 0
    uint32_t w11;             // dw 11    weight | lps << 8 | allScored << 16 | spill << 17
    uint32_t slot[4];         // dw 12-15 (bit + 1, seed offset) byte pairs, first-use order; 0 = free
    static constexpr int DWORDS = 16;
};
static_assert(sizeof(Elem512) == 144 && sizeof(Elem64) == 64, "Elem layout");
constexpr uint32_t W11_ALLSCORED = 1u << 16;
constexpr int W11_SPILL_SHIFT = 17;                  // spill block index (0 = none), 15 bits
constexpr uint32_t ELEM64_MAX = 0x7fffu;             // bit-plane arenas: at most this many 64-B slots
constexpr int NSLOT = 8;                             // inline offsets per Elem64
// an Elem64's spill block (an arena slot index; 0 = none): its bytes 0..47 are the seed offsets by bit
__device__ __forceinline__ uint32_t spill_index(uint32_t w11) { return w11 >> W11_SPILL_SHIFT; }
// seed offset of candidate `bit` from an Elem64's four slot dwords (0xffffffff when not held there)
__device__ __forceinline__ uint32_t slot_offset(uint32_t s0, uint32_t s1, uint32_t s2, uint32_t s3, uint32_t bit) {
    const uint32_t tag = bit + 1u;
    uint32_t r = 0xffffffffu;
    const uint32_t s[4] = {s0, s1, s2, s3};
#pragma unroll
    for (int i = 0; i < 4; i++) {
        if ((s[i] & 0xffu) == tag) r = (s[i] >> 8) & 0xffu;
        if (((s[i] >> 16) & 0xffu) == tag) r = s[i] >> 24;
    }
    return r;
}
// the inline slot (0..7) holding candidate `bit` (NSLOT when none)
__device__ __forceinline__ uint32_t slot_of(const uint32_t (&s)[4], uint32_t bit) {
    uint32_t r = NSLOT;
#pragma unroll
    for (int q = NSLOT - 1; q >= 0; q--)
        if (((s[q >> 1] >> (16 * (q & 1))) & 0xffu) == bit + 1u) r = (uint32_t)q;
    return r;
}
// slot k := (bit + 1, offset), registers only (selects, no dynamic indexing)
__device__ __forceinline__ void slot_set(uint32_t (&s)[4], uint32_t k, uint32_t bit, uint32_t offset) {
    const uint32_t sh = 16u * (k & 1u), v = ((offset & 0xffu) << 8 | (bit + 1u)) << sh, keep = ~(0xffffu << sh);
#pragma unroll
    for (int d = 0; d < 4; d++) s[d] = (k >> 1) == (uint32_t)d ? (s[d] & keep) | v : s[d];
}
template <int MAXLEN> struct ElemSel { using type = Elem512; };
template <> struct ElemSel<128> { using type = Elem64; };
template <> struct ElemSel<256> { using type = Elem64; };
template <int MAXLEN> using ElemOf = typename ElemSel<MAXLEN>::type;

// Genome bit planes: 32 bases per 12-byte word, 3 bits per base -- the 2-bit code (A=00 C=01 G=10
// T=11) as two planes plus the not-ACGT plane a byte-exact comparison needs (N and IUPAC bytes
// match nothing).  A window of 2*NW+1 words is one 12-B-strided run (60 B for a 128-base read),
// one or two 128-B lines.
struct alignas(4) GPlane { uint32_t hi, lo, nm; };
static_assert(sizeof(GPlane) == 12, "GPlane layout");

struct KArgs {
    uint32_t *diag;              // this aligner's watchdog record {code, read, detail, 0} (diag_report)
    // index (HBM): the seed tables as 64-B buckets (bucket_table.h), per table base (in buckets)
    // and bucket count; the overflow lists as the reference stores them
    const uint4 *buckets;
    const uint64_t *bucketBase;
    const uint32_t *bucketCount;
    const uint32_t *overflow;
    const char *genome;          // base 0; >= 256 guard bytes each side
    const uint32_t *pieces;
    int32_t nPieces;
    uint32_t nBases, seedLen, nTables, padding;
    // params
    uint32_t maxHits, maxK, maxReadSize, maxSeedsCmd;
    double seedCoverage;
    uint32_t extra, explore, stopOnFirst, kRows;
    uint32_t tripRead;           // test hook: report DIAG_TEST_TRIP when this read starts (0xffffffff: never)
    uint32_t radixMin;           // forced mode: radix-sort the pop order of reads with >= this many elements
    const DevTables *tab;
    // reads
    const char *bases;
    const char *quals;
    const uint64_t *offsets;
    const uint32_t *lengths;
    uint32_t nReads;
    snapgpu_result_t *out;
    // work queue + arenas
    uint32_t *counter;
    void *arena;                 // ElemOf<MAXLEN> per block
    uint64_t arenaElems;         // per-wave capacity
    // Main passes run on arenas capped below the worst case (maxSeeds + 2) * maxHits when that would
    // not fit the whole grid (the RNA aligners' maxHits 16000): a read that outgrows its arena is
    // abandoned (no record written) and listed here for the big-arena pass (align_kernel<512> on a
    // small grid with worst-case arenas).  nullptr: the arena is worst-case sized (arena full =
    // watchdog record, cannot happen).
    uint32_t *ovfList;
    uint32_t *ovfCount;
    // genome bit planes {hi, lo, notACGT} per 32 bases (GPlane), word 0 = position -PACK_GUARD
    const struct GPlane *gpl;
    uint32_t hasIupac;
    // three-pass dispatch: align_kernel<128> defers reads it cannot take (longer than 128
    // bases, or IUPAC codes on both sides) to align_kernel<256>, which defers reads longer than
    // 256 bases and the IUPAC ones to align_kernel<512>
    uint32_t *deferList;         // passes 1 and 2 append the read indices they defer here
    uint32_t *deferCount;        //   (atomic append count)
    const uint32_t *readList;    // passes 2 and 3: read indices (the previous passes' defers; nullptr in pass 1)
    const uint32_t *readCount;   //   and their number (the previous pass's deferCount)
    const uint4 *seedRecs;       // seed_lookup_kernel records (SeedRec, 16 per read; passes 1 and 2), or nullptr
    // pass 0 puts the reads longer than 128 bases straight onto deferList (pass 2's list) with one
    // atomic per 4-read wave that holds any, and counts them in longCount; pass 1 (longCount set)
    // then skips them instead of deferring them one by one, and ends at once when every read is long
    uint32_t *longCount;
    // longest-first order of pass 2 (SNAPGPU_ORDER_LONG, default on): pass 0 writes its long reads
    // here as read | class << 28 (class = log2 of the summed hit counts of their first seeds) and
    // order_long_kernel moves them onto deferList heaviest class first; nullptr: straight onto deferList
    uint32_t *orderTmp;
    unsigned long long *phaseBuf;   // diagnostic (SNAPGPU_PHASES=1): per-block [PH_SLOTS] cycle sums, else null
    // windowed search + multi-hit export (snapgpu_align_batch_ex; BaseAligner.h:73-86)
    const snapgpu_search_t *search;     // per read, or nullptr (= unconstrained)
    uint32_t maxHitsToGet;              // 0: no multi-hit recording
    uint32_t hitStride;                 // u32 per block in hitScratch
    uint32_t hitSlot;                   // distance stride of the hit table: min(maxHitsToGet, 512)
    uint32_t *hitScratch;               // per block: hitCount[MAX_K], then {loc, dir}[MAX_K * hitSlot (+ maxHitsToGet)]
    int32_t *multiFound;                // per read
    snapgpu_multi_hit_t *multiHits;     // [nReads][maxHitsToGet]
};

// ------------------------------------------------------------ wave helpers
// Lane id through volatile asm: the compiler cannot hoist it (or the per-lane LDS
// addresses derived from it) out of the persistent loop, which would otherwise keep
// ~100 lane-invariant VGPRs live for the whole kernel and halve occupancy.
__device__ __forceinline__ int lane_id() {
    int v;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(v));
    return v;
}
__device__ __forceinline__ uint32_t uni(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
__device__ __forceinline__ int unii(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t uni64(uint64_t v) {
    return ((uint64_t)uni((uint32_t)(v >> 32)) << 32) | uni((uint32_t)v);
}
__device__ __forceinline__ double unid(double v) { return __longlong_as_double((long long)uni64((uint64_t)__double_as_longlong(v))); }
__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }
__device__ __forceinline__ int readlane(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ uint32_t readlaneu(uint32_t v, int l) { return (uint32_t)__builtin_amdgcn_readlane((int)v, l); }
__device__ __forceinline__ double readlaned(double v, int l) {
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    return __longlong_as_double((long long)(((uint64_t)readlaneu((uint32_t)(b >> 32), l) << 32) | readlaneu((uint32_t)b, l)));
}
// value of lane `src` (any lane id; ds_bpermute)
__device__ __forceinline__ int shfl_idx(int v, int src) { return __builtin_amdgcn_ds_bpermute(src << 2, v); }

// One wave per workgroup: a wave's LDS and vector-memory instructions complete in order, so lanes
// exchanging data through LDS need only a compiler barrier (no memory-model fence: its
// `s_waitcnt lgkmcnt(0)` after every LDS write cost 0.4% on C2 and C3, profiles/r03/ab/wave_sync_ab.txt)
__device__ __forceinline__ void wave_sync() { __asm__ volatile("" ::: "memory"); __builtin_amdgcn_wave_barrier(); }
__device__ __forceinline__ int shfl_up1(int v) {     // lane i <- lane i-1 (lane 0 keeps its own)
    const int l = lane_id();
    return shfl_idx(v, l == 0 ? 0 : l - 1);
}
__device__ __forceinline__ int shfl_down1(int v) {   // lane i <- lane i+1 (lane 63 keeps its own)
    const int l = lane_id();
    return shfl_idx(v, l == 63 ? 63 : l + 1);
}

// 64-bit wave reductions without LDS: DPP butterflies inside rows, readlane across rows
template <int CTRL, bool MAX>
__device__ __forceinline__ uint64_t dpp_step64(uint64_t v) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)v, CTRL, 0xf, 0xf, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(v >> 32), CTRL, 0xf, 0xf, false);
    const uint64_t w = ((uint64_t)hi << 32) | lo;
    return MAX ? (w > v ? w : v) : (w | v);
}
template <bool MAX>
__device__ __forceinline__ uint64_t wave_reduce64(uint64_t v) {
    v = dpp_step64<0xB1, MAX>(v);    // quad_perm [1,0,3,2]
    v = dpp_step64<0x4E, MAX>(v);    // quad_perm [2,3,0,1]
    v = dpp_step64<0x141, MAX>(v);   // row_half_mirror
    v = dpp_step64<0x140, MAX>(v);   // row_mirror
    uint64_t m = 0;
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const uint64_t x = ((uint64_t)readlaneu((uint32_t)(v >> 32), 16 * r) << 32) | readlaneu((uint32_t)v, 16 * r);
        m = MAX ? (x > m ? x : m) : (m | x);
    }
    return m;
}
// uniform results (SGPR)
__device__ __forceinline__ uint64_t max_reduce64(uint64_t v) { return wave_reduce64<true>(v); }
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_max32(uint32_t v) {
    const uint32_t w = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xf, 0xf, false);
    return w > v ? w : v;
}
__device__ __forceinline__ uint32_t max_reduce32(uint32_t v) {
    v = dpp_max32<0xB1>(v);
    v = dpp_max32<0x4E>(v);
    v = dpp_max32<0x141>(v);
    v = dpp_max32<0x140>(v);
    uint32_t m = 0;
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const uint32_t x = readlaneu(v, 16 * r);
        m = x > m ? x : m;
    }
    return m;
}
__device__ __forceinline__ uint64_t or_reduce64(uint64_t v) { return wave_reduce64<false>(v); }
// wave sum (uniform): quad xor 1, xor 2, then the mirrored half-row / row partners (disjoint groups
// of equal sums at every step), one readlane per row
__device__ __forceinline__ uint32_t sum_reduce32(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xf, 0xf, false);    // quad_perm [1,0,3,2]
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xf, 0xf, false);    // quad_perm [2,3,0,1]
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xf, 0xf, false);   // row_half_mirror
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xf, 0xf, false);   // row_mirror
    return readlaneu(v, 0) + readlaneu(v, 16) + readlaneu(v, 32) + readlaneu(v, 48);
}

__device__ __forceinline__ uint32_t fmix32(uint32_t k) {   // HashTable.h:60-72
    k ^= k >> 16; k *= 0x85ebca6bu; k ^= k >> 13; k *= 0xc2b2ae35u; k ^= k >> 16;
    return k;
}
__device__ __forceinline__ int base_value(uint32_t c) {     // Tables.cpp:41-48
    return c == 'A' ? 0 : c == 'G' ? 1 : c == 'C' ? 2 : c == 'T' ? 3 : 4;
}
__device__ __forceinline__ uint32_t packed_code(uint32_t c) {   // bit-plane code (4 = not ACGT)
    return c == 'A' ? 0u : c == 'C' ? 1u : c == 'G' ? 2u : c == 'T' ? 3u : 4u;
}
__device__ __forceinline__ uint32_t complement_of(uint32_t c) {   // BaseAligner.cpp:148-152 (others -> 0)
    return c == 'A' ? 'T' : c == 'G' ? 'C' : c == 'C' ? 'G' : c == 'T' ? 'A' : c == 'N' ? 'N' : 0;
}

// ------------------------------------------------------------------ LDS
constexpr int64_t PACK_GUARD = 1024;     // bit-plane word 0 = genome position -1024
constexpr int EB = 8;                    // elements popped per batch (forced mode)
constexpr int CANDCAP = EB * ELEM;       // candidate list capacity
constexpr uint32_t ORDCAP = 128;         // forced-mode pop order window (u16; reads with more linked
                                         // elements rank in several windows, or radix-sort: radixMin)
// (256 entries were 0.35 ms faster at 4 waves/SIMD; 128 keep <128> within the 8 KB of 5 waves/SIMD)
constexpr uint32_t ordcap(int maxlen) { return maxlen <= 128 ? ORDCAP : 128u; }

// Scorer state of the bit-plane kernels align_kernel<128> / <256> (align_score.h); NW =
// 64-position words of the read masks.
template <int NW>
struct GroupLdsT {
    uint64_t rpl[2][3][NW];              // read[dir] bit planes {hi, lo, notACGT}, positions 0..64*NW-1
    uint32_t ecache[EB][16];             // popped Elem64s (authoritative while in the batch)
    uint32_t eidx[EB];
    uint16_t cand[CANDCAP];              // cand_* encoding below
    // LV path per [direction][group * GS/2 + row] (a group of GS lanes runs at k < GS/2, so rows
    // 1..k fit its GS/2 slots; 32 per direction): matched-run length and action (0 X, 1 D, 2 I);
    // probabilities in apply
    uint8_t pm[2][32];
    int8_t pa[2][32];
    int16_t pL0[2][8];                   //   exact prefix L[0][0] per group
    int8_t plen[2][8];                   //   path length (0: exact match, prob = perfect[patternLen])
};
using GroupLds = GroupLdsT<2>;
// A candidate list entry: bit [5:0], the element's slot in the popped batch [8:6], and -- for a
// candidate whose distances the forced-mode filter established (align_score.h forced_filter) --
// known [9], forward distance [12:10], reverse distance [15:13] (7: above the filter's limit).
__device__ __forceinline__ uint32_t cand_bit(uint32_t cw) { return cw & 63u; }
__device__ __forceinline__ uint32_t cand_slot(uint32_t cw) { return (cw >> 6) & 7u; }
__device__ __forceinline__ bool cand_known(uint32_t cw) { return (cw >> 9) & 1u; }
__device__ __forceinline__ int cand_e1(uint32_t cw) { return (int)((cw >> 10) & 7u); }
__device__ __forceinline__ int cand_e2(uint32_t cw) { return (int)((cw >> 13) & 7u); }
static_assert(EB <= 8 && ELEM <= 64, "cand_* encoding: 3-bit slot, 6-bit bit");

template <int MAXLEN>
struct Lds {
    static constexpr uint32_t ORD = ordcap(MAXLEN);
    static constexpr int NB = MAXLEN / 64;          // 64-position blocks
    static constexpr bool BYTE_PATH = MAXLEN > 256; // byte-compare LV (align_device.h) vs bit planes
    static constexpr int NW = BYTE_PATH ? 1 : NB;   // bit-plane mask words
    // The bit-plane kernels keep only the forward read: the reverse complement's planes are built
    // from it, its qualities read backwards.  The byte path keeps both, with 64 bytes of slack.
    static constexpr int RL = BYTE_PATH ? MAXLEN + 64 : MAXLEN;
    static constexpr int RCL = BYTE_PATH ? MAXLEN + 64 : 1;
    // element hash-chain heads: u16 on the bit-plane kernels (arenas capped below 0xffff elements,
    // snapgpu_aligner_create), u32 on the byte path (the big-arena pass's worst-case arenas)
    using HeadT = typename std::conditional<BYTE_PATH, uint32_t, uint16_t>::type;
    static constexpr HeadT HEAD_NONE = (HeadT)~(HeadT)0;
    char fwd[RL];                                   // read[FORWARD], zero slack
    char rc[RCL];                                   // read[RC] (byte path)
    char fwdQ[RL];
    char rcQ[RCL];
    uint32_t win[BYTE_PATH ? (MAXLEN + 192) / 4 : 1];   // genome window [g-64, g+n+64+64)
    HeadT head[NBUCKET];                            // element hash chains
    // hit insertion and scoring never overlap in time: their scratch shares LDS (the
    // insertion table is cleared again after every score call that used it)
    union {
        struct {
            uint32_t btKey[BT];
            uint64_t btMask[BT];
            uint32_t scrLoc[WAVE];                  // batch scratch: hit location per lane
        } ins;
        struct {
            // LV rows 1..MAX_K-1 (L + 2 per row, lane; actions recomputed; row 0 is never stored:
            // lv_rows() maps row e to rows8[e - 1]); between passes, the staged selection keys of
            // the forced-mode ranking
            alignas(16) uint8_t rows8[BYTE_PATH ? 1 : MAX_K - 1][WAVE];
            uint16_t order[ordcap(MAXLEN)];         // forced-mode pop order
        } sc;
    } u;
    uint64_t laneMax[WAVE];                         // per-owner-lane max (sortkey<<32 | idx)
    uint32_t nElems;
    uint32_t nSpill;                                // Elem64 spill blocks, taken from the arena's top
    uint32_t nUsed;                                 // nElems + nSpill: the arena is full at arenaElems
    uint32_t pad_[1];
    alignas(16) uint32_t sk[SKCAP];                 // selection keys of elements < SKCAP
    uint32_t ekey[MIRCAP];                          // element key / hash-chain link of elements < MIRCAP
    uint16_t enext[MIRCAP];                         //   (0xffff = end of chain)
    uint64_t seedUsed[NB + 1];                      // BaseAligner::seedUsed bit vector
    int16_t btAct[BYTE_PATH ? MAX_K + 1 : 1];       // LV backtrace scratch (byte path)
    int16_t btMatched[BYTE_PATH ? MAX_K + 1 : 1];
    uint16_t rows[BYTE_PATH ? MAX_K : 1][WAVE];     // byte-path LV rows: (L+2) | action<<12
    GroupLdsT<NW> grp[BYTE_PATH ? 0 : 1];           // scorer of align_kernel<128> / <256>
    // the read's first ELCAP candidate elements (Elem64) live here, not in the HBM arena
    alignas(16) uint32_t eloc[BYTE_PATH ? 1 : ELCAP][16];
};
// LV row e (1 <= e < MAX_K) of the bit-plane scorer at rows8[e - 1]
template <int MAXLEN>
__device__ __forceinline__ uint8_t (*lv_rows(Lds<MAXLEN> &S))[WAVE] {
    return reinterpret_cast<uint8_t (*)[WAVE]>(&S.u.sc.rows8[0][0] - WAVE);
}
// head of element hash chain h (NONE when empty)
template <int MAXLEN>
__device__ __forceinline__ uint32_t head_get(const Lds<MAXLEN> &S, uint32_t h) {
    const auto v = S.head[h];
    return v == Lds<MAXLEN>::HEAD_NONE ? NONE : (uint32_t)v;
}
// head[h] = e, returning the previous head (NONE when empty); leaders of one insertion step may
// share a bucket, so the exchange is atomic (a CAS on the dword holding a u16 head)
template <int MAXLEN>
__device__ __forceinline__ uint32_t head_exchange(Lds<MAXLEN> &S, uint32_t h, uint32_t e) {
    if constexpr (Lds<MAXLEN>::BYTE_PATH) {
        return atomicExch(&S.head[h], e);
    } else {
        uint32_t *w = reinterpret_cast<uint32_t *>(&S.head[h & ~1u]);
        const uint32_t sh = 16u * (h & 1u);
        uint32_t old = *w, assumed;
        do {
            assumed = old;
            old = atomicCAS(w, assumed, (assumed & ~(0xffffu << sh)) | ((e & 0xffffu) << sh));
        } while (old != assumed);
        const uint32_t o = (old >> sh) & 0xffffu;
        return o == 0xffffu ? NONE : o;
    }
}

// ------------------------------------------------------------ LV engine
// Per-lane mismatch bitmap over read positions m in [0, NB*64):
// bit m of F[m>>6] = (read[m] != genome[g + x + m]) with x = lane - 31, and
// positions m >= n forced to 1 (the byte past a pattern never matches genome).
template <int NB>
struct Bitmap { uint64_t w[NB]; };

// first set bit at position >= m0 (m0 >= 0); returns NB*64 if none
template <int NB>
__device__ __forceinline__ int bm_first_from(const Bitmap<NB> &F, int m0) {
    int r = NB * 64;
    bool found = false;
#pragma unroll
    for (int j = NB - 1; j >= 0; j--) {
        uint64_t x = F.w[j];
        int lo = j * 64;
        if (m0 > lo + 63) x = 0;
        else if (m0 > lo) x &= ~0ull << (m0 - lo);
        if (x) { r = lo + __builtin_ctzll(x); found = true; }
    }
    (void)found;
    return r;
}
// highest set bit at position <= m0; returns -1 if none (m0 may be < 0)
template <int NB>
__device__ __forceinline__ int bm_last_upto(const Bitmap<NB> &F, int m0) {
    int r = -1;
#pragma unroll
    for (int j = 0; j < NB; j++) {
        uint64_t x = F.w[j];
        int lo = j * 64;
        if (m0 < lo) x = 0;
        else if (m0 < lo + 63) x &= (2ull << (m0 - lo)) - 1;
        if (x) r = lo + 63 - __builtin_clzll(x);
    }
    return r;
}
template <int NB>
__device__ __forceinline__ bool bm_bit(const Bitmap<NB> &F, int m) {
    if (m < 0 || m >= NB * 64) return true;
    bool b = false;
#pragma unroll
    for (int j = 0; j < NB; j++)
        if ((m >> 6) == j) b = (F.w[j] >> (m & 63)) & 1;
    return b;
}

// Build F for lanes x in [-kmax, kmax]; lane i of block b holds read byte rb[b].
// win: LDS bytes with win[w0 + p] = genome[g + p] for p in [-64, n + 64).
template <int NB>
__device__ __forceinline__ void build_bitmap(Bitmap<NB> &F, const uint32_t (&rbF)[NB], const uint32_t (&rbR)[NB],
                                             bool useR, const char *win, int w0, int n, int kmax) {
    const int lane = lane_id();
#pragma unroll
    for (int b = 0; b < NB; b++) { F.w[b] = ~0ull; }
    for (int x = -kmax; x <= kmax; x++) {
        const int tl = 31 + x;
#pragma unroll
        for (int b = 0; b < NB; b++) {
            if (b * 64 < n) {
                int m = b * 64 + lane;
                uint32_t gbyte = (uint8_t)win[w0 + x + m];
                uint32_t rbyte = useR ? rbR[b] : rbF[b];
                bool mm = (m >= n) || (gbyte != rbyte);
                uint64_t mask = ballot(mm);
                if (lane == tl) F.w[b] = mask;   // v_cndmask from the SGPR ballot
            }
        }
    }
}

struct LvOut { int score; int netIndel; double prob; };

// LandauVishkin<DIR>::computeEditDistance on the wave.  Pattern index i maps to
// read position m = p0 + DIR*i; text position j of diagonal d maps to the
// bitmap of x = DIR*d.  textLen only bounds end_d = min(patternLen, textLen-d).
// qual: LDS quality in read coordinates.  rows: LDS row history.
template <int DIR, int NB>
__device__ __forceinline__ LvOut lv_wave(const Bitmap<NB> &F, int p0, int patternLen, int textLen, int k,
                                         const char *qual, uint16_t (*rows)[WAVE], int16_t *btAct,
                                         int16_t *btMatched, const DevTables *tab) {
    const int lane = lane_id();
    LvOut r;
    r.netIndel = 0;
    if (k > MAX_K - 1) k = MAX_K - 1;
    const int d = DIR > 0 ? lane - 31 : 31 - lane;   // diagonal held by this lane
    // row 0 (exact prefix), diagonal 0 lives on lane 31
    int end0 = patternLen < textLen ? patternLen : textLen;
    int L0;
    {
        int fm;
        if (DIR > 0) fm = bm_first_from(F, p0) - p0;
        else fm = p0 - bm_last_upto(F, p0);
        int v = fm < end0 ? fm : end0;
        L0 = unii(readlane(v, 31));
    }
    if (L0 == end0) {
        int result = patternLen > end0 ? patternLen - end0 : 0;
        r.prob = g_tab.perfect[patternLen];
        r.score = result > k ? -1 : result;
        return r;
    }
    int Lp = (lane == 31) ? L0 : -2;
    if (lane == 31) rows[0][31] = (uint16_t)(L0 + 2);
    int endd = patternLen < textLen - d ? patternLen : textLen - d;
    for (int e = 1; e <= k; e++) {
        // neighbours: diagonal d-1 and d+1
        int nUp = shfl_up1(Lp), nDn = shfl_down1(Lp);
        int left = DIR > 0 ? nUp : nDn;           // L[e-1][d-1]
        int right = (DIR > 0 ? nDn : nUp) + 1;    // L[e-1][d+1] + 1
        int best = Lp + 1, act = 0;               // 0 = X, 1 = D, 2 = I
        if (left > best) { best = left; act = 1; }
        if (right > best) { best = right; act = 2; }
        bool active = (d <= e) && (d >= -e);
        // extension (LandauVishkin.h:325-354)
        int mpos = p0 + DIR * best;
        if (best < endd) {
            int fm;
            if (DIR > 0) fm = bm_first_from(F, mpos) - p0;
            else fm = p0 - bm_last_upto(F, mpos);
            best = fm < endd ? fm : endd;
        } else {
            if (!bm_bit(F, mpos)) best = endd;
        }
        int Ln = active ? best : Lp;
        if (active) rows[e][lane] = (uint16_t)((Ln + 2) | (act << 12));
        uint64_t done = ballot(active && Ln == patternLen);
        if (done) {
            // first d in the order 0, 1, -1, 2, -2, ... (LandauVishkin.h:180-182)
            int wd = 0;
            for (int j = 0; j <= e; j++) {
                int lp = DIR > 0 ? 31 + j : 31 - j;
                int ln = DIR > 0 ? 31 - j : 31 + j;
                if ((done >> lp) & 1) { wd = j; break; }
                if (j > 0 && ((done >> ln) & 1)) { wd = -j; break; }
            }
            wd = unii(wd);
            wave_sync();
            // backtrace (LandauVishkin.h:376-431); uniform work, scratch in LDS
            int curD = wd;
            for (int ce = e; ce >= 1; ce--) {
                int ln = DIR > 0 ? 31 + curD : 31 - curD;
                uint32_t cell = uni(rows[ce][ln]);
                int a = (int)(cell >> 12);
                int Lcur = (int)(cell & 0xfff) - 2;
                int src = a == 2 ? curD + 1 : (a == 1 ? curD - 1 : curD);
                int ls = DIR > 0 ? 31 + src : 31 - src;
                int Lsrc = (ce - 1 == 0) ? (src == 0 ? L0 : -2) : ((int)(uni(rows[ce - 1][ls]) & 0xfff) - 2);
                if (lane == 0) {
                    btAct[ce] = (int16_t)a;
                    btMatched[ce] = (int16_t)(a == 1 ? Lcur - Lsrc : Lcur - Lsrc - 1);
                }
                curD = src;
            }
            wave_sync();
            double p = 1.0;
            int ce = 1, offset = L0, net = 0;
            while (ce <= e) {
                int a = unii(btAct[ce]);
                int cnt = 1;
                while (ce + 1 <= e && unii(btMatched[ce]) == 0 && unii(btAct[ce + 1]) == a) { cnt++; ce++; }
                if (a == 2) { p *= g_tab.indel[cnt]; offset += cnt; net += cnt; }
                else if (a == 1) { p *= g_tab.indel[cnt]; offset -= cnt; net -= cnt; }
                else {
                    for (int q = 0; q < cnt; q++) {
                        int qi = offset < 0 ? 0 : offset;
                        if (qi > patternLen - 1) qi = patternLen - 1;
                        uint32_t qc = uni((uint8_t)qual[p0 + DIR * qi]);
                        p *= g_tab.phred[qc];
                        offset++;
                    }
                }
                offset += unii(btMatched[ce]);
                ce++;
            }
            p *= g_tab.perfect[patternLen - e];
            r.score = e;
            r.prob = p;
            r.netIndel = net;
            return r;
        }
        Lp = Ln;
    }
    r.score = -1;
    r.prob = 1.0;   // LandauVishkin.h:259: left at 1.0 when no alignment within k
    return r;
}

// Stage genome bytes [g - 64, g + n + 128) into LDS window (4-byte aligned start).
// Returns w0 such that win[w0 + p] == genome[g + p].
template <int MAXLEN>
__device__ __forceinline__ int stage_window(Lds<MAXLEN> &S, const char *genome, uint32_t g, int n) {
    const int lane = lane_id();
    int64_t start = (int64_t)g - 64;
    int64_t astart = start & ~(int64_t)3;
    int nwords = (n + 192 + 4) / 4;
    const uint32_t *src = (const uint32_t *)(genome + astart);
    for (int i = lane; i < nwords && i < (MAXLEN + 192) / 4; i += WAVE) S.win[i] = src[i];
    wave_sync();
    return (int)((int64_t)g - astart);
}

// Genome::getSubstring (Genome.h:78-148): is [offset, offset+len) servable?
template <class G>   // KArgs, CigarArgs: anything with nBases, padding, pieces, nPieces
__device__ __forceinline__ bool substring_ok(const G &A, uint32_t offset, uint32_t len) {
    if (offset > A.nBases || (uint64_t)offset + len > (uint64_t)A.nBases + NPAD) return false;
    if (len <= A.padding) return true;
    if (A.nPieces > 100) {
        if (A.pieces[A.nPieces - 1] <= offset) return true;
        int lo = 0, hi = A.nPieces - 2;
        while (lo <= hi) {
            int m = (lo + hi) / 2;
            if (A.pieces[m] <= offset) {
                if (A.pieces[m + 1] > offset) return !(A.pieces[m + 1] <= offset + len - 1);
                lo = m + 1;
            } else hi = m - 1;
        }
        return false;
    }
    for (int i = 0; i < A.nPieces; i++)
        if (offset + len - 1 >= A.pieces[i]) return !(offset < A.pieces[i]);
    return false;
}
__device__ __forceinline__ int next_piece_after(const KArgs &A, uint32_t loc) {   // Genome.cpp:376-401
    int lo = 0, hi = A.nPieces - 1;
    while (lo <= hi) {
        int m = (lo + hi) / 2;
        if (A.pieces[m] <= loc && (m == A.nPieces - 1 || A.pieces[m + 1] > loc)) return m >= A.nPieces - 1 ? -1 : m + 1;
        else if (A.pieces[m] <= loc) lo = m + 1;
        else hi = m - 1;
    }
    return -1;
}

// ------------------------------------- multi-hit export / windowed lookups
// BaseAligner.cpp:1255-1261: remember a scored hit (score != -1) while fewer than
// maxHitsToGet are held at that distance.  The scratch is per block; lane 0 owns it.
// The reference's table is hitLocations[MAX_K][512] / hitRCs[MAX_K][512] (BaseAligner.h:
// 148-151) indexed [score][hitCount[score]] with hitCount < maxHitsToGet: for maxHitsToGet >
// 512 (the RNA paired path asks for 1000, PairedAligner.cpp:584) entries 512.. of a distance
// land in the next distances' rows.  The flat index score * hitSlot + count keeps exactly
// that aliasing (hitSlot = 512 then; = maxHitsToGet below, where nothing aliases).
template <bool EXT>
__device__ __forceinline__ void record_hit(const KArgs &A, uint32_t loc, uint32_t dir, uint32_t sc) {
    if (!EXT || A.maxHitsToGet == 0 || sc >= (uint32_t)MAX_K) return;
    if (lane_id() == 0) {
        uint32_t *cnt = A.hitScratch + (uint64_t)blockIdx.x * A.hitStride;
        const uint32_t c = cnt[sc];
        if (c < A.maxHitsToGet) {
            uint32_t *h = cnt + MAX_K + 2 * (sc * A.hitSlot + c);
            h[0] = loc;
            h[1] = dir;
            cnt[sc] = c + 1;
        }
    }
}

// BaseAligner::fillHitsFound (BaseAligner.cpp:940-975) from the block's scratch, lane 0
__device__ __forceinline__ void fill_hits(const KArgs &A, uint32_t r, bool fill) {
    if (lane_id() != 0) return;
    int32_t found = 0;
    if (fill) {
        const uint32_t *cnt = A.hitScratch + (uint64_t)blockIdx.x * A.hitStride;
        snapgpu_multi_hit_t *out = A.multiHits + (uint64_t)r * A.maxHitsToGet;
        int first = 0;
        while (first < MAX_K && cnt[first] == 0) first++;
        for (int d = first; d < first + 4 && d < MAX_K; d++) {
            const uint32_t c = cnt[d];
            bool full = false;
            for (uint32_t i = 0; i < c; i++) {
                const uint32_t *h = cnt + MAX_K + 2 * (d * A.hitSlot + i);
                snapgpu_multi_hit_t m;
                m.location = h[0];
                m.direction = (uint8_t)h[1];
                m.score = (uint8_t)d;
                m.reserved = 0;
                out[found++] = m;
                if ((uint32_t)found == A.maxHitsToGet) { full = true; break; }
            }
            if (full) break;
        }
    }
    A.multiFound[r] = found;
}

// Number of leading entries > x of a list sorted in descending order (the overflow
// hit lists, GenomeIndex.cpp:1057-1075): 64-way search, each round shrinks the
// candidate range 64-fold.  Wave-uniform.
__device__ __forceinline__ uint32_t count_above_desc(const uint32_t *L, uint32_t cnt, uint32_t x) {
    uint32_t lo = 0, hi = cnt;
    while (lo < hi) {
        const uint32_t step = (hi - lo + 63) / 64;
        const uint32_t pos = lo + (uint32_t)lane_id() * step;
        const uint32_t t = (uint32_t)__popcll(ballot(pos < hi && L[pos] > x));
        if (t == 0) break;
        const uint32_t nlo = lo + (t - 1) * step + 1;
        hi = hi < lo + t * step ? hi : lo + t * step;
        lo = nlo;
    }
    return lo;
}

// ------------------------------------------------------- phase diagnostics
// With KArgs::phaseBuf set, lane 0 of each wave adds s_memtime deltas per phase (and
// event counts) to its block's slice with no-return atomics (snapgpu_phase_cycles).
// Compiled in only with -DSNAPGPU_PHASE_TIMERS=1 (`make PHASE_TIMERS=1`): even switched off
// at run time, the timestamps held across loops cost SGPR spills in the production kernel.
enum : int { PH_SETUP = 0, PH_LOOKUP, PH_INSERT, PH_SCORE, PH_POP, PH_NLVFU, PH_STAGE, PH_LVF, PH_LVR, PH_APPLY,
             PH_WB, PH_OUT, PH_NPASS, PH_NCAND, PH_NLVF2, PH_NPASS16, PH_NPASS32, PH_NPASS64, PH_ROWSF, PH_ROWSR,
             PH_NSCORECALL, PH_NFORCED, PH_NPOPPED, PH_NSUCC, PH_PASSLOOP, PH_SEL, PH_FETCH, PH_SEEDLOOP, PH_NBATCH,
             PH_RANK, PH_NELEMSF, PH_CANDL, PH_SUCC, PH_NEARBY, PH_PROB, PH_FAILS, PH_NFAILSTEP, PH_SUCCWB,
             PH_NPASSF, PH_PASSLOOPF, PH_HEAVYCYC, PH_NHEAVY, PH_NCANDF, PH_READCYC, PH_NFILTER, PH_NLVF, PH_NLVFK, PH_NFRES,
             PH_SLOTS = 48 };
__device__ __forceinline__ uint64_t clk() { return __builtin_amdgcn_s_memtime(); }
#if SNAPGPU_PHASE_TIMERS
#define PH_T(A, v) const uint64_t v = (A).phaseBuf ? sgk::clk() : 0
#define PH_ADD(A, S, i, v) do { if ((A).phaseBuf && sgk::lane_id() == 0) \
    atomicAdd((A).phaseBuf + blockIdx.x * sgk::PH_SLOTS + (i), (unsigned long long)(sgk::clk() - (v))); } while (0)
#define PH_CNT(A, S, i, n) do { if ((A).phaseBuf && sgk::lane_id() == 0) \
    atomicAdd((A).phaseBuf + blockIdx.x * sgk::PH_SLOTS + (i), (unsigned long long)(n)); } while (0)
#else
#define PH_T(A, v)
#define PH_ADD(A, S, i, v) do { } while (0)
#define PH_CNT(A, S, i, n) do { } while (0)
#endif

// computeMAPQ (mapq.h:32-65) without log10: floor(-10*log10(x)) >= q  <=>  x <= 10^(-q/10).
// A ratio within 1e-9 (relative) of a threshold is flagged and re-derived on the host
// with glibc log10 (SNAPGPU_FLAG_MAPQ_FIXED), so boundary rounding cannot differ.
__device__ __forceinline__ int mapq_dev(const DevTables *tab, double pAll, double pBest, uint32_t score,
                                        uint32_t popular, uint32_t *flags) {
    if (pAll < pBest) pAll = pBest;
    if (pAll == pBest && popular == 0 && score < 5) return 70;
    const double c = pBest / pAll;
    int mq;
    if (c >= 1) mq = 69;
    else {
        const double x = 1 - c;
        int lo = 0, hi = 69;                 // largest q in [0, 69] with x <= T[q] (T[0] = 1 >= x)
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (x <= g_tab.mapqT[mid]) lo = mid; else hi = mid - 1;
        }
        mq = lo;
        const double t0 = g_tab.mapqT[lo], t1 = g_tab.mapqT[lo + 1];
        if (fabs(x - t0) <= 1e-9 * t0 || fabs(x - t1) <= 1e-9 * t1) *flags |= SNAPGPU_FLAG_MAPQ_FIXED;
    }
    int pen = (int)popular - 10;
    if (pen < 0) pen = 0;
    mq -= pen / 2;
    return mq < 0 ? 0 : mq;
}

// ------------------------------------------------------------ per-read state
// Device watchdog: loops whose bound rests on data-structure invariants carry an
// iteration cap; tripping one records (code, read, detail) here, ends the read and
// makes the host call fail instead of hanging the GPU.
enum : uint32_t { DIAG_SEED_LOOP = 1, DIAG_SCORE_LOOP = 2, DIAG_CHAIN = 3, DIAG_BATCH_TABLE = 4, DIAG_ARENA = 5,
                  DIAG_TEST_TRIP = 6, DIAG_OVERDUE = 16 };
// A read that runs longer than this (100 MHz s_memrealtime ticks, 2 s) is abandoned.
constexpr uint64_t READ_DEADLINE_TICKS = 200000000ull;
// The record is the aligner's own device allocation (KArgs::diag), so aligners that share a
// device (the RNA path's transcriptome and genome aligners on two host threads) neither clear
// nor trip each other's record.
__device__ __forceinline__ void diag_report(uint32_t *d, uint32_t code, uint32_t a, uint32_t b) {
    if (atomicCAS(&d[0], 0u, code) == 0u) { d[1] = a; d[2] = b; }
}

struct ReadState {
    uint32_t lps[2], mostSeeds[2], nSeedsApplied[2];
    uint32_t bestScore, bestLoc, scoreLimit;
    double pAll, pBest;
    uint32_t outLoc, outDir;
    int32_t outScore, outMapq;
    uint32_t ts;                 // running hit counter (FIFO timestamps)
    uint32_t statv;              // per-read counters, one per lane (SV_*): a VGPR instead of 6 SGPRs
    uint32_t rid;                // read index (watchdog reports)
    uint32_t abort;              // watchdog tripped (1) or capped arena full (2): finish the read now
    uint32_t tick;               // overdue(): calls left until the next clock read
    uint64_t t0;                 // s_memrealtime at read start
};

// per-read statistics: lane SV_x of ReadState::statv
enum : int { SV_LOOKUPS = 0, SV_SCORED = 1, SV_POPULAR = 2, SV_PROBES = 3, SV_HITWORDS = 4, SV_OVF = 5 };
__device__ __forceinline__ void sv_add(ReadState &st, int lane, int idx, uint32_t v) { st.statv += lane == idx ? v : 0u; }
__device__ __forceinline__ uint32_t sv_get(const ReadState &st, int idx) { return readlaneu(st.statv, idx); }

// time watchdog: true (once reported) when the read has overrun its deadline.  The
// clock (an SMEM round trip) is read on every 32nd call only.
__device__ __forceinline__ bool overdue(const KArgs &A, ReadState &st, uint32_t site) {
    if (st.abort) return true;
    if (--st.tick != 0) return false;
    st.tick = 32;
    if (__builtin_amdgcn_s_memrealtime() - st.t0 < READ_DEADLINE_TICKS) return false;
    if (lane_id() == 0) diag_report(A.diag, DIAG_OVERDUE + site, st.rid, (uint32_t)((__builtin_amdgcn_s_memrealtime() - st.t0) >> 10));
    st.abort = 1;
    return true;
}

__device__ __forceinline__ uint32_t elem_hash(uint32_t key) { return (key * 2654435761u) >> (32 - NBUCKET_LOG2); }

// find element with `key`; NONE if absent.  Elements < MIRCAP keep (key, next) in LDS
// (next always points to an older, smaller index), so most walks never touch HBM.
template <int MAXLEN>
__device__ __forceinline__ uint32_t chain_find(const KArgs &A, const Lds<MAXLEN> &S, const ElemOf<MAXLEN> *ar, uint32_t key,
                                               uint32_t cap) {
    uint32_t e = head_get(S, elem_hash(key));
    for (uint32_t steps = 0; e != NONE; steps++) {
        if (steps > cap) { diag_report(A.diag, DIAG_CHAIN, key, e); return NONE; }
        if (e < MIRCAP) {
            if (S.ekey[e] == key) break;
            const uint32_t nx = S.enext[e];
            e = nx == 0xffffu ? NONE : nx;
        } else {
            if (ar[e].key == key) break;
            e = ar[e].next;
        }
    }
    return e;
}

// selection keys: LDS for the first SKCAP elements of a read, HBM (the element) beyond.  (A compact
// owner-transposed HBM key array -- one coalesced load per selection recompute -- measured 3% slower
// on C2 and 5% on C3 in round 3: profiles/r03/ab/compact_sk_ab.txt.)
// (The asm after the HBM load keeps the two loads apart: merged into one load of a selected
// pointer they became a flat load, which waits on both the LDS and the vector-memory counters.)
template <int MAXLEN>
__device__ __forceinline__ uint32_t sk_get(const KArgs &, const Lds<MAXLEN> &S, const ElemOf<MAXLEN> *ar, uint32_t e) {
    uint32_t v;
    if (e < SKCAP) v = S.sk[e];
    else { v = ar[e].sortkey; __asm__ volatile("" :: "v"(v)); }
    return v;
}
template <int MAXLEN>
__device__ __forceinline__ void sk_set(const KArgs &, Lds<MAXLEN> &S, ElemOf<MAXLEN> *ar, uint32_t e, uint32_t v) {
    if (e < SKCAP) S.sk[e] = v;
    else ar[e].sortkey = v;
}

// recompute of `owner`'s selection maximum (elements e == owner mod 64), the whole wave
// scanning that lane's elements 64 at a time
template <int MAXLEN>
__device__ __forceinline__ void recompute_lane_max(const KArgs &A, Lds<MAXLEN> &S, const ElemOf<MAXLEN> *ar, int owner) {
    const int lane = lane_id();
    uint64_t best = 0;
    const uint32_t nElems = S.nElems;
#pragma unroll 1
    for (uint32_t b = (uint32_t)owner; b < nElems; b += WAVE * WAVE) {
        const uint32_t e = b + WAVE * (uint32_t)lane;
        const uint32_t k = e < nElems ? sk_get(A, S, ar, e) : 0u;
        const uint64_t v = ((uint64_t)k << 32) | e;
        if (k && v > best) best = v;
    }
    best = max_reduce64(best);
    if (lane == owner) S.laneMax[owner] = best;
}

// uniform field extraction from a cooperatively loaded element (lane i = dword i)
__device__ __forceinline__ uint32_t rl(uint32_t v, int k) { return (uint32_t)__builtin_amdgcn_readlane((int)v, k); }
__device__ __forceinline__ uint64_t rl64(uint32_t v, int k) { return ((uint64_t)rl(v, k + 1) << 32) | rl(v, k); }
__device__ __forceinline__ double rld(uint32_t v, int k) { return __longlong_as_double((long long)rl64(v, k)); }

}  // namespace sgk
