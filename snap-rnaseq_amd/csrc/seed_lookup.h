// seed_lookup.h -- the first SEEDS_PER_READ seed lookups of every read, resolved up front.
//
// In BaseAligner::AlignRead the sequence of seed offsets is 0, seedLen, 2*seedLen, ...,
// then the wrapped rounds (GetWrappedNextSeedToTest, skipping offsets already used; a seed
// containing a non-ACGT base is marked used and skipped without the +seedLen advance;
// BaseAligner.cpp:686-746): it depends only on the read's bases, not on any lookup result --
// results decide only how far along it a read gets.  seed_lookup_kernel resolves
// GenomeIndex::lookupSeed (GenomeIndex.cpp:971-1086, SNAPHashTable::Lookup HashTable.h:74-105)
// for the first 16 seeds of that sequence for every read <= 128 bases, one lane per (read, seed):
// 4 reads per wave, thousands of independent probe chains in flight, so the hash-table gather
// runs at memory throughput instead of as ~3 dependent HBM round trips inside each read's
// sequential aligner.  align_kernel<128> consumes the records when its seed loop reaches the same
// offset and counts probes / overflow lists exactly as before (a read that stops earlier leaves
// its later records unused).  Of a longer read it resolves the first-round seeds that lie in its
// first 128 bases -- a prefix of the same sequence, which align_kernel<256> consumes the same way --
// and weighs the read by their summed hit counts: the long reads go onto pass 2's list heaviest
// first (order_long_kernel), so a read that scores thousands of candidates starts at the head of
// the persistent kernel instead of finishing alone at its tail.  Results do not depend on the order.
//
// The lookups go to the bucket image of the tables (bucket_table.h): one 64-B line per lookup in
// the common case, the overflow-list lengths carried in the entry.
#pragma once
#include "align_device.h"
#include "bucket_table.h"
#include "order_long.h"

namespace sgk {

// 16 bytes per (read, seed k of the sequence, k < SEEDS_PER_READ)
struct SeedRec {
    uint32_t meta;      // bit31 valid, [7:0] offset, bit8 found, bit9 comp, bit10 palindrome, [30:16] probes
    uint32_t v1, v2;    // slot values (GenomeIndex.cpp:1004-1010 swaps them when comp)
    uint32_t cnt;       // overflow counts, u16 each, saturated: [15:0] value1 side, [31:16] value2 side
};
constexpr int SEEDS_PER_READ = 16;   // = lanes per read in seed_lookup_kernel: 4 reads per wave
constexpr int LOOKUP_WAVES = 4;      // waves per seed_lookup_kernel block (16 reads)

// bits [p, p+len) of a 128-bit value (len <= 32)
__device__ __forceinline__ uint32_t win128(uint64_t lo, uint64_t hi, int p, int len) {
    uint64_t w;
    if (p == 0) w = lo;
    else if (p < 64) w = (lo >> p) | (hi << (64 - p));
    else w = hi >> (p - 64);
    return (uint32_t)w & (uint32_t)((1ull << len) - 1);
}
// bit i -> bit 2i
__device__ __forceinline__ uint64_t spread2(uint32_t x32) {
    uint64_t x = x32;
    x = (x | (x << 16)) & 0x0000FFFF0000FFFFull;
    x = (x | (x << 8)) & 0x00FF00FF00FF00FFull;
    x = (x | (x << 4)) & 0x0F0F0F0F0F0F0F0Full;
    x = (x | (x << 2)) & 0x3333333333333333ull;
    x = (x | (x << 1)) & 0x5555555555555555ull;
    return x;
}

// stats[4*slot + 0..2] += seeds looked up, hash entries probed, overflow counts read (roofline
// bytes); slot = block % 256
__global__ __launch_bounds__(64 * LOOKUP_WAVES) void seed_lookup_kernel(KArgs A, SeedRec *out, unsigned long long *stats) {
    // the wrap table (GetWrappedNextSeedToTest order) in LDS: the walk below reads it per lane
    __shared__ uint32_t wrapT[32];
    if (threadIdx.x < 32) wrapT[threadIdx.x] = A.tab->wrap[threadIdx.x];
    __syncthreads();
    const int lane = lane_id();
    const uint32_t r = (blockIdx.x * LOOKUP_WAVES + threadIdx.x / 64) * 4 + (lane >> 4);
    const int k = lane & 15;
    const int sub = k & 7;          // lanes k < 8 load the read, 16 bases each
    const bool have = r < A.nReads;
    const uint32_t n = have ? A.lengths[r] : 0;
    const uint64_t off = have ? A.offsets[r] : 0;
    const int L = (int)A.seedLen;
    // 16 bases per lane (read buffer carries >= 64 bytes of slack past the last read)
    uint64_t chunk = 0;   // [15:0] bit0 of the seed code, [31:16] bit1, [47:32] not-ACGT / past the end
    bool bad = false;     // a base of the read (position < n) that is not ACGT
    {
        const uint64_t b0 = off + 16 * (uint64_t)sub;
        const uint32_t *src = (const uint32_t *)(A.bases + (b0 & ~3ull));
        const uint32_t sh = (uint32_t)(b0 & 3) * 8;
        uint32_t w[5];
#pragma unroll
        for (int i = 0; i < 5; i++) w[i] = have && k < 8 && n > 16u * sub ? src[i] : 0u;
        // branch-free per byte: upper-case (Read::init, Read.h:289-328), the seed code A0 G1 C2 T3
        // (Tables.cpp:41-48) from bits 2:1 of the upper-cased letter (A 00, C 01, G 11, T 10), and
        // ACGT membership from a bit mask over 0x40..0x5f
        uint32_t p0 = 0, p1 = 0, iv = 0;   // 16 positions each: code bit 0, code bit 1, not ACGT
        const int lim = (int)n - 16 * sub;   // positions of this lane's 16 that lie in the read
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const uint32_t d = __builtin_amdgcn_alignbit(w[i + 1], w[i], sh);
#pragma unroll
            for (int b = 0; b < 4; b++) {
                const uint32_t c = (d >> (8 * b)) & 0xffu;
                const uint32_t uc = (c >= 'a' && c <= 'z') ? c - 0x20u : c;
                const uint32_t o = uc - 0x40u;
                constexpr uint32_t kAcgt = (1u << 1) | (1u << 3) | (1u << 7) | (1u << 20);   // A C G T
                const bool acgt = o < 32u && ((kAcgt >> (o & 31u)) & 1u);
                const uint32_t x0 = (uc >> 1) & 1u, x1 = (uc >> 2) & 1u;
                const int bit = 4 * i + b;
                const bool inside = bit < lim;
                const bool inv = !inside || !acgt;
                bad |= k < 8 && inside && !acgt;   // (lanes 8..15 load nothing)
                p0 |= (inv ? 0u : x1) << bit;               // code bit 0: A 0, G 1, C 0, T 1
                p1 |= (inv ? 0u : (x0 ^ x1)) << bit;        // code bit 1: A 0, G 0, C 1, T 1
                iv |= (inv ? 1u : 0u) << bit;
            }
        }
        chunk = (uint64_t)p0 | ((uint64_t)p1 << 16) | ((uint64_t)iv << 32);
    }
    SeedRec rec = {0u, 0u, 0u, 0u};
    uint32_t weight = 0;   // a long read's seed: its hit count (0: popular or not found)
    uint32_t nSeed = 0, nProbe = 0, nOvfRead = 0;
    const int grp = lane & ~15;
    const uint64_t badMask = ballot(bad);
    const bool can = have && (int)n >= L;
    const bool lng = n > 128;   // records: the first-round seeds inside positions 0..127 only
    const int firstRound = 128 / L;   // of a long read: offsets 0, L, .., (firstRound - 1) L (all-ACGT prefix)
    int my = -1;             // offset of this lane's seed k of the sequence (-1: none)
    uint32_t w0 = 0, w1 = 0;   // code bits 0 and 1 of the seed's positions my .. my + L - 1
    if (badMask == 0) {
        // every read of the wave is all ACGT: its sequence of seed offsets depends on its length
        // alone (a table entry), and a seed's bits come from the three chunks it can span
        if (can && !lng) {
            const uint32_t t = A.tab->seedSeq[n][k];
            my = t == 0xffu ? -1 : (int)t;
        } else if (can) my = k < firstRound ? k * L : -1;
        const int c0 = my > 0 ? my >> 4 : 0;
        const uint32_t a = (uint32_t)shfl_idx((int)(uint32_t)chunk, grp + c0);
        const uint32_t b = (uint32_t)shfl_idx((int)(uint32_t)chunk, grp + (c0 + 1 < 8 ? c0 + 1 : 7));
        const uint32_t c = (uint32_t)shfl_idx((int)(uint32_t)chunk, grp + (c0 + 2 < 8 ? c0 + 2 : 7));
        const uint64_t q0 = (uint64_t)(a & 0xffffu) | ((uint64_t)(b & 0xffffu) << 16) | ((uint64_t)(c & 0xffffu) << 32);
        const uint64_t q1 = (uint64_t)(a >> 16) | ((uint64_t)(b >> 16) << 16) | ((uint64_t)(c >> 16) << 32);
        const int sh = my > 0 ? my - 16 * c0 : 0;
        const uint32_t M = (uint32_t)((1ull << L) - 1);
        w0 = (uint32_t)(q0 >> sh) & M;
        w1 = (uint32_t)(q1 >> sh) & M;
    } else {
        // the read's full 128-position planes in every lane of its group
        uint64_t P0[2] = {0, 0}, P1[2] = {0, 0}, IV[2] = {0, 0};
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const int src = grp + j;
            const uint32_t lo = (uint32_t)shfl_idx((int)(uint32_t)chunk, src);
            const uint32_t hi = (uint32_t)shfl_idx((int)(uint32_t)(chunk >> 32), src);
            const int wd = j >> 2, s = 16 * (j & 3);
            P0[wd] |= (uint64_t)(lo & 0xffff) << s;
            P1[wd] |= (uint64_t)(lo >> 16) << s;
            IV[wd] |= (uint64_t)(hi & 0xffff) << s;
        }
        const bool clean = ((badMask >> grp) & 0xffffull) == 0;
        if (can) {
            // offset of the k-th seed of the sequence (BaseAligner.cpp:686-746), simulated with the
            // read's seedUsed bits: rounds 0, seedLen, ... then the wrap table's starts
            const int nPossible = (lng ? 128 : (int)n) - L + 1;
            uint64_t u0 = 0, u1 = 0;   // seedUsed, positions 0..127
            int p = 0, wrap = 0, idx = 0;
            if (clean && lng) my = k < firstRound ? k * L : -1;
            else if (clean) {
                const uint32_t t = A.tab->seedSeq[n][k];
                my = t == 0xffu ? -1 : (int)t;
            }
#pragma nounroll
            for (int guard = 0; !clean && guard < 4 * 128; guard++) {   // each step marks, wraps or ends
                if (p >= nPossible) {
                    if (lng || ++wrap >= L) break;               // wrapCount == seedLen: the read is scored
                    p = (int)wrapT[wrap];
                }
#pragma clang loop vectorize(disable) interleave(disable) unroll(disable)
                while (p < nPossible && (((p < 64 ? u0 >> p : u1 >> (p - 64)) & 1ull) != 0)) p++;   // (rolled: rare path)
                if (p >= nPossible) continue;
                if (p < 64) u0 |= 1ull << p; else u1 |= 1ull << (p - 64);
                if (win128(IV[0], IV[1], p, L)) continue;        // not a seed: used, no advance (:740-744)
                if (idx == k) { my = p; break; }
                idx++;
                p += L;
            }
            if (my >= 0) { w0 = win128(P0[0], P0[1], my, L); w1 = win128(P1[0], P1[1], my, L); }
        }
    }
    {
        const uint32_t M = (uint32_t)((1ull << L) - 1);
        // Seed.h:38-51: first base most significant; reverse complement = reverse of code ^ 3
        const uint32_t r0 = __builtin_bitreverse32(w0) >> (32 - L), r1 = __builtin_bitreverse32(w1) >> (32 - L);
        const uint64_t f = (spread2(r1) << 1) | spread2(r0);
        const uint64_t rcv = (spread2(~w1 & M) << 1) | spread2(~w0 & M);
        const bool comp = (int64_t)f > (int64_t)rcv;
        const uint64_t canon = comp ? rcv : f;
        const uint32_t table = (uint32_t)(canon >> 32);
        const uint32_t key = (uint32_t)canon;
        // SNAPHashTable::Lookup's answer from the bucket image: one 64-B line per bucket visited,
        // four lanes per line (the whole wave takes part)
        uint32_t v1 = 0, v2 = 0, aux = 0, probes = 0;
        const bool found = bucket_lookup_quad(A, my >= 0, table, key, v1, v2, aux, probes);
        if (my >= 0 && found && lng) {   // the long read's weight: hits of its seeds that are not popular
            const uint32_t c1 = aux & BK_CSAT, c2 = (aux >> 15) & BK_CSAT;
            auto side = [&](uint32_t v, uint32_t c) -> uint32_t {
                return v == UNUSED_SIDE ? 0u : v < A.nBases ? 1u : c >= BK_CSAT ? 0xffffu : c;
            };
            const uint32_t h = side(v1, c1) + (f != rcv ? side(v2, c2) : 0u);
            weight = h <= A.maxHits ? h : 0u;
        }
        if (my >= 0) {
            uint32_t cnt = 0;
            nSeed = 1;
            nProbe = probes;
            if (found) {   // overflow list lengths (GenomeIndex.cpp:1013-1086), from the entry
                const uint32_t c1 = aux & BK_CSAT, c2 = (aux >> 15) & BK_CSAT;
                const uint32_t vf = comp ? v2 : v1, vr = comp ? v1 : v2;
                const uint32_t nf = comp ? c2 : c1, nr = comp ? c1 : c2;
                uint32_t cf = 0, cr = 0;
                if (vf >= A.nBases && vf != UNUSED_SIDE) { cf = bucket_count(A, nf, vf); nOvfRead += nf >= BK_CSAT; }
                if (f != rcv && vr >= A.nBases && vr != UNUSED_SIDE) { cr = bucket_count(A, nr, vr); nOvfRead += nr >= BK_CSAT; }
                cnt = (cf < 0xffffu ? cf : 0xffffu) | ((cr < 0xffffu ? cr : 0xffffu) << 16);
            }
            rec.meta = 0x80000000u | (uint32_t)my | (found ? 0x100u : 0u) | (comp ? 0x200u : 0u) |
                       (f == rcv ? 0x400u : 0u) | ((probes < 0x7fffu ? probes : 0x7fffu) << 16);
            rec.v1 = v1;
            rec.v2 = v2;
            rec.cnt = cnt;
        }
    }
    if (have) out[(uint64_t)r * SEEDS_PER_READ + k] = rec;
    // route the wave's long reads (lane 16j speaks for read j) onto pass 2's list, or with their
    // weight class onto the order list
    if (A.longCount) {
        const bool isLong = have && lng;
        const uint64_t ml = ballot(k == 0 && isLong);
        if (ml) {
            uint32_t w = weight;   // the read's summed weight, in every lane of its 16
#pragma unroll
            for (int s = 8; s >= 1; s >>= 1) w += (uint32_t)__shfl_xor((int)w, s, 64);
            uint32_t bl = 0;
            if (lane == 0) {
                bl = atomicAdd(A.deferCount, (uint32_t)__popcll(ml));
                atomicAdd(A.longCount, (uint32_t)__popcll(ml));
            }
            bl = (uint32_t)readlane((int)bl, 0);
            const uint32_t at = bl + (uint32_t)__popcll(ml & ((1ull << lane) - 1));
            if (k == 0 && isLong) {
                if (A.orderTmp) A.orderTmp[at] = r | (order_class(w) << ORDER_CLASS_SHIFT);
                else A.deferList[at] = r;
            }
        }
    }
    if (stats) {
        const uint32_t seeds = (uint32_t)__popcll(ballot(nSeed != 0));
        const uint32_t ovf = (uint32_t)__popcll(ballot(nOvfRead >= 1)) + (uint32_t)__popcll(ballot(nOvfRead >= 2));
        const uint32_t probes = sum_reduce32(nProbe);
        if (lane == 0) {   // 256 slot groups: no single-address atomic hot spot
            unsigned long long *st = stats + 4 * ((blockIdx.x * LOOKUP_WAVES + threadIdx.x / 64) & 255);
            atomicAdd(st + 0, (unsigned long long)seeds);
            atomicAdd(st + 1, (unsigned long long)probes);
            atomicAdd(st + 2, (unsigned long long)ovf);
        }
    }
}

}  // namespace sgk
