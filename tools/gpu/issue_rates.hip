// issue_rates.hip -- scalar vs vector issue capacity of a gfx950 CU (verdict r4 item 3).
//
// align_kernel<128> issues ~14.3k VALU, ~9.1k SALU and ~2.0k branch instructions per read.  Is the
// scalar side a per-CU resource (one scalar unit shared by the 4 SIMDs, as on GCN) or per SIMD, and
// does SALU issue overlap VALU issue of other waves?  Each kernel runs a long unrolled stream over 8
// independent registers (no dependency stalls) on `w` waves per CU (one block of w waves per CU),
// and reports shader cycles (s_memtime) per instruction per CU = cycles / (instructions per wave * w).
//
//   SALU   16 x s_add_u32 over 8 SGPRs
//   VALU   16 x v_add_u32 over 8 VGPRs
//   MIX    8 x s_add_u32 + 8 x v_add_u32 interleaved (one wave's stream): both pipes from one wave
//   SBR    16 x (s_cmp_eq_u32 + s_cbranch_scc1 to the next instruction, never taken)
//   RLCH   a dependent VALU -> SGPR -> VALU chain (v_readlane_b32, s_add_u32, v_add_u32 with the SGPR):
//          the aligner's uniform-value idiom, latency per link
//
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/issue_rates tools/gpu/issue_rates.hip && /tmp/issue_rates
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

constexpr int ITERS = 2048;
enum Kind { SALU, VALU, MIX, SBR, RLCH, NKIND };
static const char *kName[NKIND] = {"s_add_u32", "v_add_u32", "8 x s_add_u32 + 8 x v_add_u32 interleaved (one stream)",
                                   "s_cmp_eq_u32 + s_cbranch_scc1 (not taken)",
                                   "dependent v_readlane_b32 -> s_add_u32 -> v_add_u32 (per link)"};
static const int kPerIter[NKIND] = {16, 16, 16, 32, 3 * 8};

#define SA(i) "s_add_u32 %" #i ", %" #i ", %8\n"
#define VA(i) "v_add_u32 %" #i ", %" #i ", %8\n"

template <int KIND>
__global__ __launch_bounds__(1024) void rate_kernel(uint32_t seed, uint64_t *cyc, uint32_t *sink) {
    const uint32_t t = threadIdx.x + seed;
    uint32_t r0 = t, r1 = t ^ 1, r2 = t ^ 2, r3 = t ^ 3, r4 = t ^ 4, r5 = t ^ 5, r6 = t ^ 6, r7 = t ^ 7;
    uint32_t s0 = seed, s1 = seed + 1, s2 = seed + 2, s3 = seed + 3, s4 = seed + 4, s5 = seed + 5, s6 = seed + 6,
             s7 = seed + 7;
    const uint32_t k = (seed & 7) + 1;
    __syncthreads();
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
    for (int it = 0; it < ITERS; it++) {
        if constexpr (KIND == SALU) {
            asm volatile(SA(0) SA(1) SA(2) SA(3) SA(4) SA(5) SA(6) SA(7) SA(0) SA(1) SA(2) SA(3) SA(4) SA(5) SA(6) SA(7)
                         : "+s"(s0), "+s"(s1), "+s"(s2), "+s"(s3), "+s"(s4), "+s"(s5), "+s"(s6), "+s"(s7)
                         : "s"(k) : "scc");
        } else if constexpr (KIND == VALU) {
            asm volatile(VA(0) VA(1) VA(2) VA(3) VA(4) VA(5) VA(6) VA(7) VA(0) VA(1) VA(2) VA(3) VA(4) VA(5) VA(6) VA(7)
                         : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6), "+v"(r7)
                         : "s"(k));
        } else if constexpr (KIND == MIX) {
            asm volatile("s_add_u32 %0, %0, %16\n v_add_u32 %8, %8, %16\n s_add_u32 %1, %1, %16\n v_add_u32 %9, %9, %16\n"
                         "s_add_u32 %2, %2, %16\n v_add_u32 %10, %10, %16\n s_add_u32 %3, %3, %16\n v_add_u32 %11, %11, %16\n"
                         "s_add_u32 %4, %4, %16\n v_add_u32 %12, %12, %16\n s_add_u32 %5, %5, %16\n v_add_u32 %13, %13, %16\n"
                         "s_add_u32 %6, %6, %16\n v_add_u32 %14, %14, %16\n s_add_u32 %7, %7, %16\n v_add_u32 %15, %15, %16\n"
                         : "+s"(s0), "+s"(s1), "+s"(s2), "+s"(s3), "+s"(s4), "+s"(s5), "+s"(s6), "+s"(s7),
                           "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6), "+v"(r7)
                         : "s"(k) : "scc");
        } else if constexpr (KIND == SBR) {
#define BR(i) "s_cmp_eq_u32 %" #i ", 0xdeadbeef\n s_cbranch_scc1 1f\n1:\n"
            asm volatile(BR(0) BR(1) BR(2) BR(3) BR(4) BR(5) BR(6) BR(7) BR(0) BR(1) BR(2) BR(3) BR(4) BR(5) BR(6) BR(7)
                         : "+s"(s0), "+s"(s1), "+s"(s2), "+s"(s3), "+s"(s4), "+s"(s5), "+s"(s6), "+s"(s7)
                         :: "scc");
#undef BR
        } else {
#define LK "v_readlane_b32 %1, %0, 0\n s_add_u32 %1, %1, %2\n v_add_u32 %0, %0, %1\n"
            asm volatile(LK LK LK LK LK LK LK LK : "+v"(r0), "+s"(s0) : "s"(k) : "scc");
#undef LK
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
    const uint32_t x = r0 ^ r1 ^ r2 ^ r3 ^ r4 ^ r5 ^ r6 ^ r7 ^ s0 ^ s1 ^ s2 ^ s3 ^ s4 ^ s5 ^ s6 ^ s7;
    if (x == 0x12345678u) sink[0] = x;
}

template <int KIND>
static int run(int ncu, int wpc, double &cpi_wave, double &cpi_cu) {
    uint64_t *dc;
    uint32_t *ds;
    CHK(hipMalloc(&dc, sizeof(uint64_t) * ncu * wpc));
    CHK(hipMalloc(&ds, 4));
    // at most 16 waves (1024 lanes) per block: more waves per CU come as 2 blocks per CU
    const int bpc = wpc > 16 ? 2 : 1, wpb = wpc / bpc;
    hipLaunchKernelGGL(rate_kernel<KIND>, dim3(ncu * bpc), dim3(64 * wpb), 0, 0, 1u, dc, ds);   // warm
    CHK(hipGetLastError());
    CHK(hipDeviceSynchronize());
    hipLaunchKernelGGL(rate_kernel<KIND>, dim3(ncu * bpc), dim3(64 * wpb), 0, 0, 2u, dc, ds);
    CHK(hipGetLastError());
    CHK(hipDeviceSynchronize());
    std::vector<uint64_t> c(ncu * wpc);
    CHK(hipMemcpy(c.data(), dc, c.size() * 8, hipMemcpyDeviceToHost));
    double avg = 0;
    for (auto v : c) avg += (double)v;
    avg /= (double)c.size();
    const double instr = (double)ITERS * kPerIter[KIND];
    cpi_wave = avg / instr;
    cpi_cu = avg / (instr * wpc);
    (void)hipFree(dc);
    (void)hipFree(ds);
    return 0;
}

template <int KIND>
static int row(int ncu) {
    printf("  {\"instruction\": \"%s\"", kName[KIND]);
    for (int w : {1, 2, 4, 8, 16, 20, 32}) {
        double cw, cc;
        if (run<KIND>(ncu, w, cw, cc)) return 1;
        printf(", \"wpc%d\": {\"cycles_per_instr_per_wave\": %.3f, \"cycles_per_instr_per_cu\": %.3f}", w, cw, cc);
    }
    printf("}%s\n", KIND + 1 < NKIND ? "," : "");
    return 0;
}

int main() {
    hipDeviceProp_t p;
    CHK(hipGetDeviceProperties(&p, 0));
    const int ncu = p.multiProcessorCount;
    printf("{\"device\": \"%s\", \"cus\": %d, \"note\": \"shader cycles (s_memtime) per instruction; wpcN = N waves per "
           "CU (one block, two above 16; N/4 per SIMD from 4 up)\", \"rates\": [\n", p.gcnArchName, ncu);
    if (row<SALU>(ncu) || row<VALU>(ncu) || row<MIX>(ncu) || row<SBR>(ncu) || row<RLCH>(ncu)) return 1;
    printf("]}\n");
    return 0;
}
