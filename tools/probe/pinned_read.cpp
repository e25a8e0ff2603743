// Host read rate of a 64 MB pinned staging buffer (hipHostMalloc flags) vs pageable memory,
// 1 / 4 / 16 threads: what the stream path's host tail (records copy) pays per 1M records.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>
static double run(const char *src, char *dst, size_t bytes, unsigned nt) {
    auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> th;
    for (unsigned t = 0; t < nt; t++)
        th.emplace_back([=] { size_t b = bytes * t / nt, e = bytes * (t + 1) / nt; memcpy(dst + b, src + b, e - b); });
    for (auto &x : th) x.join();
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}
int main() {
    const size_t bytes = 64ull << 20;
    std::vector<char> dst(bytes, 1), page(bytes, 2);
    void *dev;
    if (hipMalloc(&dev, bytes) != hipSuccess) return 1;
    hipMemset(dev, 3, bytes);
    struct { const char *name; unsigned flags; } kinds[] = {{"hipHostMallocDefault", hipHostMallocDefault},
        {"hipHostMallocNonCoherent", hipHostMallocNonCoherent}, {"hipHostMallocCoherent", hipHostMallocCoherent}};
    for (auto &k : kinds) {
        char *h;
        if (hipHostMalloc((void **)&h, bytes, k.flags) != hipSuccess) { printf("%s: alloc failed\n", k.name); continue; }
        for (unsigned nt : {1u, 4u, 16u}) {
            double best = 1e9;
            for (int r = 0; r < 3; r++) {
                hipMemcpy(h, dev, bytes, hipMemcpyDeviceToHost);   // fresh DMA write, as the records arrive
                double ms = run(h, dst.data(), bytes, nt);
                best = ms < best ? ms : best;
            }
            printf("%-26s threads %2u: %6.2f ms (%.1f GB/s)\n", k.name, nt, best, bytes / best / 1e6);
        }
        hipHostFree(h);
    }
    for (unsigned nt : {1u, 4u, 16u}) {
        double best = 1e9;
        for (int r = 0; r < 3; r++) { double ms = run(page.data(), dst.data(), bytes, nt); best = ms < best ? ms : best; }
        printf("%-26s threads %2u: %6.2f ms (%.1f GB/s)\n", "pageable", nt, best, bytes / best / 1e6);
    }
    // the stream path's pattern: records DMA'd into pinned staging while the host sleeps ~25 ms, then
    // copied out by 4 threads into a pageable array touched before -- every repetition timed
    {
        char *h;
        if (hipHostMalloc((void **)&h, bytes, hipHostMallocDefault) == hipSuccess) {
            printf("pinned -> pageable, 4 threads, after a 25 ms pause:");
            for (int r = 0; r < 12; r++) {
                hipMemcpy(h, dev, bytes, hipMemcpyDeviceToHost);
                std::this_thread::sleep_for(std::chrono::milliseconds(25));
                printf(" %.2f", run(h, dst.data(), bytes, 4));
            }
            printf(" ms\n");
            hipHostFree(h);
        }
    }
    return 0;
}
