// threads.cpp -- the host thread budget of one rank.
//
// The reference sizes its worker pool from the command line (`-t`, default the machine's cores,
// AlignerOptions.cpp / ParallelTask.h:104-161).  Here the host stages (record writers, the RNA
// filter, the stream path's host tail, the index builder) size themselves from what this process
// may actually run on: the affinity mask, capped by the cgroup CPU quota (a GPU box shows every
// core of the host but gives the job a quota of 16), divided among the ranks of the node
// (LOCAL_WORLD_SIZE, set by torch.distributed.run), so that N ranks together stay inside the
// quota.  std::thread::hardware_concurrency() sees none of that (256 on the bench box).
#include "internal.h"

#include <sched.h>
#include <unistd.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <fstream>
#include <string>

namespace snapgpu {
namespace {

// CPUs granted by the cgroup quota, or 0 when there is none.  cgroup v2: cpu.max "<quota> <period>"
// or "max <period>"; v1: cpu.cfs_quota_us (-1 = none) / cpu.cfs_period_us.
unsigned cgroupQuotaCpus() {
    {
        std::ifstream f("/sys/fs/cgroup/cpu.max");
        std::string q, p;
        if (f >> q >> p) {
            if (q == "max") return 0;
            const double per = atof(p.c_str());
            return per > 0 ? (unsigned)std::max(1.0, std::ceil(atof(q.c_str()) / per)) : 0;
        }
    }
    std::ifstream fq("/sys/fs/cgroup/cpu/cpu.cfs_quota_us"), fp("/sys/fs/cgroup/cpu/cpu.cfs_period_us");
    long long q = -1, p = 0;
    if ((fq >> q) && (fp >> p) && q > 0 && p > 0) return (unsigned)std::max(1.0, std::ceil((double)q / (double)p));
    return 0;
}

unsigned affinityCpus() {
    cpu_set_t set;
    CPU_ZERO(&set);
    if (sched_getaffinity(0, sizeof(set), &set) == 0) {
        const int n = CPU_COUNT(&set);
        if (n > 0) return (unsigned)n;
    }
    const long n = sysconf(_SC_NPROCESSORS_ONLN);
    return n > 0 ? (unsigned)n : 1u;
}

unsigned envPositive(const char *name) {
    const char *v = getenv(name);
    if (!v || !*v) return 0;
    const long x = strtol(v, nullptr, 10);
    return x > 0 ? (unsigned)std::min(x, 1024L) : 0u;
}

}  // namespace

unsigned hostThreadBudget() {
    static const unsigned budget = [] {
        if (unsigned o = envPositive("SNAPGPU_HOST_THREADS")) return std::min(o, 256u);
        unsigned usable = affinityCpus();
        if (unsigned q = cgroupQuotaCpus()) usable = std::min(usable, q);
        const unsigned ranks = std::max(1u, envPositive("LOCAL_WORLD_SIZE"));
        return std::max(1u, usable / ranks);
    }();
    return budget;
}

unsigned hostThreads(unsigned cap) { return std::max(1u, std::min(cap ? cap : 1u, hostThreadBudget())); }

}  // namespace snapgpu

extern "C" int snapgpu_host_threads(void) { return (int)snapgpu::hostThreadBudget(); }
