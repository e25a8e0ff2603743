"""Host thread budget (snapgpu_host_threads, csrc/host/threads.cpp): every host stage of the
library -- record writers, the RNA filter, the stream path's host tail, the index builder -- sizes
its threads from it, so N ranks of one node together stay inside the job's CPU share (the GPU box
shows every core of the host, 256, but grants a quota of 16; std::thread::hardware_concurrency
sees only the 256).  The reference takes its thread count from `-t` (ParallelTask.h:104-161)."""
import math
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _usable_cpus():
    """The same rule, restated: affinity mask capped by the cgroup v2 / v1 quota."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = math.ceil(int(q) / int(per))
    except (OSError, ValueError):
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0 and per > 0:
                quota = math.ceil(q / per)
        except (OSError, ValueError):
            pass
    return max(1, min(aff, quota) if quota else aff)


def _budget(**env):
    e = {k: v for k, v in os.environ.items() if k not in ("SNAPGPU_HOST_THREADS", "LOCAL_WORLD_SIZE")}
    e.update({k: str(v) for k, v in env.items()})
    code = ("import sys; sys.path.insert(0, %r); import snapgpu; print(snapgpu.host_threads())"
            % os.path.join(ROOT, "snap-rnaseq_amd"))
    out = subprocess.run([sys.executable, "-c", code], env=e, capture_output=True, text=True, check=True)
    return int(out.stdout.strip())


def test_budget_is_the_usable_cpus_of_one_rank():
    assert _budget() == _usable_cpus()


def test_eight_rank_budgets_fit_the_quota():
    """8 rehearsal ranks of one node (LOCAL_WORLD_SIZE=8, as torch.distributed.run sets it): their
    budgets sum to at most the usable CPUs, and each has at least one thread."""
    usable = _usable_cpus()
    budgets = [_budget(LOCAL_WORLD_SIZE=8, LOCAL_RANK=r) for r in range(8)]
    assert all(b >= 1 for b in budgets)
    assert sum(budgets) <= max(usable, 8), (budgets, usable)
    assert _budget(LOCAL_WORLD_SIZE=2) == max(1, usable // 2)


def test_override_beyond_sixteen_is_honoured_and_bounded():
    """SNAPGPU_HOST_THREADS replaces the budget (per-thread arrays of the RNA stages
    are sized by the stage's worker count, which caps at 16, never by a constant)."""
    assert _budget(SNAPGPU_HOST_THREADS=40) == 40
    assert _budget(SNAPGPU_HOST_THREADS=100000) == 256
    assert _budget(SNAPGPU_HOST_THREADS="junk") == _usable_cpus()
