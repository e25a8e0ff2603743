"""N>1 orchestration of bench.py on CPU: two ranks over gloo (127.0.0.1), each
generating its own read shard against the shared deterministic genome, a barrier-
bracketed timed region and the max-over-ranks reduction.  The aligner itself needs a
GPU; the per-rank compute here is the oracle on the rank's shard, and the check is
that sharding + reduction behave as the driver's N-GPU bench expects (SURVEY 8(e):
reads shard with no data-path collective)."""
import hashlib
import os
import socket
import sys
import time

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "snap-rnaseq_amd"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import bench
    import snapgpu
    from oracle_ffi import oracle_align
    w, r, local, dist = bench.init_distributed()
    genome, reads = bench.make_workload(snapgpu, 300_000, 400, r)
    idx = snapgpu.GenomeIndex.build(genome, 20, 2)
    res = {}

    def step():
        res["out"] = oracle_align(idx, reads, snapgpu.default_params(), n_threads=1)
        time.sleep(0.05 * (r + 1))          # rank 1 is the slow one

    elapsed = bench.timed_steps(step, 2, dist, lambda: None)
    gdig = hashlib.sha256(snapgpu.Genome.synthetic(300_000, seed=2121, n_contigs=1,
                                                   n_repeat_families=200).bases(0, 300_000)).hexdigest()
    rdig = hashlib.sha256(bytes(reads.get(0)[0]) + bytes(reads.get(399)[0])).hexdigest()
    single = int((res["out"]["result"] == snapgpu.SingleHit).sum())
    dist.destroy_process_group()
    q.put((r, w, elapsed, gdig, rdig, single))


def test_two_rank_sharding_and_max_reduction():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    import queue
    got, t0 = [], time.time()
    while len(got) < len(procs) and time.time() - t0 < 300:
        try:
            got.append(q.get(timeout=2))
        except queue.Empty:
            assert all(p.exitcode in (None, 0) for p in procs), [p.exitcode for p in procs]
    out = sorted(got)
    assert len(out) == 2
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, w0, e0, g0, d0, s0), (r1, w1, e1, g1, d1, s1) = out
    assert (r0, r1, w0, w1) == (0, 1, 2, 2)
    assert e0 == e1 >= 2 * 0.1                 # every rank reports the slowest rank's time
    assert g0 == g1                            # replicated genome/index
    assert d0 != d1                            # disjoint read shards
    assert s0 > 300 and s1 > 300               # each shard aligns (oracle stand-in for the GPU)
