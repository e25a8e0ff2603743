"""N>1 orchestration of bench.py on CPU: two ranks over gloo (127.0.0.1).  Rank 0 builds the
index once and shares it through /dev/shm; rank 1 maps it (no second build); each rank
generates its own read shard; the timed region is barrier-bracketed and reports the max over
ranks.  The aligner itself needs a GPU; the per-rank compute here is the oracle on the rank's
shard, and the checks are that index sharing, sharding and the reduction behave as the
driver's N-GPU bench expects (reads shard with no data-path collective)."""
import hashlib
import os
import socket
import sys
import time

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
    from snapgpu import shared_index
    from oracle_ffi import oracle_align
    w, r, local, dist = bench.init_distributed()
    gen = dict(seed=2121, n_contigs=2, n_repeat_families=40)
    idx, info = shared_index.build_once(snapgpu, 300_000, gen, 20, 2, r, w, dist)
    reads = snapgpu.Reads.synthetic(idx.genome_handle(), 400, seed=99 + r)
    res = {}

    def step():
        res["out"] = oracle_align(idx, reads, snapgpu.default_params(), n_threads=1)
        time.sleep(0.05 * (r + 1))          # rank 1 is the slow one

    elapsed = bench.timed_steps(step, 2, dist, lambda: None)
    ii = idx.info()
    v = idx.view()
    import ctypes as C
    gdig = hashlib.sha256(C.string_at(v.slots, 12 * ii["totalHashSlots"]) +
                          C.string_at(v.genome, ii["nBases"])).hexdigest()
    rdig = hashlib.sha256(bytes(reads.get(0)[0]) + bytes(reads.get(399)[0])).hexdigest()
    single = int((res["out"]["result"] == snapgpu.SingleHit).sum())
    path = info["shared_file"]
    dist.barrier()
    shared_index.cleanup(r, w)
    dist.barrier()
    gone = not os.path.exists(path)
    dist.destroy_process_group()
    q.put((r, w, elapsed, gdig, rdig, single, info["built_by_this_rank"], gone))


def test_two_rank_index_built_once_sharding_and_max_reduction():
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
    (r0, w0, e0, g0, d0, s0, b0, x0), (r1, w1, e1, g1, d1, s1, b1, x1) = out
    assert (r0, r1, w0, w1) == (0, 1, 2, 2)
    assert e0 == e1 >= 2 * 0.1                 # every rank reports the slowest rank's time
    assert (b0, b1) == (True, False)           # the index is built exactly once (rank 0)
    assert g0 == g1                            # rank 1 maps the very same tables and genome
    assert x0 and x1                           # the shared file is removed at the end
    assert d0 != d1                            # disjoint read shards
    assert s0 > 300 and s1 > 300               # each shard aligns (oracle stand-in for the GPU)


def _bench_env():
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_PORT", "MASTER_ADDR")}
    env["OMP_NUM_THREADS"] = "1"
    return env


def test_bench_gpus_2_self_launches_two_ranks():
    """`python bench.py --gpus 2` with no launcher around it starts two ranks itself
    (torch.distributed.run, 127.0.0.1) and relays rank 0's line: n_gpus 2, the index built once
    (the other rank attached it), disjoint shards, both ranks' own figures."""
    import json
    import subprocess
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--oracle-standin", "--reads", "300",
           "--genome-bases", "300000", "--steps", "2", "--warmup", "0"]
    r = subprocess.run(cmd, capture_output=True, text=True, env=_bench_env(), timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and "standin" in d
    pr = d["config"]["per_rank"]
    assert sorted(p["rank"] for p in pr) == [0, 1]
    assert sum(p["index_built_here"] for p in pr) == 1
    assert pr[0]["shard_first_read"] != pr[1]["shard_first_read"]
    assert all(p["single_hits"] > 200 for p in pr)
    assert d["value"] == pytest.approx(2 * 300 * 2 / (d["ms_per_step"] * 2 / 1000.0), rel=1e-6)
    assert d["ms_per_step"] * 2 / 1000.0 >= max(p["elapsed_s"] for p in pr) - 1e-3


def test_bench_gpus_8_rehearsal_one_image_per_node():
    """The driver's 8-GPU scaling run, rehearsed on CPU through the real self-launch (verdict r4 item 6):
    `bench.py --gpus 8` starts 8 ranks, one builds the index, every rank -- the builder included -- maps
    the one shared /dev/shm image (host RAM holds one copy: C3's 56 GB once, not per rank), the 8 read
    shards are disjoint, the reduction covers all ranks, and the image is removed at the end."""
    import json
    import subprocess
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--oracle-standin", "--reads", "120",
           "--genome-bases", "200000", "--steps", "1", "--warmup", "0"]
    r = subprocess.run(cmd, capture_output=True, text=True, env=_bench_env(), timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 8 and "standin" in d
    pr = d["config"]["per_rank"]
    assert sorted(p["rank"] for p in pr) == list(range(8))
    assert sum(p["index_built_here"] for p in pr) == 1
    assert all(p["index_attached"] for p in pr)
    files = {p["shared_file"] for p in pr}
    assert len(files) == 1 and not os.path.exists(files.pop())
    assert len({p["shard_first_read"] for p in pr}) == 8
    assert all(p["single_hits"] > 50 for p in pr)
    assert d["ms_per_step"] / 1000.0 >= max(p["elapsed_s"] for p in pr) - 1e-3
    assert d["value"] == pytest.approx(8 * 120 / (d["ms_per_step"] / 1000.0), rel=1e-6)


def test_bench_refuses_world_gpus_mismatch():
    """A run whose rank count differs from --gpus exits non-zero instead of mislabelling n_gpus."""
    import subprocess
    env = dict(_bench_env(), WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--oracle-standin",
                        "--reads", "10", "--genome-bases", "100000"], capture_output=True, text=True, env=env,
                       timeout=300)
    assert r.returncode == 2 and "refusing" in r.stderr


def test_shared_index_roundtrip(tmp_path):
    """snapgpu_index_share / snapgpu_index_attach: identical info, tables, genome and lookups."""
    import ctypes as C
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "snap-rnaseq_amd"))
    import snapgpu
    g = snapgpu.Genome.synthetic(200_000, seed=5, n_contigs=3, n_repeat_families=20)
    idx = snapgpu.GenomeIndex.build(g, 20, 2)
    idx.share(tmp_path / "idx.bin")
    at = snapgpu.GenomeIndex.attach(tmp_path / "idx.bin")
    i1, i2 = idx.info(), at.info()
    assert i1 == i2
    v1, v2 = idx.view(), at.view()
    assert C.string_at(v1.slots, 12 * i1["totalHashSlots"]) == C.string_at(v2.slots, 12 * i2["totalHashSlots"])
    assert C.string_at(v1.overflow, 4 * i1["overflowTableSize"]) == C.string_at(v2.overflow, 4 * i2["overflowTableSize"])
    assert C.string_at(v1.genome - 256, i1["nBases"] + 512) == C.string_at(v2.genome - 256, i2["nBases"] + 512)
    gen1 = snapgpu.Genome(idx.genome_handle())
    gen2 = snapgpu.Genome(at.genome_handle())
    try:
        assert [p for p in gen1.pieces] == [p for p in gen2.pieces]
    finally:
        gen1._h = gen2._h = None   # borrowed handles: the indexes own the genomes
    rng = np.random.default_rng(1)
    for p in rng.integers(1000, i1["nBases"] - 1000, 200):
        s = idx.genome_bases(int(p), 20).decode()
        if set(s) <= set("ACGT"):
            assert idx.lookupSeed(s) == at.lookupSeed(s)
    with pytest.raises(snapgpu.SnapGpuError):
        (tmp_path / "bad.bin").write_bytes(b"x" * 8192)
        snapgpu.GenomeIndex.attach(tmp_path / "bad.bin")
