"""GPU parity: the HIP path (through the C ABI) against the CPU restatement
(oracle/snap_oracle.c, itself pinned bit-exact against the compiled reference).

Bar: bit-exact on every output of BaseAligner::AlignRead (result, location,
direction, score, MAPQ) and on the per-read counters and the two MAPQ input
probabilities (compared as IEEE-754 bit patterns: tolerance 0).
"""
import random

import numpy as np
import pytest

import snapgpu
from oracle_ffi import mismatches, oracle_align, oracle_lv
from readsets import edge_reads

pytestmark = pytest.mark.gpu


def _report(gpu, cpu, reads, bad, k=5):
    lines = []
    for i in bad[:k]:
        b, q = reads.get(int(i))
        lines.append(f"read {i} len={len(b)} {b[:60]!r}\n  gpu={gpu[i]}\n  cpu={cpu[i]}")
    return "\n".join(lines)


# LandauVishkinTest.cpp:11-32 known answers (text, pattern, k, expected)
LV_KNOWN = [
    ("abcde", "abcde", 2, 0), ("abcde", "abcd", 2, 0), ("abcde", "abc", 2, 0), ("abcde", "ab", 2, 0),
    ("abcde", "abcdX", 2, 1), ("abcde", "abde", 2, 1), ("abcde", "bcde", 2, 1), ("abcde", "abcXde", 2, 1),
    ("abcde", "abXXe", 2, 2), ("abcde", "abcXXde", 2, 2), ("abcde", "XXXXX", 2, -1),
]


def test_lv_known_answers_gpu(gpu_available):
    res = snapgpu.lv_batch(1, [(t, p, "I" * len(p), k) for t, p, k, _ in LV_KNOWN])
    for (t, p, k, want), (e, net, prob) in zip(LV_KNOWN, res):
        assert e == want, (t, p, k, e)
        assert (e, net, prob) == oracle_lv(1, t, p, "I" * len(p), k)


def _random_lv_tasks(rng, n):
    tasks = []
    for _ in range(n):
        L = rng.choice([5, 20, 50, 80, 100, 150, 300])
        t = "".join(rng.choice("ACGT") for _ in range(L + 40))
        p = list(t[:L] if rng.random() < 0.5 else t[10:10 + L])
        for _ in range(rng.randrange(0, 12)):
            op = rng.random()
            i = rng.randrange(len(p)) if p else 0
            if op < 0.6 and p:
                p[i] = rng.choice("ACGTN")
            elif op < 0.8:
                p.insert(i, rng.choice("ACGT"))
            elif p:
                del p[i]
        p = "".join(p) or "A"
        q = "".join(chr(33 + rng.randrange(0, 45)) for _ in p)
        k = rng.choice([0, 1, 2, 4, 8, 14, 16, 20, 30])
        tl = rng.choice([len(t), len(p) + 31, max(1, len(p) - 3)])
        tasks.append((t[:tl], p, q, k))
    return tasks


@pytest.mark.parametrize("direction", [1, -1])
def test_lv_random_vs_oracle(gpu_available, direction):
    rng = random.Random(11 + direction)
    tasks = _random_lv_tasks(rng, 600)
    got = snapgpu.lv_batch(direction, tasks)
    for (t, p, q, k), g in zip(tasks, got):
        want = oracle_lv(direction, t, p, q, k)
        assert g[0] == want[0] and g[1] == want[1] and np.float64(g[2]).view(np.uint64) == np.float64(
            want[2]).view(np.uint64), (t, p, k, g, want)


def test_align_small_vs_oracle(gpu_available, small_world):
    idx, reads = small_world["index"], small_world["reads"]
    al = snapgpu.BaseAligner(idx)
    gpu = al.AlignReads(reads)
    cpu = oracle_align(idx, reads, al.params)
    bad = mismatches(gpu, cpu)
    assert len(bad) == 0, f"{len(bad)} of {len(gpu)} differ\n" + _report(gpu, cpu, reads, bad)
    # sanity: the workload is non-trivial
    assert (gpu["result"] == snapgpu.SingleHit).mean() > 0.8
    assert gpu["nLocationsScored"].sum() > len(gpu)


def test_align_edge_reads_vs_oracle(gpu_available, small_world):
    idx = small_world["index"]
    reads = snapgpu.Reads.from_list(edge_reads(small_world["genome"]))
    al = snapgpu.BaseAligner(idx)
    gpu = al.AlignReads(reads)
    cpu = oracle_align(idx, reads, al.params)
    bad = mismatches(gpu, cpu)
    assert len(bad) == 0, f"{len(bad)} of {len(gpu)} differ\n" + _report(gpu, cpu, reads, bad)


PARAM_SETS = [
    dict(maxHitsToConsider=16),
    dict(maxK=5, extraSearchDepth=1),
    dict(maxHitsToConsider=50, maxK=8, maxSeedsToUse=4, extraSearchDepth=0),
    dict(maxK=20, maxSeedsToUse=40, extraSearchDepth=5),
    dict(maxHitsToConsider=8, maxK=3, maxSeedsToUse=10, extraSearchDepth=3),
    dict(maxSeedsToUse=0, maxSeedCoverage=5.0),
    dict(explorePopularSeeds=True, maxHitsToConsider=40),
    dict(stopOnFirstHit=True),
    dict(maxK=28, extraSearchDepth=3),
    # scoreLimit falls below a partly scored element's lowestPossibleScore (BaseAligner.cpp:1129
    # tests it once per element)
    dict(maxK=2, extraSearchDepth=0),
    dict(maxK=4, extraSearchDepth=0, maxSeedsToUse=8),
]


@pytest.mark.parametrize("kw", PARAM_SETS, ids=[",".join(f"{k}={v}" for k, v in p.items()) for p in PARAM_SETS])
def test_align_params_vs_oracle(gpu_available, small_world, kw):
    idx = small_world["index"]
    reads = small_world["reads"]
    al = snapgpu.BaseAligner(idx, **kw)
    gpu = al.AlignReads(reads)
    cpu = oracle_align(idx, reads, al.params)
    bad = mismatches(gpu, cpu)
    assert len(bad) == 0, f"{kw}: {len(bad)} of {len(gpu)} differ\n" + _report(gpu, cpu, reads, bad)


def test_getters_aggregate(gpu_available, small_world):
    al = snapgpu.BaseAligner(small_world["index"])
    res = al.AlignReads(small_world["reads"])
    assert al.getNHashTableLookups() == int(res["nLookups"].sum())
    assert al.getLocationsScored() == int(res["nLocationsScored"].sum())
    assert al.getMaxK() == 14


def test_stream_submit_wait(gpu_available, small_world, monkeypatch):
    """snapgpu_align_batch_submit / _wait: batches of different sizes (several chunks, one
    read, a one-chunk batch) stream through the two lanes before one wait; every record equals
    the blocking call's, and a resident run closes an open stream first."""
    idx, reads = small_world["index"], small_world["reads"]
    monkeypatch.setenv("SNAPGPU_CHUNK_READS", "700")   # several chunks per batch, lanes alternate across batches
    al = snapgpu.BaseAligner(idx)
    want = al.AlignReads(reads)
    cuts = [(0, 2500), (2500, 1), (2501, 600), (3101, reads.n - 3101)]
    parts = [reads.slice(s, c) for s, c in cuts]
    outs = [np.zeros(p.n, dtype=snapgpu.RESULT_DTYPE) for p in parts]
    for p, o in zip(parts, outs):
        al.submit(p, o)
    al.wait()
    got = np.concatenate(outs)
    assert np.array_equal(got.view(np.uint8), want.view(np.uint8))
    t = al.timing()
    assert t["nLaunches"] == 4 + 1 + 1 + 2   # every chunk of the whole stream (700 reads a chunk)
    # submit, then a resident run without an explicit wait
    o2 = np.zeros(parts[0].n, dtype=snapgpu.RESULT_DTYPE)
    al.submit(parts[0], o2)
    dev = al.upload(parts[2])
    dev.run()
    assert np.array_equal(dev.results().view(np.uint8), want[2501:3101].view(np.uint8))
    assert np.array_equal(o2.view(np.uint8), want[:2500].view(np.uint8))
    al.wait()   # nothing left: a no-op


@pytest.mark.parametrize("kw", [dict(), dict(maxK=20, maxSeedsToUse=40, extraSearchDepth=5),
                                dict(maxHitsToConsider=16), dict(maxK=2, extraSearchDepth=0)],
                         ids=["default", "k20", "h16", "k2"])
def test_forced_radix_order_vs_oracle(gpu_available, small_world, monkeypatch, kw):
    """Forced-mode pop order from the arena-tail radix sort (score_batched / forced_sort),
    which production uses for reads with > 256 elements, forced here for every read."""
    monkeypatch.setenv("SNAPGPU_RADIX_MIN", "1")
    idx = small_world["index"]
    reads = snapgpu.Reads.from_list(edge_reads(small_world["genome"]) + [
        small_world["reads"].get(i) for i in range(3000)])
    al = snapgpu.BaseAligner(idx, **kw)
    gpu = al.AlignReads(reads)
    cpu = oracle_align(idx, reads, al.params)
    bad = mismatches(gpu, cpu)
    assert len(bad) == 0, f"{len(bad)} of {len(gpu)} differ\n" + _report(gpu, cpu, reads, bad)
    assert (gpu["nElements"] >= 8).sum() > 10   # orders of many elements were sorted


@pytest.mark.parametrize("kw", [dict(), dict(maxHitsToConsider=16000, maxK=15, maxSeedsToUse=8, extraSearchDepth=2)],
                         ids=["default", "rna"])
def test_arena_overflow_pass_vs_oracle(gpu_available, small_world, monkeypatch, kw):
    """Capped element arenas (snapgpu_aligner_create, KArgs::ovfList): a read that outgrows its
    arena in passes 1-3 is abandoned and aligned again from scratch by the big-arena pass
    (align_kernel<512> on worst-case arenas).  Forced here with a 4-element cap: every output
    still equals the oracle."""
    monkeypatch.setenv("SNAPGPU_ARENA_CAP", "4")
    idx = small_world["index"]
    reads = snapgpu.Reads.from_list(edge_reads(small_world["genome"]) + [
        small_world["reads"].get(i) for i in range(3000)])
    al = snapgpu.BaseAligner(idx, **kw)
    gpu = al.AlignReads(reads)
    t = al.timing()
    cpu = oracle_align(idx, reads, al.params)
    bad = mismatches(gpu, cpu)
    assert len(bad) == 0, f"{len(bad)} of {len(gpu)} differ\n" + _report(gpu, cpu, reads, bad)
    assert t["nArenaOverflow"] == int((gpu["nElements"] > 4).sum()) > 20   # the overflowing reads took the big pass


@pytest.mark.gpu
@pytest.mark.parametrize("kw", [dict(), dict(maxHitsToConsider=16000, maxK=15, maxSeedsToUse=8, extraSearchDepth=2)],
                         ids=["defaults", "rna_transcriptome"])
def test_align_independent_of_wave_history(gpu_available, small_world, monkeypatch, kw):
    """A read's record must not depend on the reads its persistent wave aligned before (LDS, arena or
    spill-block state left behind): the batch on one wave per CU (256 waves, ~16 reads each)
    equals the full grid's records bitwise, nProbes included, and the oracle."""
    idx = small_world["index"]
    reads = snapgpu.Reads.from_list(edge_reads(small_world["genome"]) + [
        small_world["reads"].get(i) for i in range(small_world["reads"].n)])
    full = snapgpu.BaseAligner(idx, **kw).AlignReads(reads)
    monkeypatch.setenv("SNAPGPU_WAVES_PER_CU", "1")
    al = snapgpu.BaseAligner(idx, **kw)
    few = al.AlignReads(reads)
    bad = [i for i in range(len(full)) if full[i].tobytes() != few[i].tobytes()]
    assert not bad, f"{len(bad)} of {len(full)} records differ on one wave per CU, first {bad[:5]}"
    cpu = oracle_align(idx, reads, al.params)
    bad = mismatches(few, cpu)
    assert len(bad) == 0, f"{len(bad)} of {len(few)} differ from the oracle\n" + _report(few, cpu, reads, bad)
