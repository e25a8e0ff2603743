"""Longest-first order of the long-read lists (snap-rnaseq_amd/csrc/order_long.h).

Pass 0 (seed_lookup_kernel) weighs each read longer than 128 bases by the summed hit counts of the
first-round seeds in its first 128 bases and order_long_kernel puts pass 2's list heaviest first;
the paired aligner does the same for its long pairs (pair_weight_kernel) ahead of pass 1b.  Pass 2
also consumes pass 0's seed records for those reads.  Each read or pair is aligned by one wave on
its own arena, so the order must change no field of any record: SNAPGPU_ORDER_LONG=0 (pass 0's
atomic order) and =1 must agree bitwise, and the ordered run must agree with the CPU restatement
(BaseAligner::AlignRead, IntersectingPairedEndAligner::align) on a sample.  The workload is RNA-like: 150-base reads on a
repeat-rich genome with maxHits 16000, so the weights span many classes."""
import numpy as np
import pytest

import snapgpu
from oracle_ffi import mismatches, oracle_align, oracle_paired
from snapgpu import _ffi as F


@pytest.fixture(scope="module")
def world():
    g = snapgpu.Genome.synthetic(3_000_000, seed=41, n_contigs=3, n_repeat_families=120, repeat_fraction=0.6)
    g2 = snapgpu.Genome.synthetic(3_000_000, seed=41, n_contigs=3, n_repeat_families=120, repeat_fraction=0.6)
    idx = snapgpu.GenomeIndex.build(g, 20, 4)
    return idx, g2


def _single(idx, monkeypatch, order, reads):
    monkeypatch.setenv("SNAPGPU_ORDER_LONG", str(order))
    al = snapgpu.BaseAligner(idx, maxHitsToConsider=16000, maxK=15, maxSeedsToUse=8, extraSearchDepth=2)
    monkeypatch.delenv("SNAPGPU_ORDER_LONG")
    return al, al.AlignReads(reads)


@pytest.mark.gpu
def test_single_end_order_changes_no_record(gpu_available, world, monkeypatch):
    idx, g2 = world
    reads = snapgpu.Reads.synthetic(g2, 6000, seed=17, read_length=150, random_read_fraction=0.02)
    _, off = _single(idx, monkeypatch, 0, reads)
    al, on = _single(idx, monkeypatch, 1, reads)
    assert al.timing()["nSpilled"] == reads.n   # every read went through pass 2's list
    bad = mismatches(on, off)
    assert len(bad) == 0, f"{len(bad)} reads differ with the order on, e.g. {on[bad[0]]} vs {off[bad[0]]}"
    for f in ("nLookups", "nLocationsScored", "nElements"):
        assert np.array_equal(on[f], off[f]), f
    sub = reads.slice(0, 400)
    cpu = oracle_align(idx, sub, al.params, n_threads=8)
    bad = mismatches(on[:400], cpu)
    assert len(bad) == 0, f"{len(bad)} reads differ from the oracle, e.g. {on[bad[0]]} vs {cpu[bad[0]]}"


def _pparams():
    p = F.PairedParams()
    for k, v in dict(maxCandidatePoolSize=1000000, maxReadSize=500, forceSpacing=0, seedCoverage=0.0).items():
        setattr(p, k, v)
    p.maxHits, p.maxK, p.maxSeedsToUse, p.extraSearchDepth = 16000, 15, 8, 2
    p.minSpacing, p.maxSpacing, p.maxBigHits = 50, 1000, 16000
    return p


@pytest.mark.gpu
def test_paired_order_changes_no_record(gpu_available, world, monkeypatch):
    idx, g2 = world
    r0, r1 = snapgpu.Reads.synthetic_pairs(g2, 3000, seed=23, read_length=150, insert_mean=400, insert_sd=40)
    p = _pparams()
    kw = {f: getattr(p, f) for f in ("maxHits", "maxK", "maxSeedsToUse", "extraSearchDepth", "minSpacing",
                                      "maxSpacing", "maxBigHits", "maxCandidatePoolSize", "maxReadSize",
                                      "forceSpacing", "seedCoverage")}
    fields = ("status", "location", "direction", "score", "mapq", "nLocationsScored", "popularSeedsSkipped",
              "probabilityOfAllPairs", "probabilityOfBestPair")
    got = {}
    for order in (0, 1):
        monkeypatch.setenv("SNAPGPU_ORDER_LONG", str(order))
        pa = snapgpu.PairedAligner(idx, device=0, **kw)
        monkeypatch.delenv("SNAPGPU_ORDER_LONG")
        got[order] = pa.intersect(r0, r1)
    for f in fields:
        a, b = got[1][f], got[0][f]
        if a.dtype.kind == "f":
            a, b = a.view(np.uint64), b.view(np.uint64)
        assert np.array_equal(a, b), f
    cpu = oracle_paired(idx, r0, r1, p, chimeric=False)
    for f in fields:
        a, b = got[1][f], cpu[f]
        if a.dtype.kind == "f":
            a, b = a.view(np.uint64), b.view(np.uint64)
        nbad = int((a != b).reshape(len(a), -1).any(axis=1).sum())
        assert nbad == 0, f"{nbad} pairs differ from the oracle in {f}"
