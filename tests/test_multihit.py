"""Windowed search + multi-hit export: the richer
BaseAligner::AlignRead (BaseAligner.h:73-86; window BaseAligner.cpp:596-602,
749-751, 781-786, 849-853; windowed GenomeIndex::fillInLookedUpResults
GenomeIndex.cpp:1013-1086; recording :1255-1261; fillHitsFound :940-975).

Golden fixtures: tests/golden/expected_small_mh*.tsv, written by the reference's
own BaseAligner (oracle/ref_harness.cpp mode alignx) for the per-read windows in
tests/golden/small_search.tsv.
"""
import os

import numpy as np
import pytest

import snapgpu
from golden_common import MULTIHIT_RUNS, PARAM_SETS, params_to_aligner_kwargs
from oracle_ffi import canonical_tsv_ex, oracle_align, oracle_align_ex, mismatches

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def small_index():
    return snapgpu.GenomeIndex.build(snapgpu.Genome.from_fasta(os.path.join(G, "small.fa"), 500), 20, 4)


@pytest.fixture(scope="module")
def small_reads():
    return snapgpu.Reads.from_fastq(os.path.join(G, "small_reads.fq"))


@pytest.fixture(scope="module")
def small_search():
    return np.loadtxt(os.path.join(G, "small_search.tsv"), dtype=np.uint64).reshape(-1, 3)


def _params(pset):
    p = snapgpu.default_params()
    for k, v in params_to_aligner_kwargs(PARAM_SETS[pset]).items():
        setattr(p, k, v)
    return p


def _first_diff(got, want):
    for i, (a, b) in enumerate(zip(got.splitlines(), want.splitlines())):
        if a != b:
            return f"line {i}:\n got  {a}\n want {b}"
    return None


@pytest.mark.parametrize("name", sorted(MULTIHIT_RUNS))
def test_oracle_multihit_matches_reference(small_index, small_reads, small_search, name):
    maxget, pset = MULTIHIT_RUNS[name]
    res, found, hits = oracle_align_ex(small_index, small_reads, _params(pset), small_search, maxget, n_threads=4)
    got = canonical_tsv_ex(res, found, hits)
    want = open(os.path.join(G, f"expected_small_{name}.tsv")).read()
    assert got == want, _first_diff(got, want)


def test_oracle_ex_unconstrained_equals_plain(small_index, small_reads):
    p = _params("default")
    plain = oracle_align(small_index, small_reads, p, n_threads=4)
    res, found, hits = oracle_align_ex(small_index, small_reads, p, None, 0, n_threads=4)
    assert len(mismatches(plain, res)) == 0


def test_search_array_validation():
    s = snapgpu.search_array([(5, 100, 1), (0, 0, 0)], 2)
    assert s.dtype == snapgpu.SEARCH_DTYPE and list(s["searchRadius"]) == [5, 0]
    with pytest.raises(ValueError):
        snapgpu.search_array([(5, 100, 1)], 2)
    assert snapgpu.search_array(None, 3) is None


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(MULTIHIT_RUNS))
def test_gpu_multihit_matches_reference(small_index, small_reads, small_search, name):
    maxget, pset = MULTIHIT_RUNS[name]
    al = snapgpu.BaseAligner(small_index, **params_to_aligner_kwargs(PARAM_SETS[pset]))
    res, found, hits = al.AlignReadsEx(small_reads, small_search, maxget)
    got = canonical_tsv_ex(res, found, hits)
    want = open(os.path.join(G, f"expected_small_{name}.tsv")).read()
    assert got == want, _first_diff(got, want)


@pytest.mark.gpu
def test_gpu_multihit_c1_matches_oracle():
    """C1-sized genome, 20k reads (incl. >128-base and IUPAC reads on the byte path),
    windows around the true origin and elsewhere, 32 hits per read."""
    from golden_common import C1
    from readsets import edge_reads
    g = snapgpu.Genome.synthetic(**C1["genome"])
    syn = snapgpu.Reads.synthetic(g, 20000, seed=5, read_length=100)
    tloc, tdir = syn.truth()
    edge = edge_reads(g, n_random=300, seed=4)
    reads = snapgpu.Reads.from_list(edge + [tuple(x.decode() for x in syn.get(i)) for i in range(syn.n)])
    nb = g.n_bases
    idx = snapgpu.GenomeIndex.build(g, 20, 8)   # takes ownership of g
    rng = np.random.default_rng(3)
    n = reads.n
    ne = len(edge)
    loc = np.concatenate([rng.integers(0, nb, ne), np.asarray(tloc, dtype=np.int64)])
    dr = np.concatenate([rng.integers(0, 2, ne), np.asarray(tdir, dtype=np.int64)])
    kind = rng.integers(0, 5, n)
    s = np.zeros((n, 3), dtype=np.uint64)
    s[:, 0] = np.where(kind == 0, 0, rng.choice([16, 300, 20000], n))
    s[:, 1] = np.where(kind == 3, rng.integers(0, nb, n), np.maximum(loc + rng.integers(-50, 50, n), 0))
    s[:, 2] = np.where(kind == 4, 1 - dr, dr)
    p = _params("default")
    want = oracle_align_ex(idx, reads, p, s, 32)
    al = snapgpu.BaseAligner(idx, **params_to_aligner_kwargs(PARAM_SETS["default"]))
    got = al.AlignReadsEx(reads, s, 32)
    bad = mismatches(got[0], want[0])
    assert len(bad) == 0, f"{len(bad)} result mismatches, first {bad[:5]}"
    assert np.array_equal(got[1], want[1])
    for i in np.nonzero(want[1] > 0)[0]:
        f = want[1][i]
        assert np.array_equal(got[2][i, :f], want[2][i, :f]), i


@pytest.mark.gpu
def test_gpu_ex_rejects_bad_arguments(small_index, small_reads):
    al = snapgpu.BaseAligner(small_index)
    with pytest.raises(snapgpu.SnapGpuError):
        al.AlignReadsEx(small_reads, None, 1025)
    s = np.zeros((small_reads.n, 3), dtype=np.uint64)
    s[:, 0] = 10
    s[:, 2] = 2
    with pytest.raises(snapgpu.SnapGpuError):
        al.AlignReadsEx(small_reads, s, 0)


# maxHitsToGet 1000 (PairedAligner.cpp:584) with > 512 hits per distance: the reference's rows
# hitLocations[MAX_K][512] alias (BaseAligner.h:148-151); fixture from ref_harness alignx on
# tests/golden/repeat.fa (make_golden.py --only-mh1000), paired CLI aligner parameters
REPEAT_KW = dict(maxHitsToConsider=16000, maxK=15, maxSeedsToUse=8, extraSearchDepth=2)


@pytest.fixture(scope="module")
def repeat_index():
    return snapgpu.GenomeIndex.build(snapgpu.Genome.from_fasta(os.path.join(G, "repeat.fa"), 500), 20, 4)


def test_oracle_mh1000_aliasing_matches_reference(repeat_index):
    reads = snapgpu.Reads.from_fastq(os.path.join(G, "repeat_reads.fq"))
    p = snapgpu.default_params()
    for k, v in REPEAT_KW.items():
        setattr(p, k, v)
    res, found, hits = oracle_align_ex(repeat_index, reads, p, None, 1000, n_threads=4)
    got = canonical_tsv_ex(res, found, hits)
    want = open(os.path.join(G, "expected_repeat_mh1000.tsv")).read()
    assert got == want, _first_diff(got, want)
    assert (found == 1000).sum() >= 20


@pytest.mark.gpu
def test_gpu_mh1000_aliasing_matches_reference(repeat_index):
    reads = snapgpu.Reads.from_fastq(os.path.join(G, "repeat_reads.fq"))
    al = snapgpu.BaseAligner(repeat_index, **REPEAT_KW)
    res, found, hits = al.AlignReadsEx(reads, None, 1000)
    got = canonical_tsv_ex(res, found, hits)
    want = open(os.path.join(G, "expected_repeat_mh1000.tsv")).read()
    assert got == want, _first_diff(got, want)


@pytest.mark.gpu
def test_gpu_mh1000_arena_overflow_matches_reference(repeat_index, monkeypatch):
    """The multi-hit path (align_kernel<*, true>) through the big-arena pass: with 256-element
    arenas in passes 1-3 the repeat reads outgrow them, are aligned again on worst-case arenas,
    and the hits still equal the reference's."""
    monkeypatch.setenv("SNAPGPU_ARENA_CAP", "256")
    reads = snapgpu.Reads.from_fastq(os.path.join(G, "repeat_reads.fq"))
    al = snapgpu.BaseAligner(repeat_index, **REPEAT_KW)
    res, found, hits = al.AlignReadsEx(reads, None, 1000)
    assert al.timing()["nArenaOverflow"] > 0
    got = canonical_tsv_ex(res, found, hits)
    want = open(os.path.join(G, "expected_repeat_mh1000.tsv")).read()
    assert got == want, _first_diff(got, want)
