"""Reads of 129..256 bases: align_kernel<256> (pass 2, bit-plane LV on 256-bit masks).

Fixtures (tests/golden/make_golden.py --only-long, from the reference built in oracle/_ref):
* small_long_reads.fq -- synthetic 150 / 250 / 129 / 256 bp reads and mixed lengths 129..256
  (some lower-case, some N bases) on tests/golden/small.fa, with the reference's AlignRead
  outputs for three parameter sets (expected_small_long_{default,k20,s4}.tsv);
* lv_long_{fwd,rev}.tsv -- LandauVishkin<+-1> calls with patterns of 128..253 bases.
CPU tests pin the oracle to them; GPU tests run the product path (every read goes through
pass 2, none reaches the byte-compare pass 3) and the 256-bit lv_group unit kernel."""
import os

import numpy as np
import pytest

import snapgpu
from golden_common import PARAM_SETS, params_to_aligner_kwargs
from oracle_ffi import canonical_tsv, oracle_align, oracle_lv

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
SETS = ("default", "k20", "s4")


@pytest.fixture(scope="module")
def small_index():
    return snapgpu.GenomeIndex.build(snapgpu.Genome.from_fasta(os.path.join(G, "small.fa"), 500), 20, 4)


@pytest.fixture(scope="module")
def long_reads():
    return snapgpu.Reads.from_fastq(os.path.join(G, "small_long_reads.fq"))


def _params(name):
    p = snapgpu.default_params()
    for k, v in params_to_aligner_kwargs(PARAM_SETS[name]).items():
        setattr(p, k, v)
    return p


def _diff(got, want):
    g, w = got.splitlines(), want.splitlines()
    assert len(g) == len(w)
    return [(a, b) for a, b in zip(g, w) if a != b]


def _lv_rows(fn):
    return [line.rstrip("\n").split("\t") for line in open(os.path.join(G, fn))]


def test_long_fixture_shape(long_reads):
    L = long_reads.lengths()
    assert L.min() == 129 and L.max() == 256 and (L == 150).sum() >= 1200 and (L == 250).sum() >= 600


@pytest.mark.parametrize("name", SETS)
def test_oracle_matches_reference_long_reads(small_index, long_reads, name):
    res = oracle_align(small_index, long_reads, _params(name), n_threads=4)
    bad = _diff(canonical_tsv(res), open(os.path.join(G, f"expected_small_long_{name}.tsv")).read())
    assert not bad, f"{len(bad)} differ, first: {bad[:3]}"


@pytest.mark.parametrize("direction,fn", [(1, "lv_long_fwd.tsv"), (-1, "lv_long_rev.tsv")])
def test_oracle_lv_matches_reference_long_patterns(direction, fn):
    rows = _lv_rows(fn)
    assert max(len(r[3]) for r in rows) >= 250
    for d, k, t, p, q, e, net, prob in rows:
        ge, gn, gp = oracle_lv(direction, t, p, q, int(k))
        assert ge == int(e), (p, k)
        if ge >= 0:
            if direction < 0:
                assert gn == int(net), (p, k)
            assert np.float64(gp).view(np.uint64) == np.float64(float.fromhex(prob)).view(np.uint64)


# ------------------------------------------------------------------------- GPU
@pytest.mark.gpu
@pytest.mark.parametrize("name", SETS)
def test_gpu_long_reads_match_reference(gpu_available, small_index, long_reads, name):
    al = snapgpu.BaseAligner(small_index, **params_to_aligner_kwargs(PARAM_SETS[name]))
    res = al.AlignReads(long_reads)
    t = al.timing()
    # every read leaves pass 1; pass 2 (align_kernel<256>) keeps all but the reads holding IUPAC
    # codes (sampled from the genome's IUPAC bytes), which the byte-compare pass 3 takes
    iupac = sum(1 for i in range(long_reads.n) if set(long_reads.get(i)[0].upper()) - set(b"ACGTN"))
    assert 0 < iupac < 100
    assert t["nSpilled"] == long_reads.n and t["nByteReads"] == iupac, t
    assert ((res["flags"] & snapgpu.FLAG_DEFERRED) != 0).all()
    assert int(((res["flags"] & snapgpu.FLAG_BYTE_PATH) != 0).sum()) == iupac
    bad = _diff(canonical_tsv(res), open(os.path.join(G, f"expected_small_long_{name}.tsv")).read())
    assert not bad, f"{len(bad)} differ, first: {bad[:3]}"
    cpu = oracle_align(small_index, long_reads, al.params, n_threads=4)   # counters too
    for f in ("nLookups", "nLocationsScored", "nHitWords", "nElements"):   # nProbes: bucket lines, device-only
        assert np.array_equal(res[f], cpu[f]), f


@pytest.mark.gpu
@pytest.mark.parametrize("direction,fn", [(1, "lv_long_fwd.tsv"), (-1, "lv_long_rev.tsv")])
def test_gpu_bitplane_lv256_matches_reference(gpu_available, direction, fn):
    """lv_group on 256-bit masks (a batch holding a pattern > 127 bases runs on them) against the
    reference's LandauVishkin<dir> vectors: distance, reverse netIndel, probability bits."""
    rows = _lv_rows(fn)
    tasks = [(t, p, q, int(k)) for _, k, t, p, q, _, _, _ in rows]
    got = snapgpu.lv_batch(direction, tasks, engine="bitplane")
    for (d, k, t, p, q, e, net, prob), (ge, gn, gp) in zip(rows, got):
        assert ge == int(e), (t, p, k, ge, e)
        if int(e) >= 0:
            if direction < 0:
                assert gn == int(net), (t, p, k, gn, net)
            assert np.float64(gp).view(np.uint64) == np.float64(float.fromhex(prob)).view(np.uint64), (t, p, k, gp)
    # the short-pattern vectors through the 256-bit masks too (one long task puts the batch there)
    short = [r for r in _lv_rows("lv_fwd.tsv" if direction > 0 else "lv_rev.tsv") if 0 < len(r[3]) <= 127]
    got = snapgpu.lv_batch(direction, [(t, p, q, int(k)) for _, k, t, p, q, _, _, _ in short] + tasks[:1],
                           engine="bitplane")
    for (d, k, t, p, q, e, net, prob), (ge, gn, gp) in zip(short, got):
        assert ge == int(e), (t, p, k, ge, e)
        if int(e) >= 0:
            assert np.float64(gp).view(np.uint64) == np.float64(float.fromhex(prob)).view(np.uint64)
