"""Parity on the reference's own index and at other seed lengths.

* tests/golden/small_ref_index.tar.gz is the on-disk index `snap-rna index` (the reference,
  seed 20, slack 0.3) wrote for tests/golden/small.fa.  snapgpu_index_load
  (GenomeIndex::loadFromDirectory, GenomeIndex.cpp:845-963) reads it; the oracle and the GPU
  aligner over it must reproduce the reference's AlignRead fixture -- this is the index a
  drop-in adapter is handed, with the reference's slot layout and probe chains.
* expected_small_seed{16,22,25}.tsv are the reference's AlignRead outputs over indexes built
  with `snap-rna index -s N`; our builder at those seed lengths (1, 4096 and 262144 tables)
  and the wrap orders of SeedSequencer.h:28-287 must give the same records.
* In the build container, the reference itself loads an index our builder saved.
* The production bit-plane LV (lv_group, align_score.h) against the reference's LV vectors.
"""
import io
import os
import subprocess
import tarfile

import numpy as np
import pytest

import snapgpu
from golden_common import PARAM_SETS, params_to_aligner_kwargs, ref_tsv_to_canonical
from oracle_ffi import canonical_tsv, mismatches, oracle_align

HERE = os.path.dirname(os.path.abspath(__file__))
G = os.path.join(HERE, "golden")
ROOT = os.path.dirname(HERE)
HARNESS = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
SEED_LENS = (16, 22, 25)


def _params():
    p = snapgpu.default_params()
    for k, v in params_to_aligner_kwargs(PARAM_SETS["default"]).items():
        setattr(p, k, v)
    return p


@pytest.fixture(scope="module")
def ref_index_dir(tmp_path_factory):
    d = tmp_path_factory.mktemp("refidx")
    with tarfile.open(os.path.join(G, "small_ref_index.tar.gz"), "r:gz") as t:
        t.extractall(d)
    return str(d)


@pytest.fixture(scope="module")
def small_reads():
    return snapgpu.Reads.from_fastq(os.path.join(G, "small_reads.fq"))


def _diff(got, want):
    g, w = got.splitlines(), want.splitlines()
    assert len(g) == len(w)
    return [(a, b) for a, b in zip(g, w) if a != b]


def test_reference_index_loads(ref_index_dir):
    idx = snapgpu.GenomeIndex.load(ref_index_dir)
    info = idx.info()
    ours = snapgpu.GenomeIndex.build(snapgpu.Genome.from_fasta(os.path.join(G, "small.fa"), 500), 20, 2)
    oi = ours.info()
    for k in ("nBases", "seedLen", "nHashTables", "chromosomePadding", "nPieces", "totalUsedSlots", "hasIupac"):
        assert info[k] == oi[k], k
    # same lookups, different slot layout (the reference inserts in genome order, multi-threaded)
    assert idx.genome_bases(0, info["nBases"]) == ours.genome_bases(0, oi["nBases"])
    rng = np.random.default_rng(4)
    for p in rng.integers(600, info["nBases"] - 600, 400):
        s = idx.genome_bases(int(p), 20).decode()
        if set(s) <= set("ACGT"):
            assert idx.lookupSeed(s) == ours.lookupSeed(s)


def test_oracle_on_reference_index(ref_index_dir, small_reads):
    idx = snapgpu.GenomeIndex.load(ref_index_dir)
    res = oracle_align(idx, small_reads, _params(), n_threads=4)
    bad = _diff(canonical_tsv(res), open(os.path.join(G, "expected_small_default.tsv")).read())
    assert not bad, f"{len(bad)} differ, first: {bad[:3]}"


@pytest.mark.parametrize("seed_len", SEED_LENS)
def test_oracle_seed_lengths(small_reads, seed_len):
    idx = snapgpu.GenomeIndex.build(snapgpu.Genome.from_fasta(os.path.join(G, "small.fa"), 500), seed_len, 4)
    assert idx.info()["nHashTables"] == 1 << (2 * (seed_len - 16))
    res = oracle_align(idx, small_reads, _params(), n_threads=4)
    bad = _diff(canonical_tsv(res), open(os.path.join(G, f"expected_small_seed{seed_len}.tsv")).read())
    assert not bad, f"{len(bad)} differ, first: {bad[:3]}"


@pytest.mark.reference
def test_reference_loads_our_index(tmp_path):
    """The reference's own loader and BaseAligner over an index snapgpu_index_save wrote."""
    if not os.path.exists(HARNESS):
        pytest.skip("oracle/_ref not built (build container only)")
    idx = snapgpu.GenomeIndex.build(snapgpu.Genome.from_fasta(os.path.join(G, "small.fa"), 500), 20, 2)
    d = tmp_path / "ours"
    idx.save(d)
    out = subprocess.run([HARNESS, "align", str(d), os.path.join(G, "small_reads.fq")], capture_output=True,
                         text=True, check=True).stdout
    bad = _diff(ref_tsv_to_canonical(out), open(os.path.join(G, "expected_small_default.tsv")).read())
    assert not bad, f"{len(bad)} differ, first: {bad[:3]}"


# ------------------------------------------------------------------------- GPU
@pytest.mark.gpu
def test_gpu_on_reference_index(gpu_available, ref_index_dir, small_reads):
    idx = snapgpu.GenomeIndex.load(ref_index_dir)
    al = snapgpu.BaseAligner(idx, **params_to_aligner_kwargs(PARAM_SETS["default"]))
    res = al.AlignReads(small_reads)
    bad = _diff(canonical_tsv(res), open(os.path.join(G, "expected_small_default.tsv")).read())
    assert not bad, f"{len(bad)} differ, first: {bad[:3]}"
    cpu = oracle_align(idx, small_reads, al.params, n_threads=4)   # and the counters too (nProbes
    assert not len(mismatches(res, cpu))                           # counts bucket lines: not compared)


@pytest.mark.gpu
@pytest.mark.parametrize("seed_len", SEED_LENS)
def test_gpu_seed_lengths(gpu_available, small_reads, seed_len):
    idx = snapgpu.GenomeIndex.build(snapgpu.Genome.from_fasta(os.path.join(G, "small.fa"), 500), seed_len, 4)
    al = snapgpu.BaseAligner(idx, **params_to_aligner_kwargs(PARAM_SETS["default"]))
    res = al.AlignReads(small_reads)
    bad = _diff(canonical_tsv(res), open(os.path.join(G, f"expected_small_seed{seed_len}.tsv")).read())
    assert not bad, f"{len(bad)} differ, first: {bad[:3]}"


@pytest.mark.gpu
@pytest.mark.parametrize("direction,fn", [(1, "lv_fwd.tsv"), (-1, "lv_rev.tsv")])
def test_gpu_bitplane_lv_matches_reference(gpu_available, direction, fn):
    """lv_group + lv_prob_pair (the LV that scores every read of <= 128 bases) against the
    reference's LandauVishkin<dir> vectors: distance, reverse netIndel, probability bits."""
    rows = [line.rstrip("\n").split("\t") for line in open(os.path.join(G, fn))]
    rows = [r for r in rows if 0 < len(r[3]) <= 127]
    assert len(rows) >= 600
    tasks = [(t, p, q, int(k)) for _, k, t, p, q, _, _, _ in rows]
    got = snapgpu.lv_batch(direction, tasks, engine="bitplane")
    for (d, k, t, p, q, e, net, prob), (ge, gn, gp) in zip(rows, got):
        assert ge == int(e), (t, p, k, ge, e)
        if int(e) >= 0:
            if direction < 0:
                assert gn == int(net), (t, p, k, gn, net)
            assert np.float64(gp).view(np.uint64) == np.float64(float.fromhex(prob)).view(np.uint64), (t, p, k, gp)
