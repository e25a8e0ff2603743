"""BaseAligner::CharacterizeSeeds (BaseAligner.cpp:206-508), the seed census of
the RNA paired path's partial aligner (PairedAligner.cpp:518-527).

Fixtures: tests/golden/expected_charseeds*.tsv.gz, the reference's own std::map/std::set output
(ref_harness_rna charseeds, BaseAligner.cpp compiled at -O0 -- oracle/Makefile.ref) for the
paired and single-end fixture reads on small.fa.  The C restatement (oracle) is pinned to them on
the CPU; the GPU kernel (csrc/charseeds.hip) to them and to the oracle on a repeat-rich genome."""
import gzip
import os

import numpy as np
import pytest

from oracle_ffi import oracle_charseeds, parse_charseeds, runs_as_lists

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FQS = ("paired_1.fq", "paired_2.fq", "single_reads.fq")
VARIANTS = {"": dict(maxHits=300, maxK=15, numSeeds=12), "_tight": dict(maxHits=20, maxK=15, numSeeds=4)}


def _expected(tag):
    return parse_charseeds(gzip.open(os.path.join(G, f"expected_charseeds{tag}.tsv.gz"), "rt").read())


def _reads():
    import snapgpu
    return [snapgpu.Reads.from_fastq(os.path.join(G, f)) for f in FQS]


@pytest.fixture(scope="module")
def small_index():
    import snapgpu
    g = snapgpu.Genome.from_fasta(os.path.join(G, "small.fa"), 500)
    return snapgpu.GenomeIndex.build(g, 20, 4)


@pytest.mark.parametrize("tag", sorted(VARIANTS))
def test_oracle_matches_reference(small_index, tag):
    want = _expected(tag)
    got = []
    for r in _reads():
        got += runs_as_lists(*oracle_charseeds(small_index, r, **VARIANTS[tag]))
    assert len(got) == len(want)
    bad = [i for i in range(len(want)) if got[i] != want[i]]
    assert not bad, f"{len(bad)} reads differ, first {bad[0]}: {got[bad[0]]} vs {want[bad[0]]}"
    assert sum(len(w[2]) for w in want) > 5000   # the fixture is not trivially empty


@pytest.mark.gpu
@pytest.mark.parametrize("tag", sorted(VARIANTS))
def test_gpu_matches_reference(small_index, tag):
    import snapgpu
    al = snapgpu.BaseAligner(small_index, device=0)
    want = _expected(tag)
    got = []
    for r in _reads():
        start, nfwd, flags, runs = snapgpu.characterize_seeds(al, r, **VARIANTS[tag])
        got += runs_as_lists(start, nfwd, runs)
    bad = [i for i in range(len(want)) if got[i] != want[i]]
    assert not bad, f"{len(bad)} reads differ, first {bad[0]}: {got[bad[0]]} vs {want[bad[0]]}"


@pytest.mark.gpu
def test_gpu_matches_oracle_repeat_rich():
    """C1-sized repeat-rich genome, 20k reads (incl. random and N-rich), plus a read subset."""
    import snapgpu
    g = snapgpu.Genome.synthetic(1_000_000, seed=2121, n_contigs=3, n_repeat_families=60)
    idx = snapgpu.GenomeIndex.build(g, 20, 8)
    reads = snapgpu.Reads.synthetic(idx.genome_handle(), 20000, seed=5, random_read_fraction=0.05)
    al = snapgpu.BaseAligner(idx, device=0)
    for kw in (dict(), dict(maxHits=40, numSeeds=6)):
        s_g, f_g, fl, r_g = snapgpu.characterize_seeds(al, reads, **kw)
        s_o, f_o, r_o = oracle_charseeds(idx, reads, **{**dict(maxHits=300, maxK=15, numSeeds=12), **kw})
        assert np.array_equal(s_g, s_o) and np.array_equal(f_g, f_o)
        assert np.array_equal(r_g.view(np.uint8), r_o.view(np.uint8))
        assert len(r_g) > 20000
    sub = np.arange(7, 20000, 13, dtype=np.uint64)
    s_s, f_s, _, r_s = snapgpu.characterize_seeds(al, reads, read_list=sub)
    s_g, f_g, _, r_g = snapgpu.characterize_seeds(al, reads)
    for j, i in enumerate(sub[:200]):
        a = r_s[int(s_s[j]):int(s_s[j + 1])]
        b = r_g[int(s_g[i]):int(s_g[i + 1])]
        assert np.array_equal(a.view(np.uint8), b.view(np.uint8)) and f_s[j] == f_g[i]
