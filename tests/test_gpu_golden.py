"""GPU path against the REFERENCE's own outputs (tests/golden/, produced by
tests/golden/make_golden.py from oracle/_ref) and, at full size, against the
digests of the reference run on the C1 / C2 synthetic configs."""
import json
import os

import numpy as np
import pytest

import snapgpu
from golden_common import C1, C2, PARAM_SETS, digest, params_to_aligner_kwargs
from oracle_ffi import canonical_tsv

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def small_index():
    return snapgpu.GenomeIndex.build(snapgpu.Genome.from_fasta(os.path.join(G, "small.fa"), 500), 20, 8)


@pytest.fixture(scope="module")
def small_reads():
    return snapgpu.Reads.from_fastq(os.path.join(G, "small_reads.fq"))


@pytest.mark.parametrize("name", list(PARAM_SETS))
def test_gpu_matches_reference_small(gpu_available, small_index, small_reads, name):
    al = snapgpu.BaseAligner(small_index, **params_to_aligner_kwargs(PARAM_SETS[name]))
    got = canonical_tsv(al.AlignReads(small_reads)).splitlines()
    want = open(os.path.join(G, f"expected_small_{name}.tsv")).read().splitlines()
    bad = [(a, b) for a, b in zip(got, want) if a != b]
    assert len(got) == len(want) and not bad, f"{len(bad)} differ: {bad[:3]}"


def test_gpu_matches_reference_datatest(gpu_available):
    idx = snapgpu.GenomeIndex.build(snapgpu.Genome.from_fasta(os.path.join(G, "datatest.fa"), 500), 20, 1)
    al = snapgpu.BaseAligner(idx)
    res = al.AlignReads(snapgpu.Reads.from_fastq(os.path.join(G, "datatest.fq")))
    assert canonical_tsv(res) == open(os.path.join(G, "expected_datatest.tsv")).read()


@pytest.mark.parametrize("cfg", [C1, C2], ids=["C1", "C2"])
def test_gpu_digest_full_config(gpu_available, cfg):
    """Full-size parity: the canonical output of all reads hashes to the digest of
    the reference's own output on the same deterministic inputs."""
    meta = json.load(open(os.path.join(G, "golden.json")))
    g = snapgpu.Genome.synthetic(**cfg["genome"])
    reads = snapgpu.Reads.synthetic(g, **cfg["reads"])
    idx = snapgpu.GenomeIndex.build(g, 20, 16)
    al = snapgpu.BaseAligner(idx)
    res = al.AlignReads(reads)
    tsv = canonical_tsv(res)
    head = open(os.path.join(G, f"expected_{cfg['name']}_head.tsv")).read().splitlines()
    got_head = tsv.splitlines()[:len(head)]
    bad = [(a, b) for a, b in zip(got_head, head) if a != b]
    assert not bad, f"{len(bad)} of first {len(head)} differ: {bad[:3]}"
    assert digest(tsv) == meta["digests"][cfg["name"]]["sha256"]
    # size-independent sanity of the full run
    assert len(res) == cfg["reads"]["n_reads"]
    assert np.all(res["nLookups"] <= 81)
