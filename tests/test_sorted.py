"""Sorted SAM output (`-so`, SURVEY.md 8(f) f3 remainder): SortedDataWriter's per-block stable sort
by SAMFormat::getSortInfo's location (SortedDataWriter.cpp:186-240, SAM.cpp:639-685).

Fixtures (tests/golden/make_golden.py --only-sorted): the reference CLI's own sorted outputs,
`snap-rna single ... single_reads.fq -t 1 -o out.sam -so` and `snap-rna paired ...
contam_paired_{1,2}.fq -t 1 -o out.sam -so`.  On the CPU: the reference's own unsorted output of
the same runs, sorted by snapgpu_sam_sort_records, must equal its sorted output.  On the GPU: the
product paths with sortOutput set write it themselves."""
import gzip
import os

import pytest

import snapgpu

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _body(path):
    return b"".join(l for l in gzip.open(path).read().splitlines(keepends=True) if not l.startswith(b"@"))


def _records(text):
    return [l for l in text.splitlines() if not l.startswith("@PG")]


@pytest.fixture(scope="module")
def gidx():
    return snapgpu.GenomeIndex.build(snapgpu.Genome.from_fasta(os.path.join(G, "small.fa"), 500), 20, 4)


@pytest.mark.parametrize("unsorted,sorted_", [("expected_single.sam.gz", "expected_single_sorted.sam.gz"),
                                              ("expected_contam_paired.sam.gz", "expected_paired_sorted.sam.gz")],
                         ids=["single", "paired"])
def test_sort_of_reference_output_matches_reference_sorted(gidx, unsorted, sorted_):
    got = snapgpu.sam_sort_records(gidx, _body(os.path.join(G, unsorted)))
    want = _body(os.path.join(G, sorted_))
    assert got == want
    assert got != _body(os.path.join(G, unsorted))   # the order did change


@pytest.mark.gpu
def test_single_sorted_output_matches_reference(gpu_available, tmp_path, gidx):
    gtf = snapgpu.Gtf.load(os.path.join(G, "small.gtf"))
    tfa = tmp_path / "transcriptome.fa"
    gtf.write_transcriptome(gidx.genome_handle(), tfa)
    tidx = snapgpu.GenomeIndex.build(snapgpu.Genome.from_fasta(tfa, 500), 20, 4)
    reads = snapgpu.Reads.from_fastq(os.path.join(G, "single_reads.fq"))
    out = tmp_path / "out.sam"
    snapgpu.single_align(snapgpu.BaseAligner(gidx), snapgpu.BaseAligner(tidx), gtf, reads, out, sortOutput=1,
                         version="0.1alpha", commandLine="x")
    want = gzip.open(os.path.join(G, "expected_single_sorted.sam.gz"), "rt").read()
    assert _records(out.read_text()) == _records(want)


@pytest.mark.gpu
def test_paired_sorted_output_matches_reference(gpu_available, tmp_path, gidx):
    gtf = snapgpu.Gtf.load(os.path.join(G, "small.gtf"))
    tfa = tmp_path / "transcriptome.fa"
    gtf.write_transcriptome(gidx.genome_handle(), tfa)
    tidx = snapgpu.GenomeIndex.build(snapgpu.Genome.from_fasta(tfa, 500), 20, 4)
    pa = snapgpu.PairedAligner(gidx, device=0)
    ta = snapgpu.BaseAligner(tidx, maxHitsToConsider=16000, maxK=15, maxSeedsToUse=8, extraSearchDepth=2)
    r0 = snapgpu.Reads.from_fastq(os.path.join(G, "contam_paired_1.fq"))
    r1 = snapgpu.Reads.from_fastq(os.path.join(G, "contam_paired_2.fq"))
    out = tmp_path / "out.sam"
    snapgpu.rna_paired_align(pa, ta, gtf, r0, r1, out, sortOutput=1, version="0.1alpha", commandLine="x")
    want = gzip.open(os.path.join(G, "expected_paired_sorted.sam.gz"), "rt").read()
    assert _records(out.read_text()) == _records(want)
    f0 = snapgpu.Reads.from_fastq(os.path.join(G, "contam_paired_1.fq"))
    f1 = snapgpu.Reads.from_fastq(os.path.join(G, "contam_paired_2.fq"))
    with pytest.raises(snapgpu.SnapGpuError, match="sorted output is built for SAM only"):   # sorted BAM: not built
        snapgpu.rna_paired_align(pa, ta, gtf, f0, f1, tmp_path / "out.bam", sortOutput=1)


def test_sort_refuses_records_without_final_newline(gidx):
    body = _body(os.path.join(G, "expected_single.sam.gz"))
    assert body.endswith(b"\n")
    with pytest.raises(snapgpu.SnapGpuError, match="must end with a newline"):
        snapgpu.sam_sort_records(gidx, body[:-1])
    assert snapgpu.sam_sort_records(gidx, b"") == b""
