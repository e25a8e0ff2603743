"""The contamination database (`-ct`, SURVEY.md 8(f) f1/f4 remainder): ContaminationFilter.

Fixtures (tests/golden/make_golden.py --only-contam) are the reference CLI's own outputs:
`snap-rna single|paired <genome> <transcriptome> <gtf> ... -t 1 -o out.sam -ct <contam index>` on
tests/golden/small.fa + small.gtf + contam.fa (five random contigs) with reads and pairs mixed from
the existing fixtures and from the contigs: out.contaminants.txt (contig, count; by count,
descending -- three contigs tie) and the SAM file (the generator checked that -ct leaves it as it
is without).  Our runs build the three indexes themselves and must write the same file."""
import gzip
import os

import pytest

import snapgpu

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _contam_index():
    return snapgpu.GenomeIndex.build(snapgpu.Genome.from_fasta(os.path.join(G, "contam.fa"), 500), 20, 4)


def test_counts_file_format_and_order(tmp_path):
    """ContaminationFilter::Write from counts added in any order: name-ordered counts sorted by count
    descending with the reference's own std::sort call (ties as it leaves them), and the file name
    from the output template (up to its last '.'; "default" without one)."""
    idx = _contam_index()
    want = open(os.path.join(G, "expected_contam_single.contaminants.txt")).read()
    per = {l.split("\t")[0]: int(l.split("\t")[1]) for l in want.splitlines()}
    # one location inside each contig (the index's genome: the same FASTA loader and padding)
    c = snapgpu.Contaminants(idx)
    pieces = snapgpu.Genome.from_fasta(os.path.join(G, "contam.fa"), 500).pieces
    starts = [off for _, off in pieces]
    names = [name for name, _ in pieces]
    assert sorted(per) == names   # cont1..cont5 in FASTA order
    order = [n for n in names for _ in range(per[n])]
    order = order[::7] + [x for i, x in enumerate(order) if i % 7]   # interleaved adds
    for n in order:
        c.add(starts[names.index(n)] + 17)
    c.add(0xFFFFFFFF)   # rname "*", pos 0: not counted
    assert c.text() == want
    c.write(tmp_path / "out.sam")
    assert (tmp_path / "out.contaminants.txt").read_text() == want
    d = snapgpu.Contaminants(idx)
    cwd = os.getcwd()
    try:
        os.chdir(tmp_path)
        d.write(None)
        assert (tmp_path / "default.contaminants.txt").read_text() == ""
    finally:
        os.chdir(cwd)


def _indexes(tmp_path):
    gtf = snapgpu.Gtf.load(os.path.join(G, "small.gtf"))
    gidx = snapgpu.GenomeIndex.build(snapgpu.Genome.from_fasta(os.path.join(G, "small.fa"), 500), 20, 4)
    tfa = tmp_path / "transcriptome.fa"
    gtf.write_transcriptome(gidx.genome_handle(), tfa)
    tidx = snapgpu.GenomeIndex.build(snapgpu.Genome.from_fasta(tfa, 500), 20, 4)
    return gtf, gidx, tidx, _contam_index()


def _records(text):
    return [l for l in text.splitlines() if not l.startswith("@PG")]


@pytest.mark.gpu
@pytest.mark.parametrize("sub", [None, 53])
def test_single_contamination_matches_reference(gpu_available, tmp_path, monkeypatch, sub):
    """(sub: SNAPGPU_SINGLE_SUBBATCH -- the contamination batches and counts of a pipelined call)"""
    if sub:
        monkeypatch.setenv("SNAPGPU_SINGLE_SUBBATCH", str(sub))
    gtf, gidx, tidx, cidx = _indexes(tmp_path)
    ga, ta, ca = snapgpu.BaseAligner(gidx), snapgpu.BaseAligner(tidx), snapgpu.BaseAligner(cidx)
    counts = snapgpu.Contaminants(cidx)
    reads = snapgpu.Reads.from_fastq(os.path.join(G, "contam_single.fq"))
    out = tmp_path / "out.sam"
    snapgpu.single_align(ga, ta, gtf, reads, out, contamination=(ca, counts), version="0.1alpha", commandLine="x")
    want = gzip.open(os.path.join(G, "expected_contam_single.sam.gz"), "rt").read()
    assert _records(out.read_text()) == _records(want)
    counts.write(out)
    assert (tmp_path / "out.contaminants.txt").read_text() == \
        open(os.path.join(G, "expected_contam_single.contaminants.txt")).read()


@pytest.mark.gpu
def test_paired_contamination_matches_reference(gpu_available, tmp_path):
    gtf, gidx, tidx, cidx = _indexes(tmp_path)
    pa = snapgpu.PairedAligner(gidx, device=0)   # paired CLI defaults (maxHits 16000, maxK 15, 8 seeds)
    ta = snapgpu.BaseAligner(tidx, maxHitsToConsider=16000, maxK=15, maxSeedsToUse=8, extraSearchDepth=2)
    ca = snapgpu.PairedAligner(cidx, device=0)   # the genome aligner's parameters (PairedAligner.cpp:487-505)
    counts = snapgpu.Contaminants(cidx)
    r0 = snapgpu.Reads.from_fastq(os.path.join(G, "contam_paired_1.fq"))
    r1 = snapgpu.Reads.from_fastq(os.path.join(G, "contam_paired_2.fq"))
    out = tmp_path / "out.sam"
    snapgpu.rna_paired_align(pa, ta, gtf, r0, r1, out, contamination=(ca, counts), version="0.1alpha", commandLine="x")
    want = gzip.open(os.path.join(G, "expected_contam_paired.sam.gz"), "rt").read()
    assert _records(out.read_text()) == _records(want)
    counts.write(out)
    assert (tmp_path / "out.contaminants.txt").read_text() == \
        open(os.path.join(G, "expected_contam_paired.contaminants.txt")).read()


@pytest.mark.gpu
def test_refused_single_call_leaves_counts_unchanged(gpu_available, tmp_path):
    """A sorted-BAM single-end call is refused (not built) before any alignment or counting, so the
    caller's GTF read counts and contamination counts are what they were; the same call as SAM then
    counts exactly as the reference's -ct run."""
    gtf, gidx, tidx, cidx = _indexes(tmp_path)
    ga, ta, ca = snapgpu.BaseAligner(gidx), snapgpu.BaseAligner(tidx), snapgpu.BaseAligner(cidx)
    counts = snapgpu.Contaminants(cidx)
    reads = snapgpu.Reads.from_fastq(os.path.join(G, "contam_single.fq"))
    gtf.write_counts(tmp_path / "before")
    with pytest.raises(snapgpu.SnapGpuError, match="sorted output is built for SAM only"):
        snapgpu.single_align(ga, ta, gtf, reads, tmp_path / "out.bam", sortOutput=1, contamination=(ca, counts))
    assert counts.text() == ""
    gtf.write_counts(tmp_path / "after")
    files = sorted(tmp_path.glob("before.*counts.txt"))
    assert len(files) == 6
    for f in files:
        assert f.read_bytes() == (tmp_path / f.name.replace("before", "after", 1)).read_bytes(), f.name
    out = tmp_path / "out.sam"
    snapgpu.single_align(ga, ta, gtf, reads, out, contamination=(ca, counts), version="0.1alpha", commandLine="x")
    counts.write(out)
    assert (tmp_path / "out.contaminants.txt").read_text() == \
        open(os.path.join(G, "expected_contam_single.contaminants.txt")).read()
