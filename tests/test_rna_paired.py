"""The RNA paired-end product path: `snap-rna paired` rebuilt on the GPU.

Fixtures (tests/golden/make_golden.py --only-rna-paired): the reference CLI's own outputs
(`snap-rna paired <genome> <transcriptome> <gtf> rna_1.fq rna_2.fq -t 1`, BaseAligner.cpp built at
-O0 -- oracle/Makefile.ref) on tests/golden/small.fa + small.gtf for 2,999 pairs aligned in blocks
of 200 (the reference crashes at the end of larger runs in GTFReader::AnalyzeReadIntervals, which
is not restated; one pair whose block crashes alone is left out): the SAM records (default and -M)
and the six read-count files of every block.  Our run builds both indexes itself, aligns each
block through snapgpu_rna_paired_align with fresh GTF counters and must write the same SAM
records and count files byte for byte (the @PG line echoes a different command line).
The 2 x 150 set (make_golden.py --only-rna150, 2,000 pairs, BASELINE configs[4]'s read length)
is checked the same way over the block partition its generator recorded."""
import gzip
import os

import numpy as np
import pytest

import snapgpu

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
BLOCK = 200
COUNT_FILES = ("transcript_id", "transcript_name", "gene_id", "gene_name", "junction_id", "junction_name")


def _expected_counts(stem="rna"):
    out, cur = {}, None
    for line in open(os.path.join(G, f"expected_{stem}_paired.counts.txt")):
        if line.startswith("## block "):
            _, _, b, name = line.split()
            cur = (int(b), name)
            out[cur] = ""
        else:
            out[cur] += line
    return out


def test_count_files_layout_matches_reference(tmp_path):
    """GTFReader::WriteReadCounts' keys and order (transcripts and genes in id order, each gene's
    introns by key, gene names merged) from the GTF model alone, with every counter at zero."""
    gtf = snapgpu.Gtf.load(os.path.join(G, "small.gtf"))
    gtf.write_counts(tmp_path / "z")
    want = _expected_counts()
    for name in COUNT_FILES:
        got = open(tmp_path / f"z.{name}.counts.txt").read().splitlines()
        exp = want[(0, name)].splitlines()
        assert [l.split("\t")[0] for l in got] == [l.split("\t")[0] for l in exp], name
        assert all(l.endswith("\t0") for l in got), name


def _indexes(tmp_path):
    gtf = snapgpu.Gtf.load(os.path.join(G, "small.gtf"))
    gidx = snapgpu.GenomeIndex.build(snapgpu.Genome.from_fasta(os.path.join(G, "small.fa"), 500), 20, 4)
    tfa = tmp_path / "transcriptome.fa"
    gtf.write_transcriptome(gidx.genome_handle(), tfa)
    tidx = snapgpu.GenomeIndex.build(snapgpu.Genome.from_fasta(tfa, 500), 20, 4)
    return gtf, gidx, tidx


def _blocks(stem, n):
    """[start, end) of each reference run's pairs: fixed blocks of 200 (the 2 x 101 set), or the
    partition make_golden.py recorded (expected_<stem>_blocks.json: blocks halved where the
    reference's AnalyzeReadIntervals crash came up)."""
    p = os.path.join(G, f"expected_{stem}_blocks.json")
    if not os.path.exists(p):
        return [(c, min(n, c + BLOCK)) for c in range(0, n, BLOCK)]
    import json
    sizes = json.load(open(p))["block_sizes"]
    ends = np.cumsum(sizes)
    assert ends[-1] == n
    return list(zip([0] + list(ends[:-1]), ends))


def _fastq_block(path, a, b, dst):
    lines = open(path).read().splitlines()
    with open(dst, "w") as f:
        f.write("\n".join(lines[4 * a:4 * b]) + "\n")


# stem: 2 x <=101 pairs (rna_*.fq) and 2 x 150 pairs, BASELINE configs[4]'s read length (rna150_*.fq:
# 150-b mates through align_kernel<256> multi-hit, paired_kernel<256>, 150-b CIGARs and splices)
@pytest.fixture
def subbatch(request, monkeypatch):
    """SNAPGPU_RNA_SUBBATCH: pairs per pipelined sub-batch of snapgpu_rna_paired_align (None: the
    default, one sub-batch below 40k pairs -- these fixtures -- and two halves above; small values
    cut a block into several)."""
    if request.param:
        monkeypatch.setenv("SNAPGPU_RNA_SUBBATCH", str(request.param))
    else:
        monkeypatch.delenv("SNAPGPU_RNA_SUBBATCH", raising=False)
    return request.param


@pytest.mark.gpu
@pytest.mark.parametrize("stem,use_m,subbatch", [("rna", 0, None), ("rna", 1, None), ("rna150", 0, None),
                                                 ("rna150", 1, None), ("rna150", 0, 37)], indirect=["subbatch"])
def test_rna_paired_product_path_matches_reference(gpu_available, tmp_path, use_m, stem, subbatch):
    fixture = f"expected_{stem}_paired{'_M' if use_m else ''}.sam.gz"
    gtf, gidx, tidx = _indexes(tmp_path)
    pa = snapgpu.PairedAligner(gidx, device=0)   # paired CLI defaults (maxHits 16000, maxK 15, 8 seeds)
    ta = snapgpu.BaseAligner(tidx, maxHitsToConsider=16000, maxK=15, maxSeedsToUse=8, extraSearchDepth=2)
    n = sum(1 for _ in open(os.path.join(G, f"{stem}_1.fq"))) // 4
    body, counts = [], _expected_counts(stem)
    totals = dict(partialPairs=0, partialMatches=0, transcriptomeRecords=0, multiHits=0)
    for b, (a0, a1) in enumerate(_blocks(stem, n)):
        f0, f1 = tmp_path / "b_1.fq", tmp_path / "b_2.fq"
        _fastq_block(os.path.join(G, f"{stem}_1.fq"), a0, a1, f0)
        _fastq_block(os.path.join(G, f"{stem}_2.fq"), a0, a1, f1)
        r0, r1 = snapgpu.Reads.from_fastq(f0), snapgpu.Reads.from_fastq(f1)
        gtf.reset_counts()
        sam = tmp_path / "b.sam"
        res, st = snapgpu.rna_paired_align(pa, ta, gtf, r0, r1, sam, useM=use_m)
        for k in totals:
            totals[k] += st[k]
        assert st["subBatches"] == (-(-(a1 - a0) // subbatch) if subbatch else 1)
        lines = open(sam).read().splitlines(keepends=True)
        if b == 0:
            body += [l for l in lines if l.startswith("@") and not l.startswith("@PG")]
        body += [l for l in lines if not l.startswith("@")]
        if not use_m:
            gtf.write_counts(tmp_path / "c")
            for name in COUNT_FILES:
                got = open(tmp_path / f"c.{name}.counts.txt").read()
                assert got == counts[(b, name)], f"block {b} {name}"
    want = [l for l in gzip.open(os.path.join(G, fixture), "rt").read().splitlines(keepends=True)
            if not l.startswith("@PG")]
    got = "".join(body).splitlines(keepends=True)
    assert len(got) == len(want)
    bad = [i for i in range(len(want)) if got[i] != want[i]]
    assert not bad, f"{len(bad)} SAM lines differ, first:\n got  {got[bad[0]]} want {want[bad[0]]}"
    # the fixture exercises the filter's branches: transcriptome records, FindPartialMatches
    # scans on the GPU, MultipleHits
    assert totals["transcriptomeRecords"] > 100 and totals["partialPairs"] > 20 and totals["multiHits"] > 10, totals
    if stem == "rna150":   # the configs[4] read length really is exercised
        r0 = snapgpu.Reads.from_fastq(os.path.join(G, "rna150_1.fq"))
        assert sum(1 for i in range(r0.n) if len(r0.get(i)[0]) == 150) > 0.5 * r0.n


@pytest.mark.gpu
@pytest.mark.parametrize("stem,use_m,subbatch", [("rna", 0, None), ("rna", 1, None), ("rna150", 0, None),
                                                 ("rna150", 1, None), ("rna", 0, 29)], indirect=["subbatch"])
def test_rna_paired_bam_matches_reference(gpu_available, tmp_path, use_m, stem, subbatch):
    """`snap-rna paired ... -o out.bam`: SimpleReadWriter::writePair -> BAMFormat::writeRead of both
    ends with their mate fields (ReadWriter.cpp:133-217, Bam.cpp:596-790) in a BGZF stream; the
    decompressed records of every block equal the reference's byte for byte, including the NM the
    reference carries over onto unmapped records (fixtures: make_golden.py --only-rna-bam), also across
pipelined sub-batches (subbatch 29).  As for
    the single-end BAM, a transcriptome record may differ only by the trailing uninitialised CIGAR
    slot the reference counts in n_cigar_op (insertSpliceJunctions)."""
    import json
    from test_single import _bam_fields, _bam_records, _bam_split
    gtf, gidx, tidx = _indexes(tmp_path)
    pa = snapgpu.PairedAligner(gidx, device=0)
    ta = snapgpu.BaseAligner(tidx, maxHitsToConsider=16000, maxK=15, maxSeedsToUse=8, extraSearchDepth=2)
    n = sum(1 for _ in open(os.path.join(G, f"{stem}_1.fq"))) // 4
    recs, refs = [], None
    for b, (a0, a1) in enumerate(_blocks(stem, n)):
        f0, f1 = tmp_path / "b_1.fq", tmp_path / "b_2.fq"
        _fastq_block(os.path.join(G, f"{stem}_1.fq"), a0, a1, f0)
        _fastq_block(os.path.join(G, f"{stem}_2.fq"), a0, a1, f1)
        r0, r1 = snapgpu.Reads.from_fastq(f0), snapgpu.Reads.from_fastq(f1)
        gtf.reset_counts()
        out = tmp_path / "b.bam"
        snapgpu.rna_paired_align(pa, ta, gtf, r0, r1, out, useM=use_m)
        data = out.read_bytes()
        assert data[:4] == b"\x1f\x8b\x08\x04" and data[-28:] == bytes.fromhex(
            "1f8b08040000000000ff0600424302001b0003000000000000000000")
        text, rf, rb = _bam_split(gzip.decompress(data))
        refs = refs or rf
        recs += _bam_records(rb)
    assert refs == json.load(open(os.path.join(G, f"expected_{stem}_paired.bam.refs.json")))
    want = _bam_records(gzip.decompress(open(os.path.join(
        G, f"expected_{stem}_paired{'_M' if use_m else ''}.bam.records.gz"), "rb").read()))
    assert len(recs) == len(want) == 2 * n
    bad, extra = [], 0
    for k in range(len(want)):
        if recs[k] == want[k]:
            continue
        a, b = _bam_fields(recs[k]), _bam_fields(want[k])
        if all(a[f] == b[f] for f in a if f not in ("cigar_ops", "bin")) and b["cigar_ops"] and \
                b["cigar_ops"][:-1] == a["cigar_ops"]:
            extra += 1
            continue
        bad.append(k)
    diffs = [(k, {f: (_bam_fields(recs[k])[f], v) for f, v in _bam_fields(want[k]).items()
                  if _bam_fields(recs[k])[f] != v}) for k in bad[:12]]
    assert not bad, f"{len(bad)} records differ:\n" + "\n".join(f"#{k} {d}" for k, d in diffs)
    paired = sum(1 for r in want if _bam_fields(r)["flag"] & 0x2)
    assert paired > 100 and extra <= len(want) // 50, (paired, extra)


@pytest.mark.gpu
def test_rna_paired_through_big_arena_pass_matches_reference(gpu_available, tmp_path, monkeypatch):
    """The whole RNA paired product path with every aligner's arena capped at 2 elements: the
    transcriptome multi-hit reads, the chimeric fallback's reads and the reads of the seed census
    that outgrow it are aligned again by the big-arena pass (align_kernel<512> on worst-case arenas);
    the 2 x 150 SAM records still equal the reference CLI's."""
    monkeypatch.setenv("SNAPGPU_ARENA_CAP", "2")
    test_rna_paired_product_path_matches_reference(gpu_available, tmp_path, 0, "rna150", None)
    gtf, gidx, tidx = _indexes(tmp_path)
    ta = snapgpu.BaseAligner(tidx, maxHitsToConsider=16000, maxK=15, maxSeedsToUse=8, extraSearchDepth=2)
    r0 = snapgpu.Reads.from_fastq(os.path.join(G, "rna150_1.fq"))
    r0.clip(3)
    ta.AlignReadsEx(r0, maxHitsToGet=1000)
    assert ta.timing()["nArenaOverflow"] > 0   # the cap really sent reads through the big-arena pass


@pytest.mark.gpu
def test_rna_paired_force_spacing_matches_reference(gpu_available, tmp_path):
    """`snap-rna paired ... -fs` (PairedAligner.cpp:274-275; the chimeric aligner keeps a pair with
    a NotFound end as it is, ChimericPairedEndAligner.cpp:93-96, and a pair with exactly one end
    SingleHit becomes NotFound on both ends, PairedAligner.cpp:648-651): SAM records of the blocks
    the reference completes with -fs (it segfaults in the others, make_golden.py --only-rna-fs).
    The CIGAR batches are issued before the spacing adjustment (rna_paired.cpp, stage B), so this is
    also the test that a record losing its location there is written without one.

    Excluded: the pairs IntersectingPairedEndAligner::align leaves without writing a location (a
    mate shorter than 50 bases or more than maxK Ns in the pair, IntersectingPairedEndAligner.cpp:
    185-187, 226-228).  With -fs the chimeric aligner returns them as they are (:93-100), so
    PairedAligner.cpp:577's uninitialised `result` hands the filter whatever the stack slot held --
    the previous pair's locations (the reference writes such a pair mapped with CIGAR `*` and NM -1).
    That is undefined behaviour, not a rule to restate; every other pair must match."""
    import json
    meta = json.load(open(os.path.join(G, "expected_rna_paired_fs_blocks.json")))
    assert meta["records_differing_from_plain"] > 100   # -fs really changes the records
    gtf, gidx, tidx = _indexes(tmp_path)
    pa = snapgpu.PairedAligner(gidx, device=0, forceSpacing=1)
    ta = snapgpu.BaseAligner(tidx, maxHitsToConsider=16000, maxK=15, maxSeedsToUse=8, extraSearchDepth=2)
    n = sum(1 for _ in open(os.path.join(G, "rna_1.fq"))) // 4
    body = []
    for b, a0 in enumerate(meta["starts"]):
        a1 = min(n, a0 + meta["block"])
        f0, f1 = tmp_path / "b_1.fq", tmp_path / "b_2.fq"
        _fastq_block(os.path.join(G, "rna_1.fq"), a0, a1, f0)
        _fastq_block(os.path.join(G, "rna_2.fq"), a0, a1, f1)
        r0, r1 = snapgpu.Reads.from_fastq(f0), snapgpu.Reads.from_fastq(f1)
        gtf.reset_counts()
        sam = tmp_path / "b.sam"
        snapgpu.rna_paired_align(pa, ta, gtf, r0, r1, sam, forceSpacing=1)
        lines = open(sam).read().splitlines(keepends=True)
        if b == 0:
            body += [l for l in lines if l.startswith("@") and not l.startswith("@PG")]
        body += [l for l in lines if not l.startswith("@")]
    want = [l for l in gzip.open(os.path.join(G, "expected_rna_paired_fs.sam.gz"), "rt").read().splitlines(keepends=True)
            if not l.startswith("@PG")]
    got = "".join(body).splitlines(keepends=True)
    assert len(got) == len(want)
    recs = [open(os.path.join(G, f"rna_{k}.fq")).read().splitlines() for k in (1, 2)]
    early = set()
    for a0 in meta["starts"]:
        for i in range(a0, min(n, a0 + meta["block"])):
            s0, s1 = recs[0][4 * i + 1], recs[1][4 * i + 1]
            if len(s0) < 50 or len(s1) < 50 or sum(c in "Nn" for c in s0 + s1) > pa.params.maxK:
                early.add(recs[0][4 * i][1:].split()[0].split("/")[0])
    assert 0 < len(early) < 0.05 * len(want) / 2
    bad = [i for i in range(len(want)) if got[i] != want[i] and want[i].split("\t")[0] not in early]
    assert not bad, f"{len(bad)} SAM lines differ, first:\n got  {got[bad[0]]} want {want[bad[0]]}"
    assert sum(1 for i in range(len(want)) if got[i] == want[i]) >= len(want) - 2 * len(early)
