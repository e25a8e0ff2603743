"""The single-end RNA product path: `snap-rna single` rebuilt on the GPU.

Fixtures (tests/golden/make_golden.py --only-single) are the reference CLI's own outputs on
tests/golden/small.fa + small.gtf + single_reads.fq: the transcriptome FASTA of
`snap-rna transcriptome` and the SAM files of `snap-rna single ... -t 1` (default and -M).
Our run builds both indexes itself (the GPU box has no reference), loads the GTF, and must
write the same SAM bytes (the @PG line differs only in the command line it echoes)."""
import gzip
import os

import pytest

import snapgpu

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_gtf_model():
    gtf = snapgpu.Gtf.load(os.path.join(G, "small.gtf"))
    c = gtf.counts()
    assert c["transcripts"] >= 20 and c["genes"] == 13 and c["features"] > c["transcripts"]
    # GenomicPosition: exon coordinates only, 0 past the transcript end
    first = [l.split("\t") for l in open(os.path.join(G, "small.gtf")) if '"T0.0"' in l]
    a, b = int(first[0][3]), int(first[0][4])
    assert gtf.genomic_position("T0.0", 1, 100) == a
    assert gtf.genomic_position("T0.0", 10, 0) == a + 9
    assert gtf.genomic_position("T0.0", 10**7, 100) == 0
    ln = b - a + 1
    # a match run across exon 1's end gets the intron as an N run (insertSpliceJunctions)
    nxt = int(first[1][3])
    cig = gtf.splice_cigar("T0.0", ln - 9, [(100, "=")])
    assert cig == f"10={nxt - b - 1}N90="
    assert gtf.splice_cigar("T0.0", 1, [(3, "S"), (50, "="), (2, "I"), (45, "=")]) == "3S50=2I45="


def test_transcriptome_fasta_matches_reference(tmp_path):
    gtf = snapgpu.Gtf.load(os.path.join(G, "small.gtf"))
    g = snapgpu.Genome.from_fasta(os.path.join(G, "small.fa"), 500)
    out = tmp_path / "transcriptome.fa"
    gtf.write_transcriptome(g, out)
    assert out.read_bytes() == gzip.open(os.path.join(G, "expected_transcriptome.fa.gz")).read()


def _indexes(tmp_path):
    gtf = snapgpu.Gtf.load(os.path.join(G, "small.gtf"))
    gidx = snapgpu.GenomeIndex.build(snapgpu.Genome.from_fasta(os.path.join(G, "small.fa"), 500), 20, 4)
    tfa = tmp_path / "transcriptome.fa"
    gtf.write_transcriptome(gidx.genome_handle(), tfa)
    tidx = snapgpu.GenomeIndex.build(snapgpu.Genome.from_fasta(tfa, 500), 20, 4)
    return gtf, gidx, tidx


def _records(text):
    lines = text.splitlines()
    return [l for l in lines if not l.startswith("@PG")]


@pytest.fixture
def single_sub(request, monkeypatch):
    """SNAPGPU_SINGLE_SUBBATCH: useful reads per pipelined sub-batch of snapgpu_single_align (None: the
    default, one sub-batch below 200k reads -- this fixture -- and two halves above; small values cut
    the fixture into many: stage A of sub-batch s + 1 runs while stage B writes sub-batch s)."""
    if request.param:
        monkeypatch.setenv("SNAPGPU_SINGLE_SUBBATCH", str(request.param))
    else:
        monkeypatch.delenv("SNAPGPU_SINGLE_SUBBATCH", raising=False)
    return request.param


@pytest.mark.gpu
@pytest.mark.parametrize("use_m,fixture,single_sub", [(0, "expected_single.sam.gz", None), (1, "expected_single_M.sam.gz", None),
                                                      (0, "expected_single.sam.gz", 97)], indirect=["single_sub"])
def test_single_end_product_path_matches_reference(gpu_available, tmp_path, use_m, fixture, single_sub):
    gtf, gidx, tidx = _indexes(tmp_path)
    ga = snapgpu.BaseAligner(gidx)
    ta = snapgpu.BaseAligner(tidx)
    reads = snapgpu.Reads.from_fastq(os.path.join(G, "single_reads.fq"))
    out = tmp_path / "out.sam"
    st = snapgpu.single_align(ga, ta, gtf, reads, out, useM=use_m, version="0.1alpha", commandLine="x")
    got = out.read_text()
    want = gzip.open(os.path.join(G, fixture), "rt").read()
    g, w = _records(got), _records(want)
    assert len(g) == len(w)
    bad = [(a, b) for a, b in zip(g, w) if a != b]
    assert not bad, f"{len(bad)} lines differ, first: {bad[:2]}"
    assert st["totalReads"] == reads.n and 0 < st["usefulReads"] < reads.n
    assert st["transcriptomeRecords"] > 50
    assert "N" in "".join(l.split("\t")[5] for l in g if not l.startswith("@"))   # junctions exercised
    if not use_m:   # the gene read counts FilterSingle records, written as GTFReader::WriteReadCounts
        gtf.write_counts(tmp_path / "out")
        want, cur = {}, None
        for line in open(os.path.join(G, "expected_single.counts.txt")):
            if line.startswith("## "):
                cur = line[3:].strip()
                want[cur] = ""
            else:
                want[cur] += line
        for name, text in want.items():
            assert open(tmp_path / f"out.{name}.counts.txt").read() == text, name


def _bam_split(raw):
    """Decompressed BAM -> (SAM header text, [(name, l_ref)], record bytes)."""
    import struct
    assert raw[:4] == b"BAM\1"
    l_text = struct.unpack_from("<i", raw, 4)[0]
    text = raw[8:8 + l_text].decode()
    at = 8 + l_text
    n_ref = struct.unpack_from("<i", raw, at)[0]
    at += 4
    refs = []
    for _ in range(n_ref):
        ln = struct.unpack_from("<i", raw, at)[0]
        refs.append([raw[at + 4:at + 4 + ln - 1].decode(), struct.unpack_from("<i", raw, at + 4 + ln)[0]])
        at += 8 + ln
    return text, refs, raw[at:]


@pytest.mark.gpu
@pytest.mark.parametrize("use_m,fixture", [(0, "expected_single"), (1, "expected_single_M")])
def test_single_end_bam_matches_reference(gpu_available, tmp_path, use_m, fixture):
    """`-o out.bam`: BAMFormat::writeHeader / writeRead (Bam.cpp:542-790) in a BGZF stream; the
    decompressed records equal the reference's byte for byte (incl. its NM carry-over on unmapped
    records), the reference list too (the header text echoes the command line)."""
    import json
    gtf, gidx, tidx = _indexes(tmp_path)
    ga = snapgpu.BaseAligner(gidx)
    ta = snapgpu.BaseAligner(tidx)
    reads = snapgpu.Reads.from_fastq(os.path.join(G, "single_reads.fq"))
    out = tmp_path / "out.bam"
    snapgpu.single_align(ga, ta, gtf, reads, out, useM=use_m, version="0.1alpha", commandLine="x")
    data = out.read_bytes()
    assert data[:4] == b"\x1f\x8b\x08\x04" and data[12:14] == b"BC"           # BGZF blocks
    assert data[-28:] == bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")
    text, refs, recs = _bam_split(gzip.decompress(data))
    assert text.startswith("@HD") and "@SQ" in text
    assert refs == json.load(open(os.path.join(G, f"{fixture}.bam.refs.json")))
    want = gzip.decompress(open(os.path.join(G, f"{fixture}.bam.records.gz"), "rb").read())
    g, w = _bam_records(recs), _bam_records(want)
    assert len(g) == len(w)
    # Byte-identical records, except transcriptome records where the reference's n_cigar_op counts
    # one op more than its insertSpliceJunctions (LandauVishkin.cpp:119-236) wrote: that trailing
    # slot is uninitialised stack (a zero op, or an op left over from an earlier record).  Those
    # must equal ours in every other field, with our ops = the reference's minus that last one.
    bad, extra = [], 0
    for k in range(len(w)):
        if g[k] == w[k]:
            continue
        a, b = _bam_fields(g[k]), _bam_fields(w[k])
        same = all(a[f] == b[f] for f in a if f not in ("cigar_ops", "bin"))
        if same and b["cigar_ops"][:-1] == a["cigar_ops"] and b["cigar_ops"]:
            extra += 1
            continue
        bad.append(k)
    diffs = [(k, {f: (_bam_fields(g[k])[f], v) for f, v in _bam_fields(w[k]).items() if _bam_fields(g[k])[f] != v})
             for k in bad[:12]]
    assert not bad, f"{len(bad)} records differ:\n" + "\n".join(f"#{k} {d}" for k, d in diffs)
    assert extra <= 12, extra


def _bam_records(raw):
    import struct
    out, at = [], 0
    while at < len(raw):
        bs = struct.unpack_from("<i", raw, at)[0]
        out.append(raw[at:at + 4 + bs])
        at += 4 + bs
    return out


def _bam_fields(r):
    import struct
    refID, pos, lrn, mapq, bin_, ncig, flag, lseq, nref, npos, tlen = struct.unpack_from("<iiBBHHHiiii", r, 4)
    o = 36
    name = r[o:o + lrn - 1]
    o += lrn
    ops = list(struct.unpack_from("<%dI" % ncig, r, o))
    o += 4 * ncig
    return dict(name=name, refID=refID, pos=pos, mapq=mapq, bin=bin_, flag=flag, lseq=lseq,
                cigar_ops=["%d%s" % (c >> 4, "MIDNSHP=X"[c & 15]) for c in ops],
                seq=r[o:o + (lseq + 1) // 2].hex(), qual=r[o + (lseq + 1) // 2:o + (lseq + 1) // 2 + lseq],
                aux=r[o + (lseq + 1) // 2 + lseq:], nextRef=nref, nextPos=npos, tlen=tlen)
