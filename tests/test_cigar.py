"""CIGAR strings and SAM records: the reference SAM writer's
per-read work -- SAMFormat::writeRead / computeCigarString (SNAPLib/SAM.cpp:804-1230)
around LandauVishkinWithCigar (SNAPLib/LandauVishkin.cpp:252-535).

Pinned against the reference itself (tests/golden/, tests/golden/make_golden.py
--only-cigar): 6.6k LandauVishkinWithCigar calls at aligned, perturbed and random
locations (expected_cigar.tsv) and the reference's own SAM lines for the 2,225
small-genome reads, useM = 0 and 1 (expected_small.sam.gz).  CPU tests pin the
oracle restatement and the host SAM formatter; GPU tests run the HIP cigar_kernel."""
import gzip
import os

import numpy as np
import pytest

import snapgpu
from oracle_ffi import mismatches, oracle_align, oracle_cigars, sam_pattern

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _fastq(path):
    lines = open(path).read().split("\n")
    return [(lines[i][1:], lines[i + 1], lines[i + 3]) for i in range(0, len(lines) - 3, 4)]


@pytest.fixture(scope="module")
def small():
    idx = snapgpu.GenomeIndex.build(snapgpu.Genome.from_fasta(os.path.join(G, "small.fa"), 500), 20, 8)
    fq = _fastq(os.path.join(G, "small_reads.fq"))
    reads = snapgpu.Reads.from_fastq(os.path.join(G, "small_reads.fq"))
    return idx, fq, reads


@pytest.fixture(scope="module")
def calls():
    rows = [l.split("\t") for l in open(os.path.join(G, "cigar_calls.tsv")).read().splitlines()]
    want = []
    for l in open(os.path.join(G, "expected_cigar.tsv")).read().splitlines():
        ed, cig = l.split("\t")
        want.append((-1, "*") if int(ed) < 0 else (int(ed), cig))   # -3: no substring -> "*"
    return [(int(a), int(b), int(c), d) for a, b, c, d in rows], want


def _reference_results(n):
    """The reference's AlignRead records for the small reads (expected_small_default.tsv)."""
    res = np.zeros(n, dtype=snapgpu.RESULT_DTYPE)
    for i, l in enumerate(open(os.path.join(G, "expected_small_default.tsv")).read().splitlines()):
        x = l.split("\t")
        res[i]["result"], res[i]["location"], res[i]["direction"] = int(x[1]), int(x[2]), int(x[3])
        res[i]["score"], res[i]["mapq"] = int(x[4]), int(x[5])
    return res


def _cigars_from_pairs(pairs):
    c = snapgpu.Cigars.empty(len(pairs))
    for i, (ed, s) in enumerate(pairs):
        c.editDistance[i] = ed
        k = 0
        num = ""
        for ch in s if ed >= 0 else "":
            if ch.isdigit():
                num += ch
            else:
                c.ops[i, k] = (int(num) << 4) | snapgpu.CIGAR_OPS.index(ch)
                k += 1
                num = ""
        c.nOps[i] = k
    return c


def _sam_lines(use_m):
    lines = gzip.open(os.path.join(G, "expected_small.sam.gz"), "rt").read().splitlines()
    return lines[use_m::2]


# ------------------------------------------------------------------ CPU
def test_oracle_cigar_matches_reference(small, calls):
    idx, _, _ = small
    rows, want = calls
    for use_m in (0, 1):
        sel = [i for i, r in enumerate(rows) if r[2] == use_m]
        got = oracle_cigars(idx, [rows[i][3] for i in sel], [rows[i][0] for i in sel], [rows[i][1] for i in sel],
                            use_m)
        bad = [(rows[i], g, want[i]) for i, g in zip(sel, got) if g != want[i]]
        assert not bad, f"{len(bad)} of {len(sel)} differ, e.g. {bad[:2]}"


def test_sam_pattern_orientation():
    assert sam_pattern("acgtNx", 0) == b"ACGTNX"
    assert sam_pattern("AACGTN", 1) == b"NACGTT"
    assert sam_pattern("AXG", 1) == b"C\0T"


@pytest.mark.parametrize("use_m", [0, 1])
def test_host_sam_format_matches_reference(small, use_m):
    """Host SAM formatter over the reference's own records + oracle CIGARs reproduces
    the reference's SAM lines byte for byte."""
    idx, fq, reads = small
    res = _reference_results(len(fq))
    loc, dirs = snapgpu.cigar_inputs(res)
    cig = _cigars_from_pairs(oracle_cigars(idx, [b for _, b, _ in fq], loc, dirs, use_m))
    got = snapgpu.sam_format(idx, reads, [i for i, _, _ in fq], res, cig).decode().splitlines()
    want = _sam_lines(use_m)
    bad = [(a, b) for a, b in zip(got, want) if a != b]
    assert len(got) == len(want) and not bad, f"{len(bad)} differ: {bad[:2]}"


def test_sam_format_rejects_small_buffer(small):
    import ctypes as C
    idx, fq, reads = small
    res = _reference_results(len(fq))
    cig = snapgpu.Cigars.empty(len(fq))
    used = C.c_uint64()
    buf = C.create_string_buffer(16)
    blob = b"".join(i.encode() for i, _, _ in fq)
    lens = np.array([len(i) for i, _, _ in fq], dtype=np.uint32)
    offs = np.concatenate([[0], np.cumsum(lens[:-1])]).astype(np.uint64)
    rc = snapgpu.lib().snapgpu_sam_format(idx._h, reads._p, blob, offs.ctypes.data, lens.ctypes.data, res.ctypes.data,
                                          cig.editDistance.ctypes.data, cig.nOps.ctypes.data, cig.ops.ctypes.data,
                                          None, buf, 16, C.byref(used))
    assert rc != 0 and used.value > 16


# ------------------------------------------------------------------ GPU
@pytest.mark.gpu
def test_gpu_cigar_matches_reference(gpu_available, small, calls):
    idx, _, _ = small
    rows, want = calls
    al = snapgpu.BaseAligner(idx)
    for use_m in (0, 1):
        sel = [i for i, r in enumerate(rows) if r[2] == use_m]
        reads = snapgpu.Reads.from_list([(rows[i][3], "I" * len(rows[i][3])) for i in sel])
        c = al.Cigars(reads, [rows[i][0] for i in sel], [rows[i][1] for i in sel], useM=use_m)
        got = [(int(c.editDistance[j]), c.string(j)) for j in range(len(sel))]
        bad = [(rows[i], g, want[i]) for i, g in zip(sel, got) if g != want[i]]
        assert not bad, f"{len(bad)} of {len(sel)} differ, e.g. {bad[:2]}"


@pytest.mark.gpu
@pytest.mark.parametrize("use_m", [0, 1])
def test_gpu_sam_records_match_reference(gpu_available, small, use_m):
    """Product path: GPU AlignRead -> resident GPU CIGARs -> host SAM lines, against the
    reference's `AlignRead` + `SAMFormat::writeRead` output."""
    idx, fq, reads = small
    al = snapgpu.BaseAligner(idx)
    dev = al.upload(reads)
    dev.run()
    dev.run_cigars(useM=use_m)
    res = dev.results()
    cig = dev.cigars()
    got = snapgpu.sam_format(idx, reads, [i for i, _, _ in fq], res, cig).decode().splitlines()
    want = _sam_lines(use_m)
    bad = [(a, b) for a, b in zip(got, want) if a != b]
    assert len(got) == len(want) and not bad, f"{len(bad)} differ: {bad[:2]}"


@pytest.mark.gpu
def test_gpu_cigar_matches_oracle_c1(gpu_available, small_world):
    """4,000 C1-shaped reads at their aligned location and at shifted locations (large
    edit distances, '*' results), both directions, useM 0/1: GPU vs the oracle."""
    idx, reads = small_world["index"], small_world["reads"]
    res = oracle_align(idx, reads, snapgpu.default_params())
    loc, dirs = snapgpu.cigar_inputs(res)
    rng = np.random.default_rng(5)
    shift = np.where(rng.random(len(loc)) < 0.5, 0, rng.integers(-40, 41, len(loc)))
    loc2 = np.where(loc == 0xFFFFFFFF, rng.integers(0, 1_000_000, len(loc)), loc.astype(np.int64) + shift)
    loc2 = np.clip(loc2, 0, 0xFFFFFFFE).astype(np.uint32)
    dirs2 = np.where(rng.random(len(loc)) < 0.1, 1 - dirs, dirs).astype(np.uint8)
    bases = [reads.get(i)[0] for i in range(reads.n)]
    al = snapgpu.BaseAligner(idx)
    for use_m in (0, 1):
        c = al.Cigars(reads, loc2, dirs2, useM=use_m)
        want = oracle_cigars(idx, bases, loc2, dirs2, use_m)
        got = [(int(c.editDistance[j]), c.string(j)) for j in range(reads.n)]
        bad = [j for j in range(reads.n) if got[j] != want[j]]
        assert not bad, f"{len(bad)} differ, e.g. {[(got[j], want[j]) for j in bad[:2]]}"
        assert sum(1 for e, _ in want if e > 3) > 100     # indel-heavy / large-distance cases exercised


@pytest.mark.gpu
def test_gpu_cigar_edge_cases(gpu_available, small):
    """Empty batch; zero-length and single-base reads; no location; genome start/end;
    reads longer than 512 bases rejected; all-N read."""
    idx, _, _ = small
    al = snapgpu.BaseAligner(idx)
    empty = al.Cigars(snapgpu.Reads.from_list([]), [], [])
    assert len(empty.editDistance) == 0
    g = snapgpu.Genome.from_fasta(os.path.join(G, "small.fa"), 500)
    nb = g.n_bases
    seq = g.bases(600, 120).decode()
    rows = [("", 600, 0), ("A", 600, 0), (seq, 0xFFFFFFFF, 0), (seq, 0, 0), (seq, nb - 120, 1), (seq, nb + 50, 0),
            ("N" * 100, 600, 0), (seq, 600, 1), (seq.lower(), 600, 0), (seq[:60] + "ACGT" + seq[60:], 600, 0)]
    reads = snapgpu.Reads.from_list([(b, "I" * len(b)) for b, _, _ in rows])
    for use_m in (0, 1):
        c = al.Cigars(reads, [r[1] for r in rows], [r[2] for r in rows], useM=use_m)
        want = oracle_cigars(idx, [r[0] for r in rows], [r[1] for r in rows], [r[2] for r in rows], use_m)
        got = [(int(c.editDistance[j]), c.string(j)) for j in range(len(rows))]
        assert got == want, [(i, a, b) for i, (a, b) in enumerate(zip(got, want)) if a != b]
    assert got[2] == (-1, "*") and got[5] == (-1, "*")
    long_read = snapgpu.Reads.from_list([("A" * 513, "I" * 513)])
    with pytest.raises(snapgpu.SnapGpuError):
        al.Cigars(long_read, [600], [0])


@pytest.mark.parametrize("sorted_output", [0, 1])
def test_sam_header_matches_reference(small, sorted_output):
    """SAMFormat::writeHeader (SAM.cpp:700-800) for a FASTQ input, against the reference's own."""
    idx, _, _ = small
    got = snapgpu.sam_header(idx, "snap-rna single idx reads.fq -o out.sam", "1.0dev.66",
                             sorted_output=bool(sorted_output)).decode()
    want = open(os.path.join(G, f"expected_small_header{sorted_output}.sam")).read()
    assert got == want


def _clipped_reads():
    reads = snapgpu.Reads.from_fastq(os.path.join(G, "small_reads.fq"))
    clip = reads.clip(3)   # ClipFrontAndBack, the reference FASTQ reader's default
    return reads, clip


def _clipped_lines(use_m):
    return gzip.open(os.path.join(G, "expected_small_clipped.sam.gz"), "rt").read().splitlines()[use_m::2]


@pytest.mark.parametrize("use_m", [0, 1])
def test_clipped_sam_matches_reference_cpu(small, use_m):
    """Read::clip + soft clips: oracle AlignRead and CIGARs of the clipped reads, host SAM
    lines with the unclipped SEQ/QUAL, against the reference (clipping = ClipFrontAndBack)."""
    idx, fq, _ = small
    reads, clip = _clipped_reads()
    assert sum(1 for i in range(reads.n) if int(clip[1][i]) != len(reads.get(i)[0])) > 20   # clipping exercised
    res = oracle_align(idx, reads, snapgpu.default_params())
    loc, dirs = snapgpu.cigar_inputs(res)
    cig = _cigars_from_pairs(oracle_cigars(idx, [reads.get(i)[0] for i in range(reads.n)], loc, dirs, use_m))
    got = snapgpu.sam_format(idx, reads, [i for i, _, _ in fq], res, cig, clip=clip).decode().splitlines()
    want = _clipped_lines(use_m)
    bad = [(a, b) for a, b in zip(got, want) if a != b]
    assert len(got) == len(want) and not bad, f"{len(bad)} differ: {bad[:2]}"


@pytest.mark.gpu
@pytest.mark.parametrize("use_m", [0, 1])
def test_gpu_clipped_sam_matches_reference(gpu_available, small, use_m):
    idx, fq, _ = small
    reads, clip = _clipped_reads()
    al = snapgpu.BaseAligner(idx)
    dev = al.upload(reads)
    dev.run()
    dev.run_cigars(useM=use_m)
    res, cig = dev.results(), dev.cigars()
    got = snapgpu.sam_format(idx, reads, [i for i, _, _ in fq], res, cig, clip=clip).decode().splitlines()
    want = _clipped_lines(use_m)
    bad = [(a, b) for a, b in zip(got, want) if a != b]
    assert len(got) == len(want) and not bad, f"{len(bad)} differ: {bad[:2]}"


@pytest.mark.gpu
def test_gpu_cigar_batch_views_and_buffer_reuse(gpu_available, small_world):
    """snapgpu_cigar_batch packs the listed reads into the aligner's grow-only buffers: batch views
    into a larger read buffer (slices), calls of growing and shrinking sizes and useM switches give
    the rows a single whole-batch call gives."""
    idx, reads = small_world["index"], small_world["reads"]
    res = oracle_align(idx, reads, snapgpu.default_params())
    loc, dirs = snapgpu.cigar_inputs(res)
    al = snapgpu.BaseAligner(idx)
    for use_m in (0, 1):
        whole = al.Cigars(reads, loc, dirs, useM=use_m)
        for s, c in ((1000, 37), (0, 3000), (2999, 1), (5, reads.n - 5), (123, 456)):
            part = al.Cigars(reads.slice(s, c), loc[s:s + c], dirs[s:s + c], useM=use_m)
            assert np.array_equal(part.editDistance, whole.editDistance[s:s + c])
            assert np.array_equal(part.nOps, whole.nOps[s:s + c])
            for j in range(c):   # snapgpu_cigar_batch writes each row's first nOps entries
                k = int(part.nOps[j])
                assert np.array_equal(part.ops[j, :k], whole.ops[s + j, :k])


@pytest.mark.gpu
def test_gpu_resident_cigars_ordered_before_next_run(gpu_available, small_world):
    """run(); run_cigars(); run(); cigars() on one resident batch: the CIGAR kernel reads
    the batch's records on the aligner's side stream, and the second run's 0xff pre-fill and passes
    rewrite those records on the lane streams -- the lanes wait for the side stream's CIGAR first, so
    the CIGARs equal those of a clean run() / run_cigars() / cigars() sequence, repeated 3 times."""
    idx, reads = small_world["index"], small_world["reads"]
    al = snapgpu.BaseAligner(idx)
    clean = al.upload(reads)
    clean.run()
    clean.run_cigars()
    want, want_res = clean.cigars(), clean.results()
    dev = al.upload(reads)
    for _ in range(3):
        dev.run()
        dev.run_cigars()
        dev.run()
        got = dev.cigars()
        assert np.array_equal(got.editDistance, want.editDistance)
        assert np.array_equal(got.nOps, want.nOps)
        for j in range(reads.n):
            k = int(want.nOps[j])
            assert np.array_equal(got.ops[j, :k], want.ops[j, :k]), j
        assert mismatches(dev.results(), want_res).size == 0
