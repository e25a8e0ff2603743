"""GPU edge cases of the boundary: empty batches through every entry point,
zero-length reads, and reads past maxReadSize, which the reference answers with soft_exit
(BaseAligner.cpp:609-613, IntersectingPairedEndAligner.cpp:211-215) and the C ABI with a per-read
flag (single end) or a status code (paired).  Expected values come from the oracle
(oracle/snap_oracle.c), bit-exact."""
import numpy as np
import pytest

import snapgpu
from oracle_ffi import mismatches, oracle_align

pytestmark = pytest.mark.gpu


def _edge_batch(genome):
    s = genome.bases(5000, 600).decode().upper()
    t = genome.bases(200_000, 300).decode().upper()
    return [("", ""), (s[:100], "I" * 100), (s[:501], "I" * 501), (s[:500], "5" * 500), ("A", "I"),
            ("", ""), (t[:150], "2" * 150), (t[:19], "I" * 19), (t[:20], "I" * 20), (s[:512], "I" * 512)]


def test_empty_batches(gpu_available, small_world):
    idx = small_world["index"]
    empty = snapgpu.Reads.from_list([])
    al = snapgpu.BaseAligner(idx)
    assert len(al.AlignReads(empty)) == 0
    out = np.zeros(0, dtype=snapgpu.RESULT_DTYPE)
    al.submit(empty, out)
    al.wait()
    dev = al.upload(empty)
    dev.run()
    assert len(dev.results()) == 0
    # the aligner still works after the empty calls
    part = small_world["reads"].slice(0, 300)
    got = al.AlignReads(part)
    assert len(mismatches(got, oracle_align(idx, part, al.params))) == 0
    pa = snapgpu.PairedAligner(idx)
    assert len(pa.align(empty, empty)) == 0
    assert len(pa.intersect(empty, empty)) == 0


def test_zero_length_and_too_long_reads_vs_oracle(gpu_available, small_world):
    idx = small_world["index"]
    reads = snapgpu.Reads.from_list(_edge_batch(small_world["genome"]))
    al = snapgpu.BaseAligner(idx)
    gpu = al.AlignReads(reads)
    cpu = oracle_align(idx, reads, al.params)
    bad = mismatches(gpu, cpu)
    assert len(bad) == 0, [(int(i), gpu[i], cpu[i]) for i in bad[:3]]
    lens = reads.lengths()
    too_long = lens > al.params.maxReadSize
    assert too_long.sum() == 2
    assert np.all((gpu["flags"][too_long] & 0x01) != 0)          # SNAPGPU_FLAG_READ_TOO_LONG
    assert np.all((gpu["flags"][~too_long] & 0x01) == 0)
    assert np.all(gpu["result"][lens < 20] == snapgpu.NotFound)
    assert gpu["result"][1] == snapgpu.SingleHit and gpu["location"][1] == 5000


def test_paired_read_past_max_read_size_is_a_status_code(gpu_available, small_world):
    """The reference exits the process; the C ABI returns an error status and the aligner stays usable."""
    idx, g = small_world["index"], small_world["genome"]
    s = g.bases(5000, 1200).decode().upper()
    ok0 = snapgpu.Reads.from_list([(s[:100], "I" * 100)])
    ok1 = snapgpu.Reads.from_list([(s[700:800], "I" * 100)])
    long0 = snapgpu.Reads.from_list([(s[:501], "I" * 501)])
    pa = snapgpu.PairedAligner(idx)
    with pytest.raises(Exception):
        pa.intersect(long0, ok1)
    got = pa.intersect(ok0, ok1)
    assert len(got) == 1


def test_nul_bytes_are_flagged_not_silent(gpu_available, small_world):
    """A read that reaches the device with 0x00 bytes (what a zero-fill racing an upload leaves behind)
    is aligned as the reference would align it -- 0x00 is a non-ACGT base -- but its record carries
    SNAPGPU_FLAG_NUL_BYTE (paired: SNAPGPU_PFLAG_NUL_BYTE), which every parity test asserts absent
    (oracle_ffi.assert_no_corrupt_reads).  Clean reads of the same batch stay unflagged."""
    from oracle_ffi import COMPARE_FIELDS, NUL_FLAG
    idx, g = small_world["index"], small_world["genome"]
    s = g.bases(5000, 1200).decode().upper()
    t = g.bases(200_000, 300).decode().upper()
    clean = [(s[:100], "I" * 100), (t[:100], "I" * 100)]
    holed = [(s[:40] + "\0" + s[41:100], "I" * 100), ("\0" * 100, "I" * 100), (t[:99] + "\0", "I" * 100)]
    reads = snapgpu.Reads.from_list(clean + holed)
    al = snapgpu.BaseAligner(idx)
    gpu = al.AlignReads(reads)
    cpu = oracle_align(idx, reads, al.params)
    for f in COMPARE_FIELDS:
        x, y = gpu[f], cpu[f]
        if x.dtype.kind == "f":
            x, y = x.view(np.uint64), y.view(np.uint64)
        assert np.array_equal(x, y), f
    assert list((gpu["flags"] & NUL_FLAG) != 0) == [False, False, True, True, True]
    assert al.timing()["nNulReads"] == 3 and al.timing()["nUnwritten"] == 0
    r0 = snapgpu.Reads.from_list([clean[0], holed[0]])
    r1 = snapgpu.Reads.from_list([(s[700:800], "I" * 100), (s[700:800], "I" * 100)])
    got = snapgpu.PairedAligner(idx).intersect(r0, r1)
    assert list((got["flags"] & snapgpu.PFLAG_NUL_BYTE) != 0) == [False, True]
    assert list(got["writtenBy"]) == [1, 1]


def test_stats_match_records_on_every_record_path(gpu_available, small_world):
    """Aligner.h:62-77's getters summed over the records: the stream path's host tail splits a
    1M-record chunk over host threads (aligner.hip finishChunk, per-thread sums in locals), the
    resident download sums on one thread (finishRecords); both must equal the records' own sums."""
    idx = small_world["index"]
    reads = snapgpu.Reads.synthetic(small_world["genome"], 200_000, seed=7, random_read_fraction=0.02)

    def want(res):
        return {"nHashTableLookups": int(res["nLookups"].astype(np.int64).sum()),
                "nLocationsScored": int(res["nLocationsScored"].astype(np.int64).sum()),
                "nHitsIgnoredBecauseOfTooHighPopularity": int(res["nHitsIgnored"].astype(np.int64).sum()),
                "nReadsIgnoredBecauseOfTooManyNs": int(((res["flags"] & snapgpu.FLAG_TOO_MANY_NS) != 0).sum())}

    a = snapgpu.BaseAligner(idx)
    res = a.AlignReads(reads)
    got = a.stats()
    for k, v in want(res).items():
        assert got[k] == v, (k, got[k], v)
    b = snapgpu.BaseAligner(idx)
    dev = b.upload(reads)
    dev.run()
    res2 = dev.results()
    assert np.array_equal(res.view(np.uint8), res2.view(np.uint8))
    got2 = b.stats()
    for k, v in want(res2).items():
        assert got2[k] == v, (k, got2[k], v)
