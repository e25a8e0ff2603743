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
