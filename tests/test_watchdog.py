"""Device watchdog isolation: every aligner owns its watchdog record (KArgs::diag),
so two aligners on one device -- the RNA paired path's transcriptome and genome aligners run
on two host threads (csrc/host/rna_paired.cpp) -- neither clear nor trip each other's record.
snapgpu_aligner_debug_trip makes one aligner's kernel report a trip at a chosen read."""
import threading

import numpy as np
import pytest

import snapgpu


@pytest.mark.gpu
def test_watchdog_trip_stays_in_its_aligner(gpu_available, small_world):
    idx = small_world["index"]
    reads = snapgpu.Reads.synthetic(small_world["genome"], 60_000, seed=123, random_read_fraction=0.01)
    a = snapgpu.BaseAligner(idx, device=0)
    b = snapgpu.BaseAligner(idx, device=0)
    want = b.AlignReads(reads)
    a.debug_trip(5)
    err, outs = {}, []

    def run_a():
        for _ in range(4):
            try:
                a.AlignReads(reads)
                err.setdefault("a", []).append(None)
            except snapgpu.SnapGpuError as e:
                err.setdefault("a", []).append(str(e))

    def run_b():
        for _ in range(4):
            outs.append(b.AlignReads(reads))

    ta, tb = threading.Thread(target=run_a), threading.Thread(target=run_b)
    ta.start(); tb.start()
    ta.join(120); tb.join(120)
    assert not ta.is_alive() and not tb.is_alive()
    # every call of the tripped aligner fails with its own record (code 6 = DIAG_TEST_TRIP, read 5)
    assert len(err["a"]) == 4 and all(e and "watchdog" in e and "code 6 read 5" in e for e in err["a"]), err
    # the other aligner's calls, overlapping them on the same device, are untouched
    assert len(outs) == 4
    for o in outs:
        assert np.array_equal(o.view(np.uint8), want.view(np.uint8))
    # the record is cleared per call: with the hook off the tripped aligner aligns normally again
    a.debug_trip(0xffffffff)
    assert np.array_equal(a.AlignReads(reads).view(np.uint8), want.view(np.uint8))
