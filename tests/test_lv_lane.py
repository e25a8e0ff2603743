"""The per-lane Landau-Vishkin distance of the forced-mode prefilter (snap-rnaseq_amd/csrc/lv_lane.h)
against the oracle's LandauVishkin restatement (oracle/snap_oracle.c oracle_lv, itself pinned to the
reference's LV vectors by test_oracle_golden.py): tests/c/lv_lane_test.cpp, built with hipcc as host
code, checks ~1.6M forward and reverse calls (every k <= KM) bit for bit on the CPU."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def test_lane_lv_distance_matches_oracle(tmp_path):
    from oracle_ffi import ORACLE_SO, oracle_lib
    oracle_lib()   # builds oracle/liboracle.so when missing
    exe = tmp_path / "lv_lane_test"
    odir = os.path.dirname(ORACLE_SO)
    subprocess.run(["/opt/rocm/bin/hipcc", "-O2", "-I", os.path.join(ROOT, "snap-rnaseq_amd", "csrc"),
                    os.path.join(HERE, "c", "lv_lane_test.cpp"), "-o", str(exe), "-L", odir, "-loracle",
                    "-Wl,-rpath," + odir], check=True, capture_output=True)
    out = subprocess.run([str(exe), "200000"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0 and " 0 mismatches" in out.stdout, out.stdout[-2000:]
