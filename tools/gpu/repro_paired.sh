#!/bin/bash
# Repeated intersecting-aligner calls (tools/paired_repro.py) after one failure of
# test_gpu_intersecting_matches_reference_and_oracle[tight] in a full-suite run (r04p, first attempt).
mkdir -p gpurun_out/repro && export SNAPGPU_TIMEOUT_S=60 && timeout -k 10 300 python -u tools/paired_repro.py 8 3 tight > gpurun_out/repro/tight.log 2>&1 && timeout -k 10 300 python -u tools/paired_repro.py 4 3 default > gpurun_out/repro/default.log 2>&1; tail -3 gpurun_out/repro/tight.log; tail -3 gpurun_out/repro/default.log
