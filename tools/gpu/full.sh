#!/bin/bash
# Round-end style evidence: GPU test suite, the default bench line (with CPU baseline),
# then the rocprofv3 passes (tools/gpu/prof.sh).  Run from the repo root:
#   gpurun -- bash tools/gpu/full.sh <profile-tag>
mkdir -p gpurun_out
export SNAPGPU_TIMEOUT_S=90
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
bash tools/gpu/prof.sh ${1:-r01}
