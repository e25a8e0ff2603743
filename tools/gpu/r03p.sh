#!/bin/bash
# GPU suite (incl. the contamination-database tests), then the rocprofv3 passes of this build
mkdir -p gpurun_out
export SNAPGPU_TIMEOUT_S=90
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
bash tools/gpu/prof.sh r03
