#!/bin/bash
# Round 5: the GPU suite on the HBM chain-head build, then C2 A/B against the previous build (prev).
export TMPDIR=/tmp SNAPGPU_TIMEOUT_S=90
O=gpurun_out/r05r; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
bash tools/gpu/ab_pmc.sh r05r_ab prev
