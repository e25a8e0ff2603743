#!/bin/bash
# Round-4 evidence on the last build: the wave-history tests, the GPU suite, then the rocprofv3
# passes (tools/gpu/prof.sh r04) whose PMC data bench.py reports for this library.
export TMPDIR=/tmp SNAPGPU_TIMEOUT_S=90
O=gpurun_out/final_r04b; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_paired.py -v -m gpu -k independent --timeout 300 --timeout-method thread > $O/history_tests.log 2>&1 || { tail -30 $O/history_tests.log; exit 1; }
grep -E "PASSED|FAILED" $O/history_tests.log
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
bash tools/gpu/prof.sh r04
