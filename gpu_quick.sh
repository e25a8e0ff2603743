#!/bin/bash
# GPU-box iteration step: parity tests, then (only if green) phase probe and bench.
mkdir -p gpurun_out
export SNAPGPU_TIMEOUT_S=${SNAPGPU_TIMEOUT_S:-90}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1
rc=$?; echo "EXIT $rc" >> gpurun_out/t.log; [ $rc -ne 0 ] && exit $rc
SNAPGPU_PHASES=1 timeout -k 10 300 python tools/phase_probe.py > gpurun_out/phase.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 3 --warmup 1 ${BENCH_ARGS:---no-cpu-baseline} > gpurun_out/bp.log 2>&1
