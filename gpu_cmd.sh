#!/bin/bash
# GPU-box driver: parity tests, then (only if they passed) a short bench with the
# grouped scorer and with the one-candidate scorer for comparison.
mkdir -p gpurun_out
export SNAPGPU_TIMEOUT_S=${SNAPGPU_TIMEOUT_S:-90}
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py -x -q -m gpu -rf > gpurun_out/t2.log 2>&1
rc=$?; echo "EXIT $rc" >> gpurun_out/t2.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 3 --warmup 1 > gpurun_out/b1.log 2>&1
rc=$?; echo "EXIT $rc" >> gpurun_out/b1.log
[ $rc -ne 0 ] && exit $rc
SNAPGPU_GROUPED=0 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/b0.log 2>&1
rc=$?; echo "EXIT $rc" >> gpurun_out/b0.log
exit $rc
