#!/bin/bash
# GPU-box driver: parity tests, then (only if they did not crash/hang) a short bench.
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py -q -m gpu -rf > gpurun_out/t2.log 2>&1
rc=$?; echo "EXIT $rc" >> gpurun_out/t2.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 3 --warmup 1 > gpurun_out/b1.log 2>&1
rc=$?; echo "EXIT $rc" >> gpurun_out/b1.log
exit $rc
