#!/bin/bash
# multi-hit / windowed parity on the GPU, then the full GPU suite, then A/B vs base
mkdir -p gpurun_out
export SNAPGPU_TIMEOUT_S=90
timeout -k 10 300 python -u -m pytest tests/test_multihit.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/mh.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1 || exit $?
bash tools/ab.sh > gpurun_out/ab.log 2>&1
