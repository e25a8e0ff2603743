#!/bin/bash
# round 3: whole GPU suite on the pass-0 read routing, C2 A/B vs round-2 base, <256> workload probe
mkdir -p gpurun_out/r03e
export SNAPGPU_TIMEOUT_S=90
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r03e/gpu_tests.log 2>&1 || { tail -40 gpurun_out/r03e/gpu_tests.log; exit 1; }
tail -2 gpurun_out/r03e/gpu_tests.log
bash tools/gpu/abx.sh r03e 2 cur base || exit 1
timeout -k 10 400 python tools/probe256.py > gpurun_out/r03e/probe256.txt 2> gpurun_out/r03e/probe256.err || { tail -5 gpurun_out/r03e/probe256.err; exit 1; }
cat gpurun_out/r03e/probe256.txt
