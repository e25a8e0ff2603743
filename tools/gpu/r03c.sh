#!/bin/bash
# round 3: new GPU tests (RNA 2x150 SAM + BAM, watchdog isolation, C1/C2 reference digests, parity),
# VALU issue rates, C2 A/B of the element-store / sort-key / streaming-load builds
mkdir -p gpurun_out/r03c
export SNAPGPU_TIMEOUT_S=90
timeout -k 10 600 python -u -m pytest tests/test_gpu_golden.py tests/test_gpu_parity.py tests/test_long_reads.py tests/test_multihit.py tests/test_rna_paired.py -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/r03c/new_tests.log 2>&1 || { tail -40 gpurun_out/r03c/new_tests.log; exit 1; }
tail -4 gpurun_out/r03c/new_tests.log
timeout -k 10 120 ./tools/gpu/valu_rates > gpurun_out/r03c/valu_rates.json 2>&1 || { cat gpurun_out/r03c/valu_rates.json; exit 1; }
bash tools/gpu/abx.sh r03c 2 cur base curnt || exit 1
