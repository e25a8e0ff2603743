#!/bin/bash
# round-3 check: new GPU tests, the whole GPU suite, VALU issue rates, default bench line
mkdir -p gpurun_out/r03b
export SNAPGPU_TIMEOUT_S=90
timeout -k 10 400 python -u -m pytest tests/test_rna_paired.py tests/test_watchdog.py -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/r03b/new_tests.log 2>&1 || { tail -30 gpurun_out/r03b/new_tests.log; exit 1; }
tail -8 gpurun_out/r03b/new_tests.log
timeout -k 10 120 ./tools/gpu/valu_rates > gpurun_out/r03b/valu_rates.json 2>&1 || { cat gpurun_out/r03b/valu_rates.json; exit 1; }
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r03b/gpu_tests.log 2>&1 || { tail -30 gpurun_out/r03b/gpu_tests.log; exit 1; }
tail -2 gpurun_out/r03b/gpu_tests.log
timeout -k 10 400 python bench.py > gpurun_out/r03b/bench.json 2> gpurun_out/r03b/bench.err || { tail -20 gpurun_out/r03b/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/r03b/bench.json').readline()); print('bench', round(d['value']/1e6,3), 'M reads/s; rna', d['rna_paired']['value']/1e6, d['rna_paired']['parity'])"
