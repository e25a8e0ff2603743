#!/bin/bash
# Development check on one box: the whole GPU suite, a short headline bench (no extras),
# then the RNA-path stage probe.  gpurun -- bash tools/gpu/check.sh
mkdir -p gpurun_out
export SNAPGPU_TIMEOUT_S=90
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline --no-extras > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err || exit $?
python3 -c "import json; d=json.loads(open('gpurun_out/bench_quick.json').readline()); print('bench', round(d['value']/1e6,3), 'M reads/s', round(d['ms_per_step'],2), 'ms/step')"
timeout -k 10 400 python -u tools/rna_probe.py > gpurun_out/rna_probe.log 2>&1 || exit $?
tail -1 gpurun_out/rna_probe.log
