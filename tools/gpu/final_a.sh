#!/bin/bash
# Round evidence, part A (one box): GPU suite, smoke, default bench line (C2, extras, CPU baseline),
# the C3 per-GPU-shard bench line.  Part B (tools/gpu/prof.sh <tag>) is the rocprofv3 passes.
mkdir -p gpurun_out
export SNAPGPU_TIMEOUT_S=90
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -20 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
python3 -c "import json; d=json.loads(open('gpurun_out/bench.json').readline()); print('bench', round(d['value']/1e6,3), 'M reads/s', 'rna', round(d['rna_paired']['value']/1e6,3))"
timeout -k 10 600 python bench.py --workload c3 --steps 5 --warmup 1 --paired-pairs 0 --rna-pairs 0 > gpurun_out/c3_bench.json 2> gpurun_out/c3_bench.err || exit $?
python3 -c "import json; d=json.loads(open('gpurun_out/c3_bench.json').readline()); print('c3', round(d['value']/1e6,3), 'M reads/s')"
