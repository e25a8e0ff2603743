#!/bin/bash
# Round evidence on one box: GPU suite, default bench line (C2, extras, CPU baseline), the
# rocprofv3 passes (tools/gpu/prof.sh), then the C3 per-GPU-shard bench line.
#   gpurun -- bash tools/gpu/final.sh <profile-tag>
mkdir -p gpurun_out
export SNAPGPU_TIMEOUT_S=90
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -20 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
python3 -c "import json; d=json.loads(open('gpurun_out/bench.json').readline()); print('bench', round(d['value']/1e6,3), 'M reads/s')"
bash tools/gpu/prof.sh ${1:-r03} || exit $?
timeout -k 10 600 python bench.py --workload c3 --steps 5 --warmup 1 --paired-pairs 0 --rna-pairs 0 > gpurun_out/c3_bench.json 2> gpurun_out/c3_bench.err || exit $?
python3 -c "import json; d=json.loads(open('gpurun_out/c3_bench.json').readline()); print('c3', round(d['value']/1e6,3), 'M reads/s')"
