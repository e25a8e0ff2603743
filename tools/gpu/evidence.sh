#!/bin/bash
# One box: the GPU suite, smoke(), the default bench line (C2, extras, CPU baseline) and, with a
# second argument `c3`, the C3 per-GPU-shard line.  Results in gpurun_out/<tag>/.
#   gpurun -- bash tools/gpu/evidence.sh <tag> [c3]
export TMPDIR=/tmp SNAPGPU_TIMEOUT_S=90
T=${1:?tag}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench.json').readline()); print('bench', round(d['value']/1e6,3), 'M reads/s; kernel', round(d['roofline']['kernel_ms_per_launch'],3), 'ms/launch; paired', round(d['paired']['value']/1e6,3), 'rna', round(d['rna_paired']['value']/1e6,3))"
if [ "$2" = c3 ]; then
  timeout -k 10 900 python bench.py --workload c3 --steps 5 --warmup 1 --rna-pairs 0 --single-reads 0 > $O/c3_bench.json 2> $O/c3_bench.err || { tail $O/c3_bench.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/c3_bench.json').readline()); print('c3', round(d['value']/1e6,3), 'M reads/s', 'paired', round(d['paired']['value']/1e6,3))"
fi
