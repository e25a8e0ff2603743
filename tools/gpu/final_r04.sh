#!/bin/bash
# Round-4 evidence, part A (one box): GPU suite, smoke, the default bench line (C2, extras, CPU
# baseline) and the C3 per-GPU-shard line with configs[3]'s paired shard (3,125,000 2x101 pairs).
# Part B is tools/gpu/prof.sh r04 (rocprofv3 passes).
export TMPDIR=/tmp SNAPGPU_TIMEOUT_S=90
O=gpurun_out/final_r04; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -20 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench.json').readline()); print('bench', round(d['value']/1e6,3), 'M reads/s', 'paired', round(d['paired']['value']/1e6,3), 'rna', round(d['rna_paired']['value']/1e6,3))"
timeout -k 10 900 python bench.py --workload c3 --steps 5 --warmup 1 --rna-pairs 0 > $O/c3_bench.json 2> $O/c3_bench.err || { tail $O/c3_bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/c3_bench.json').readline()); print('c3', round(d['value']/1e6,3), 'M reads/s', 'paired', round(d['paired']['value']/1e6,3))"
