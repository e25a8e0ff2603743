#!/bin/bash
# Round 6 final evidence, one box: the GPU suite, smoke(), the default bench line, the C3 line and a
# 2-rank launch sharing the GPU (the N-rank path: self-launch, one index build per node, host thread
# budget per rank) -> gpurun_out/<tag>/.
#   gpurun -- bash tools/gpu/final_r06.sh <tag>
export TMPDIR=/tmp SNAPGPU_TIMEOUT_S=120
T=${1:?tag}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench.json').readline()); print('bench', round(d['value']/1e6,3), 'M reads/s; kernel', round(d['roofline']['kernel_ms_per_launch'],3), 'ms/launch; single', round(d['single_e2e']['value']/1e6,3), d['single_e2e']['parity'].get('sha256_match'), 'paired', round(d['paired']['value']/1e6,3), 'rna', round(d['rna_paired']['value']/1e6,3), d['rna_paired']['parity'].get('sha256_match'))"
timeout -k 10 900 python bench.py --workload c3 --steps 5 --warmup 1 --rna-pairs 0 --single-reads 0 > $O/c3_bench.json 2> $O/c3_bench.err || { tail $O/c3_bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/c3_bench.json').readline()); print('c3', round(d['value']/1e6,3), 'M reads/s; upload', d['config']['index_upload_s'], 's; paired', round(d['paired']['value']/1e6,3))"
timeout -k 10 600 python bench.py --gpus 2 --steps 5 --warmup 1 --no-cpu-baseline --paired-pairs 0 --rna-pairs 0 --single-reads 0 > $O/bench_g2.json 2> $O/bench_g2.err || { tail -20 $O/bench_g2.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench_g2.json').readline()); print('g2 n_gpus', d['n_gpus'], 'value', round(d['value']/1e6,3), [(r['rank'], round(r['reads_per_s']/1e6,3), r['index_upload_s'], r['index_built_here'], r['index_attached']) for r in d['config']['per_rank']])"
