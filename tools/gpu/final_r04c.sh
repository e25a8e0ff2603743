#!/bin/bash
# Round-4 evidence on the 5-waves build (ELCAP 6, forced-order window 128, -structurizecfg-skip-uniform-regions):
# the wave-history tests, the GPU suite, smoke, the default bench line and the C3 line with its paired shard.
export TMPDIR=/tmp SNAPGPU_TIMEOUT_S=90
O=gpurun_out/final_r04c; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_paired.py -v -m gpu -k independent --timeout 300 --timeout-method thread > $O/history_tests.log 2>&1 || { tail -30 $O/history_tests.log; exit 1; }
grep -E "PASSED|FAILED" $O/history_tests.log
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench.json').readline()); print('bench', round(d['value']/1e6,3), 'M reads/s', 'kernel', round(d['roofline']['kernel_ms_per_launch'],2), 'paired', round(d['paired']['value']/1e6,3), 'rna', round(d['rna_paired']['value']/1e6,3))"
timeout -k 10 900 python bench.py --workload c3 --steps 5 --warmup 1 --rna-pairs 0 > $O/c3_bench.json 2> $O/c3_bench.err || { tail $O/c3_bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/c3_bench.json').readline()); print('c3', round(d['value']/1e6,3), 'M reads/s', 'paired', round(d['paired']['value']/1e6,3))"
