#!/bin/bash
# Round 6: the whole GPU suite on the tree with the pass-wide match probabilities adopted, then the
# single-end leg with the mapped record write -> gpurun_out/r06f/.
export TMPDIR=/tmp SNAPGPU_TIMEOUT_S=120
O=gpurun_out/r06f; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 600 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --paired-pairs 0 --rna-pairs 0 > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench.json').readline()); s=d['single_e2e']; print('bench', round(d['value']/1e6,3), 'single', round(s['value']/1e6,3), s['stage_ms'], s['parity'].get('sha256_match'))"
