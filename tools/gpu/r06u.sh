#!/bin/bash
# snap-rna single: the sub-batch writer thread (GPU tests of the single path, then the bench's
# single_e2e leg at 2 and 4 sub-batches (500k, 250k reads each)) -> gpurun_out/r06u/
export TMPDIR=/tmp SNAPGPU_TIMEOUT_S=120
O=gpurun_out/r06u; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_single.py tests/test_sorted.py tests/test_contamination.py -x -v -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for sb in 500000 250000 500000 250000; do
  SNAPGPU_SINGLE_SUBBATCH=$sb timeout -k 10 400 python bench.py --steps 2 --warmup 1 --rna-pairs 0 --paired-pairs 0 --no-cpu-baseline > $O/bench_sb$sb.json 2> $O/bench_sb$sb.err || { tail $O/bench_sb$sb.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bench_sb$sb.json').readline()); s=d['single_e2e']; print('sb', $sb, round(s['value']/1e6,3), s['parity'].get('sha256_match'), s['stage_ms'])"
done
