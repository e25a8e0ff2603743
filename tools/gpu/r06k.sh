#!/bin/bash
# Round 6: the pipelined snap-rna single path (sub-batches, parked pinned buffers): its GPU tests and
# two bench runs of the single leg -> gpurun_out/r06k/.
export TMPDIR=/tmp SNAPGPU_TIMEOUT_S=120
O=gpurun_out/r06k; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_single.py tests/test_sorted.py tests/test_contamination.py tests/test_cigar.py -x -v -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  timeout -k 10 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --paired-pairs 0 --rna-pairs 0 > $O/bench_$i.json 2> $O/bench_$i.err || { tail $O/bench_$i.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bench_$i.json').readline()); s=d['single_e2e']; print('bench', round(d['value']/1e6,3), round(d['roofline']['kernel_ms_per_launch'],3), 'single', round(s['value']/1e6,3), s['stage_ms'], s['aligners'], s['parity'].get('sha256_match'))"
done
