#!/bin/bash
# Round 6: the single-end leg's record output, mapped file vs one fwrite (SNAPGPU_SAM_WRITE), with the
# stage sub-timers, alternating -> gpurun_out/r06h/.
export TMPDIR=/tmp SNAPGPU_TIMEOUT_S=120
O=gpurun_out/r06h; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_single.py tests/test_sorted.py tests/test_contamination.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  for w in mmap fwrite; do
    SNAPGPU_SAM_WRITE=$w timeout -k 10 600 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --paired-pairs 0 --rna-pairs 0 \
      > $O/bench_${w}_$i.json 2> $O/bench_${w}_$i.err || { tail $O/bench_${w}_$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/bench_${w}_$i.json').readline()); s=d['single_e2e']; print('$w', round(s['value']/1e6,3), s['stage_ms'], s['parity'].get('sha256_match'))"
  done
done
