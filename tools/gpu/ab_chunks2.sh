#!/bin/bash
# d1-boundary bench (stream mode) over chunk sizes, 2 alternating rounds (bench only).
mkdir -p gpurun_out
for i in 1 2; do
  for c in 500000 1000000 333334 262144; do
    SNAPGPU_CHUNK_READS=$c timeout -k 10 120 python bench.py --steps 20 --no-cpu-baseline --no-extras > gpurun_out/abc2_${c}_$i.json 2>/dev/null || exit $?
    python3 -c "import json; d=json.loads(open('gpurun_out/abc2_${c}_$i.json').readline()); r=d['roofline']; print('chunk $c', round(d['value']/1e6,3), 'M reads/s', round(d['ms_per_step'],2), 'ms/step busy', round(r['kernel_busy_ms_per_step'],2))"
  done
done
