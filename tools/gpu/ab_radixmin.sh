#!/bin/bash
# Forced-mode radix threshold sweep (SNAPGPU_RADIX_MIN) on C2 (bench) and C3 (shared index),
# same library, alternating.
mkdir -p gpurun_out
export SNAPGPU_TIMEOUT_S=120
timeout -k 10 400 python -u tools/ab_c3.py build || exit $?
for i in 1 2; do
  for rm in 257 129 65; do
    echo "radixMin $rm"
    SNAPGPU_RADIX_MIN=$rm timeout -k 10 300 python -u tools/ab_c3.py run || { rm -f /dev/shm/snapgpu_ab_c3.bin; exit 1; }
  done
done
rm -f /dev/shm/snapgpu_ab_c3.bin
for i in 1 2; do
  for rm in 257 129 65; do
    SNAPGPU_RADIX_MIN=$rm timeout -k 10 200 python bench.py --steps 20 --no-cpu-baseline --no-extras > gpurun_out/abm_${rm}_$i.json 2>/dev/null || exit $?
    python3 -c "import json; d=json.loads(open('gpurun_out/abm_${rm}_$i.json').readline()); print('C2 radixMin $rm', round(d['value']/1e6,3), 'M reads/s', round(d['ms_per_step'],2), 'ms')"
  done
done
