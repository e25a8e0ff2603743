#!/bin/bash
# Round 4: forced-mode radix threshold (SNAPGPU_RADIX_MIN) now that the ranked window is 128 entries:
# 257 (default) / 129 / 65 on C3 (tools/ab_c3.py, shared index, 1M reads, records digest) and C2 (bench),
# same library, alternating.
export TMPDIR=/tmp SNAPGPU_TIMEOUT_S=120
O=gpurun_out/r04u; mkdir -p $O
timeout -k 10 400 python -u tools/ab_c3.py build > $O/build.log 2>&1 || { tail $O/build.log; exit 1; }
for i in 1 2; do
  for rm in 257 129 65; do
    SNAPGPU_RADIX_MIN=$rm timeout -k 10 300 python -u tools/ab_c3.py run > $O/c3_${rm}_$i.log 2>&1 || { tail $O/c3_${rm}_$i.log; rm -f /dev/shm/snapgpu_ab_c3.bin; exit 1; }
    echo "C3 radixMin $rm: $(tail -1 $O/c3_${rm}_$i.log)"
  done
done
rm -f /dev/shm/snapgpu_ab_c3.bin
for i in 1 2; do
  for rm in 257 129 65; do
    SNAPGPU_RADIX_MIN=$rm timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extras > $O/c2_${rm}_$i.json 2> $O/c2_${rm}_$i.err || exit 1
    python3 -c "import json; d=json.loads(open('$O/c2_${rm}_$i.json').readline()); print('C2 radixMin $rm', round(d['value']/1e6,3), 'M reads/s kernel', round(d['roofline']['kernel_ms_per_launch'],2))"
  done
done
