#!/bin/bash
# A/B of the forced-mode prune (libsnapgpu.so vs libsnapgpu_noprune.so): C2 bench (2 rounds,
# alternating) and C3 resident runs on one shared index.
mkdir -p gpurun_out
export SNAPGPU_TIMEOUT_S=120
L=$PWD/snap-rnaseq_amd/snapgpu
for i in 1 2; do
  for v in libsnapgpu.so libsnapgpu_noprune.so; do
    SNAPGPU_LIB=$L/$v timeout -k 10 200 python bench.py --steps 20 --no-cpu-baseline --no-extras > gpurun_out/abp_${v}_$i.json 2>/dev/null || exit $?
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/abp_${v}_$i.json').readline()); print('C2 $v', round(d['value']/1e6,3), 'M reads/s', round(d['ms_per_step'],2), 'ms')"
  done
done
df -h /dev/shm | tail -1
timeout -k 10 400 python -u tools/ab_c3.py build || exit $?
for i in 1 2; do
  for v in libsnapgpu.so libsnapgpu_noprune.so; do
    SNAPGPU_LIB=$L/$v timeout -k 10 300 python -u tools/ab_c3.py run || { rm -f /dev/shm/snapgpu_ab_c3.bin; exit 1; }
  done
done
rm -f /dev/shm/snapgpu_ab_c3.bin
