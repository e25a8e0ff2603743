#!/bin/bash
# occupancy experiment: align_kernel<128> at 5 waves/SIMD (SKCAP = MIRCAP = 64 to fit 8 KB LDS; 96 VGPRs,
# 72 B/lane scratch) against the same caps at 4 waves (cap64) and the current build; C2 bench + C3 digests
mkdir -p gpurun_out/r03i
bash tools/gpu/abx.sh r03i 2 cur w5 cap64 || exit 1
timeout -k 10 300 python tools/ab_c3.py build > gpurun_out/r03i/c3_build.log 2>&1 || { tail -5 gpurun_out/r03i/c3_build.log; exit 1; }
L=$PWD/snap-rnaseq_amd/snapgpu
for v in cur w5 cap64; do
  if [ $v = cur ]; then lib=$L/libsnapgpu.so; else lib=$L/libsnapgpu_$v.so; fi
  SNAPGPU_LIB=$lib timeout -k 10 200 python tools/ab_c3.py run /dev/shm/snapgpu_ab_c3.bin 1000000 >> gpurun_out/r03i/c3_ab.log 2>&1 || { tail -5 gpurun_out/r03i/c3_ab.log; rm -f /dev/shm/snapgpu_ab_c3.bin; exit 1; }
done
rm -f /dev/shm/snapgpu_ab_c3.bin
cat gpurun_out/r03i/c3_ab.log
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03i/lk -o run --output-format csv -- python3 tools/lookup_probe.py > gpurun_out/r03i/lookup_probe.txt 2>&1 || { tail -5 gpurun_out/r03i/lookup_probe.txt; exit 1; }
cat gpurun_out/r03i/lookup_probe.txt | grep run
grep seed_lookup gpurun_out/r03i/lk/run_kernel_stats.csv
