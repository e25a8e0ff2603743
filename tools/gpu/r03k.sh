#!/bin/bash
# A/B: head (round-3 commit before the micro-opts), rsk (DPP scan + forced-batch prefetch + 16-seed pass 0 +
# radix digit skip = working tree), npf (rsk without the forced-batch prefetch); C2 x3, C3 x2
mkdir -p gpurun_out/r03k
bash tools/gpu/abx.sh r03k 3 head rsk npf || exit 1
timeout -k 10 300 python tools/ab_c3.py build > gpurun_out/r03k/c3_build.log 2>&1 || { tail -5 gpurun_out/r03k/c3_build.log; exit 1; }
L=$PWD/snap-rnaseq_amd/snapgpu
for i in 1 2; do for v in head rsk npf; do
  SNAPGPU_LIB=$L/libsnapgpu_$v.so timeout -k 10 200 python tools/ab_c3.py run /dev/shm/snapgpu_ab_c3.bin 1000000 >> gpurun_out/r03k/c3_ab.log 2>&1 || { tail -5 gpurun_out/r03k/c3_ab.log; rm -f /dev/shm/snapgpu_ab_c3.bin; exit 1; }
done; done
rm -f /dev/shm/snapgpu_ab_c3.bin
cat gpurun_out/r03k/c3_ab.log
