#!/bin/bash
# whole GPU suite on the working build (maxSeeds table, 12-B plane loads, no streaming-load switch), then
# C2 A/B head / npf / tbl (= working build) x2 and C3 digests
mkdir -p gpurun_out/r03l
export SNAPGPU_TIMEOUT_S=90
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r03l/gpu_tests.log 2>&1 || { tail -30 gpurun_out/r03l/gpu_tests.log; exit 1; }
tail -1 gpurun_out/r03l/gpu_tests.log
bash tools/gpu/abx.sh r03l 2 head npf tbl || exit 1
timeout -k 10 300 python tools/ab_c3.py build > gpurun_out/r03l/c3_build.log 2>&1 || { tail -5 gpurun_out/r03l/c3_build.log; exit 1; }
L=$PWD/snap-rnaseq_amd/snapgpu
for i in 1 2; do for v in head npf tbl; do
  SNAPGPU_LIB=$L/libsnapgpu_$v.so timeout -k 10 200 python tools/ab_c3.py run /dev/shm/snapgpu_ab_c3.bin 1000000 >> gpurun_out/r03l/c3_ab.log 2>&1 || { tail -5 gpurun_out/r03l/c3_ab.log; rm -f /dev/shm/snapgpu_ab_c3.bin; exit 1; }
done; done
rm -f /dev/shm/snapgpu_ab_c3.bin
cat gpurun_out/r03l/c3_ab.log
