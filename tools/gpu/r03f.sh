#!/bin/bash
# round 3: VALU rates (VCC select variants), C2 A/B (3 rounds) and C3 A/B of cur / nosk / base
mkdir -p gpurun_out/r03f
export SNAPGPU_TIMEOUT_S=90
timeout -k 10 120 ./tools/gpu/valu_rates > gpurun_out/r03f/valu_rates.json 2>&1 || { cat gpurun_out/r03f/valu_rates.json; exit 1; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_golden.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r03f/golden.log 2>&1 || { tail -30 gpurun_out/r03f/golden.log; exit 1; }
tail -1 gpurun_out/r03f/golden.log
bash tools/gpu/abx.sh r03f 3 cur nosk base || exit 1
timeout -k 10 300 python tools/ab_c3.py build > gpurun_out/r03f/c3_build.log 2>&1 || { tail -5 gpurun_out/r03f/c3_build.log; exit 1; }
L=$PWD/snap-rnaseq_amd/snapgpu
for i in 1 2; do for v in base cur nosk; do
  if [ $v = cur ]; then lib=$L/libsnapgpu.so; else lib=$L/libsnapgpu_$v.so; fi
  SNAPGPU_LIB=$lib timeout -k 10 200 python tools/ab_c3.py run /dev/shm/snapgpu_ab_c3.bin 1000000 >> gpurun_out/r03f/c3_ab.log 2>&1 || { tail -5 gpurun_out/r03f/c3_ab.log; rm -f /dev/shm/snapgpu_ab_c3.bin; exit 1; }
done; done
rm -f /dev/shm/snapgpu_ab_c3.bin
cat gpurun_out/r03f/c3_ab.log
