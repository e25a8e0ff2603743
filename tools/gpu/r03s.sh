#!/bin/bash
# A/B of LDS mirror of the first 64 elements' candidatesUsed + header dword 11 for hit insertion (the pm/pa path slots shrunk to 32
# make room): GPU suite on the variant, then C2
# (3 alternating rounds) and C3 (2 rounds) against the current build, 2-rank self-launch rehearsal
mkdir -p gpurun_out/r03s
export SNAPGPU_TIMEOUT_S=90
L=$PWD/snap-rnaseq_amd/snapgpu
SNAPGPU_LIB=$L/libsnapgpu_hm.so timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r03s/gpu_tests_hm.log 2>&1 || { tail -30 gpurun_out/r03s/gpu_tests_hm.log; exit 1; }
tail -1 gpurun_out/r03s/gpu_tests_hm.log
bash tools/gpu/abx.sh r03s 3 cur hm || exit 1
timeout -k 10 300 python tools/ab_c3.py build > gpurun_out/r03s/c3_build.log 2>&1 || { tail -5 gpurun_out/r03s/c3_build.log; exit 1; }
for i in 1 2; do for v in cur hm; do
  if [ $v = cur ]; then lib=$L/libsnapgpu.so; else lib=$L/libsnapgpu_$v.so; fi
  SNAPGPU_LIB=$lib timeout -k 10 200 python tools/ab_c3.py run /dev/shm/snapgpu_ab_c3.bin 1000000 >> gpurun_out/r03s/c3_ab.log 2>&1 || { tail -5 gpurun_out/r03s/c3_ab.log; rm -f /dev/shm/snapgpu_ab_c3.bin; exit 1; }
done; done
rm -f /dev/shm/snapgpu_ab_c3.bin
cat gpurun_out/r03s/c3_ab.log
timeout -k 10 400 python -u tools/rna_probe.py > gpurun_out/r03s/rna_probe.log 2>&1 || exit $?; tail -1 gpurun_out/r03s/rna_probe.log
