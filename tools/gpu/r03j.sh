#!/bin/bash
# micro-optimisation A/B: head (committed), scan (DPP scan in lv_prob_pair), pf (scan + next-batch
# prefetch in forced mode); C2 bench x3 rounds, C3 resident with record digests; then the GPU parity
# tests on the pf build (the working tree's libsnapgpu.so)
mkdir -p gpurun_out/r03j
export SNAPGPU_TIMEOUT_S=90
timeout -k 10 600 python -u -m pytest tests/test_gpu_golden.py tests/test_gpu_parity.py tests/test_multihit.py tests/test_ref_index.py tests/test_long_reads.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r03j/tests.log 2>&1 || { tail -30 gpurun_out/r03j/tests.log; exit 1; }
tail -1 gpurun_out/r03j/tests.log
bash tools/gpu/abx.sh r03j 2 head pf s16 rsk || exit 1
timeout -k 10 300 python tools/ab_c3.py build > gpurun_out/r03j/c3_build.log 2>&1 || { tail -5 gpurun_out/r03j/c3_build.log; exit 1; }
L=$PWD/snap-rnaseq_amd/snapgpu
for i in 1 2; do for v in head s16 rsk; do
  SNAPGPU_LIB=$L/libsnapgpu_$v.so timeout -k 10 200 python tools/ab_c3.py run /dev/shm/snapgpu_ab_c3.bin 1000000 >> gpurun_out/r03j/c3_ab.log 2>&1 || { tail -5 gpurun_out/r03j/c3_ab.log; rm -f /dev/shm/snapgpu_ab_c3.bin; exit 1; }
done; done
rm -f /dev/shm/snapgpu_ab_c3.bin
cat gpurun_out/r03j/c3_ab.log
