#!/bin/bash
# Radix-sorted forced pops: parity with the radix path forced for every read (SNAPGPU_RADIX_MIN=1),
# then A/B against the previous build (libsnapgpu_base.so) on C2 (bench) and C3 (shared index).
mkdir -p gpurun_out
export SNAPGPU_TIMEOUT_S=120
L=$PWD/snap-rnaseq_amd/snapgpu
SNAPGPU_RADIX_MIN=1 timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_multihit.py tests/test_long_reads.py tests/test_ref_index.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/radix_tests.log 2>&1 || { tail -30 gpurun_out/radix_tests.log; exit 1; }
tail -1 gpurun_out/radix_tests.log
for i in 1 2; do
  for v in libsnapgpu.so libsnapgpu_base.so; do
    SNAPGPU_LIB=$L/$v timeout -k 10 200 python bench.py --steps 20 --no-cpu-baseline --no-extras > gpurun_out/abr_${v}_$i.json 2>/dev/null || exit $?
    python3 -c "import json; d=json.loads(open('gpurun_out/abr_${v}_$i.json').readline()); print('C2 $v', round(d['value']/1e6,3), 'M reads/s', round(d['ms_per_step'],2), 'ms')"
  done
done
timeout -k 10 400 python -u tools/ab_c3.py build || exit $?
for i in 1 2; do
  for v in libsnapgpu.so libsnapgpu_base.so; do
    SNAPGPU_LIB=$L/$v timeout -k 10 300 python -u tools/ab_c3.py run || { rm -f /dev/shm/snapgpu_ab_c3.bin; exit 1; }
  done
done
SNAPGPU_RADIX_MIN=1 SNAPGPU_LIB=$L/libsnapgpu.so timeout -k 10 300 python -u tools/ab_c3.py run
rm -f /dev/shm/snapgpu_ab_c3.bin
