#!/bin/bash
# Working tree vs libsnapgpu_base.so: parity tests, exact VALU count per read (PMC), C2 bench A/B.
mkdir -p gpurun_out
export SNAPGPU_TIMEOUT_S=120 TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_long_reads.py tests/test_ref_index.py tests/test_multihit.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/abv_tests.log 2>&1 || { tail -30 gpurun_out/abv_tests.log; exit 1; }
tail -1 gpurun_out/abv_tests.log
bash tools/gpu/valu_attr.sh libsnapgpu.so libsnapgpu_base.so | tail -2 || exit 1
L=$PWD/snap-rnaseq_amd/snapgpu
for i in 1 2 3; do
  for v in libsnapgpu.so libsnapgpu_base.so; do
    SNAPGPU_LIB=$L/$v timeout -k 10 200 python bench.py --steps 20 --no-cpu-baseline --no-extras > gpurun_out/abv_${v}_$i.json 2>/dev/null || exit $?
    python3 -c "import json; d=json.loads(open('gpurun_out/abv_${v}_$i.json').readline()); print('C2 $v', round(d['value']/1e6,3), 'M reads/s busy', round(d['roofline']['kernel_busy_ms_per_step'],2))"
  done
done
