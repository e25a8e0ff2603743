#!/bin/bash
# Parity of the working-tree build (GPU LV + parity + golden tests), then C2 bench A/B against
# libsnapgpu_base.so (tools/build_base.sh), two alternating rounds.
mkdir -p gpurun_out
export SNAPGPU_TIMEOUT_S=120
L=$PWD/snap-rnaseq_amd/snapgpu
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_long_reads.py tests/test_ref_index.py tests/test_multihit.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/abb_tests.log 2>&1 || { tail -30 gpurun_out/abb_tests.log; exit 1; }
tail -1 gpurun_out/abb_tests.log
for i in 1 2 3; do
  for v in libsnapgpu.so libsnapgpu_base.so; do
    SNAPGPU_LIB=$L/$v timeout -k 10 200 python bench.py --steps 20 --no-cpu-baseline --no-extras > gpurun_out/abb_${v}_$i.json 2>/dev/null || exit $?
    python3 -c "import json; d=json.loads(open('gpurun_out/abb_${v}_$i.json').readline()); print('C2 $v', round(d['value']/1e6,3), 'M reads/s busy', round(d['roofline']['kernel_busy_ms_per_step'],2))"
  done
done
