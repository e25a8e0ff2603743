#!/bin/bash
# One kernel iteration on the GPU box: the fast GPU parity suites, the default bench (1M-read
# oracle parity inside), and the phase probe when a phase-timer build is present.
mkdir -p gpurun_out
export SNAPGPU_TIMEOUT_S=90
timeout -k 10 300 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_golden.py tests/test_multihit.py tests/test_ref_index.py > gpurun_out/iter_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-extras "$@" > gpurun_out/iter_bench.json 2> gpurun_out/iter_bench.err || exit $?
if [ -f snap-rnaseq_amd/snapgpu/libsnapgpu_phases.so ]; then
  SNAPGPU_LIB=$PWD/snap-rnaseq_amd/snapgpu/libsnapgpu_phases.so SNAPGPU_PHASES=1 timeout -k 10 300 \
    python -u tools/phase_probe.py > gpurun_out/phase.json 2> gpurun_out/phase.err || exit $?
fi
