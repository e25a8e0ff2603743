#!/bin/bash
# GPU-box diagnostic: per-phase breakdown, then the bench (no CPU baseline).
mkdir -p gpurun_out
export SNAPGPU_TIMEOUT_S=${SNAPGPU_TIMEOUT_S:-90}
SNAPGPU_PHASES=1 timeout -k 10 300 python tools/phase_probe.py > gpurun_out/phase.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 3 --warmup 1 ${BENCH_ARGS:---no-cpu-baseline} > gpurun_out/bp.log 2>&1
