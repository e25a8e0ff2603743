#!/bin/bash
# phase probe (diagnostic timers) + one short bench line
mkdir -p gpurun_out
export SNAPGPU_TIMEOUT_S=90
SNAPGPU_PHASES=1 timeout -k 10 300 python tools/phase_probe.py > gpurun_out/phase.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bp.log 2>&1
