#!/bin/bash
# Register / LDS / scratch report of the kernels (compiler remarks, gfx950, the Makefile's flags).
cd "$(dirname "$0")/../snap-rnaseq_amd" && /opt/rocm/bin/hipcc -DSNAPGPU_PHASE_TIMERS=${PHASE_TIMERS:-0} -O3 -std=c++17 -fPIC \
  --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -munsafe-fp-atomics -I../include -Icsrc/host -Icsrc \
  -Wno-unused-result -Wno-unused-value -mllvm -disable-machine-licm -mllvm -structurizecfg-skip-uniform-regions -mllvm -amdgpu-atomic-optimizer-strategy=None --cuda-device-only \
  -c csrc/aligner.hip -o /tmp/kres.o -Rpass-analysis=kernel-resource-usage 2>&1 |
  grep -E "Function Name|VGPRs:|ScratchSize|Occupancy|LDS Size|SGPRs:" | sed 's/.*remark: //;s/ \[-Rpass.*//' |
  awk '/Function Name/{n=$3; next} {print n " | " $0}' | grep -E "${1:-align_kernel}"
