#!/bin/bash
# Register / LDS / spill report of the align kernels (compiler remarks, gfx950).
cd /root/repo/snap-rnaseq_amd && /opt/rocm/bin/hipcc -DSNAPGPU_PHASE_TIMERS=${PHASE_TIMERS:-0} -O3 -std=c++17 -fPIC \
  --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -I../include -Icsrc/host -Icsrc --cuda-device-only \
  -c csrc/aligner.hip -o /tmp/kres.o -Rpass-analysis=kernel-resource-usage 2>&1 |
  grep -E "Function Name|VGPRs:|AGPRs|ScratchSize|Occupancy|LDS Size|SGPRs:" | sed 's/.*remark: //' |
  awk '/Function Name/{n=$0; next} {print n " | " $0}' | grep -E "${1:-align_kernel}"
