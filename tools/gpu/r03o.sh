#!/bin/bash
# round-3 session-2 evidence on one box: GPU suite + quick bench + RNA probe (tools/gpu/check.sh), then
# the per-phase split of align_kernel<128> on C2 and C3 (PHASE_TIMERS variant, tools/gpu/phase_c3.sh)
bash tools/gpu/check.sh || exit $?
bash tools/gpu/phase_c3.sh
