#!/bin/bash
# Phase split of align_kernel<128> (timer build libsnapgpu_phases.so, tools/build_variant.sh phases):
# C2 (and with `c3`, C3), 1M reads each -> gpurun_out/<tag>/phase_c2.json [phase_c3.json]
export TMPDIR=/tmp SNAPGPU_TIMEOUT_S=120 SNAPGPU_PHASES=1 SNAPGPU_LIB=$PWD/snap-rnaseq_amd/snapgpu/libsnapgpu_phases.so
T=${1:?tag}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 300 python tools/phase_probe.py > $O/phase_c2.json 2> $O/phase_c2.err || { tail $O/phase_c2.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/phase_c2.json')); print('phase c2', d['forced'], d['heavy_reads'])"
if [ "$2" = c3 ]; then
  timeout -k 10 600 python tools/phase_probe.py --genome-bases 3100000000 --contigs 25 --families 2000 > $O/phase_c3.json 2> $O/phase_c3.err || { tail $O/phase_c3.err; exit 1; }
fi
