#!/bin/bash
# Round 5: phase split of the forced-mode prefilter build (libsnapgpu_fph.so) beside the base timer
# build, then the RNA longest-first A/B (tools/gpu/rna_order.sh) on libsnapgpu_rna.so.
export TMPDIR=/tmp SNAPGPU_TIMEOUT_S=120 SNAPGPU_PHASES=1
O=gpurun_out/r05g; mkdir -p $O
SNAPGPU_LIB=$PWD/snap-rnaseq_amd/snapgpu/libsnapgpu_fph.so timeout -k 10 300 python tools/phase_probe.py > $O/phase_fph.json 2> $O/phase_fph.err || { tail $O/phase_fph.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/phase_fph.json')); print('fph', d['kernel_ms'], d['forced'], d['cycles_per_read']['n_filter'])"
unset SNAPGPU_PHASES
bash tools/gpu/rna_order.sh r05g rna
