#!/bin/bash
# Select-form mask scans in the lane-pair filter + CIGARs overlapped with stage B of the RNA path:
# the evidence run (GPU suite, smoke, C2 / C3 bench), then the RNA sub-batch probe.
export TMPDIR=/tmp SNAPGPU_TIMEOUT_S=120
T=${1:?tag}; O=gpurun_out/$T; mkdir -p $O
bash tools/gpu/evidence.sh $T c3 || exit 1
timeout -k 10 600 python -u tools/rna_sub_probe.py > $O/rna_sub.txt 2> $O/rna_sub.err || { tail $O/rna_sub.err; exit 1; }
cat $O/rna_sub.txt
