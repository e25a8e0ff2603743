#!/bin/bash
# Round 5 final evidence, one box: the GPU suite, smoke(), the default bench line, the C3 line
# (tools/gpu/evidence.sh) and the RNA sub-batch probe -> gpurun_out/<tag>/.
#   gpurun -- bash tools/gpu/final_r05.sh <tag>
export TMPDIR=/tmp SNAPGPU_TIMEOUT_S=120
T=${1:?tag}; O=gpurun_out/$T; mkdir -p $O
bash tools/gpu/evidence.sh $T c3 || exit 1
timeout -k 10 600 python -u tools/rna_sub_probe.py > $O/rna_sub.txt 2> $O/rna_sub.err || { tail $O/rna_sub.err; exit 1; }
cat $O/rna_sub.txt
