#!/bin/bash
# Round 6 final profiles, one box: tools/gpu/prof.sh (kernel trace + PMC passes of the bench) and
# tools/gpu/rna_pmc.sh (the RNA leg's kernels); summarised afterwards in the build container with
# tools/pmc_summary.py and tools/rna_pmc_summary.py.
#   gpurun -- bash tools/gpu/final_r06_prof.sh <tag>
bash tools/gpu/prof.sh ${1:?tag} && bash tools/gpu/rna_pmc.sh $1
