#!/bin/bash
# The RNA paired path's sub-batch pipeline: GPU tests of the paths that use the aligners' side
# stream (CIGARs, seed census, the RNA product paths), then tools/rna_sub_probe.py (1-4 sub-batches).
#   gpurun -- bash tools/gpu/rna_sub.sh <tag>
export TMPDIR=/tmp SNAPGPU_TIMEOUT_S=120
T=${1:?tag}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_rna_paired.py tests/test_cigar.py tests/test_charseeds.py tests/test_single.py \
  tests/test_sorted.py -x -v -m gpu --timeout 200 --timeout-method thread > $O/side_tests.log 2>&1 || { tail -30 $O/side_tests.log; exit 1; }
tail -1 $O/side_tests.log
timeout -k 10 600 python -u tools/rna_sub_probe.py > $O/rna_sub.txt 2> $O/rna_sub.err || { tail $O/rna_sub.err; exit 1; }
cat $O/rna_sub.txt
