#!/bin/bash
# Side-stream priority (SNAPGPU_SIDE_PRIORITY 1: the device's highest, 0: normal) on the RNA leg:
# the side-stream tests, then tools/rna_sub_probe.py (2 sub-batches, best of 3) alternating.
export TMPDIR=/tmp SNAPGPU_TIMEOUT_S=120
T=${1:?tag}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_rna_paired.py tests/test_cigar.py tests/test_charseeds.py -x -v -m gpu \
  --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2 3; do
  for p in 1 0; do
    echo "== priority $p ($i)"
    SNAPGPU_SIDE_PRIORITY=$p timeout -k 10 300 python -u tools/rna_sub_probe.py 100000 2 2> $O/probe_${p}_$i.err || { tail $O/probe_${p}_$i.err; exit 1; }
  done
done
