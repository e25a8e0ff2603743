#!/bin/bash
# RNA leg against the host worker count of its stages (SNAPGPU_HOST_THREADS: 16, 12, 8; the job's
# CPU quota is 16): tools/rna_sub_probe.py with 2 sub-batches, alternating, best of 3 each.
export TMPDIR=/tmp SNAPGPU_TIMEOUT_S=120
T=${1:?tag}; O=gpurun_out/$T; mkdir -p $O
true
true
for i in 1 2; do
  for w in 16 12 8; do
    echo "== threads $w ($i)"
    SNAPGPU_HOST_THREADS=$w timeout -k 10 300 python -u tools/rna_sub_probe.py 100000 2 2> $O/probe_${w}_$i.err || { tail $O/probe_${w}_$i.err; exit 1; }
  done
done
