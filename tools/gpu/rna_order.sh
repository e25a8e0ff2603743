#!/bin/bash
# Longest-first order of the RNA aligners' long-read lists (order_long.h), A/B on one box with the
# library snapgpu/libsnapgpu_<lib>.so: tools/rna_probe.py (100k 2 x 150 pairs, stage times) with
# SNAPGPU_ORDER_LONG=0 / 1 alternating, then the batch-size fit (tools/rna_tail_probe.py) with the
# order on.  Results in gpurun_out/<tag>/.
#   gpurun -- bash tools/gpu/rna_order.sh <tag> <lib>
export TMPDIR=/tmp SNAPGPU_TIMEOUT_S=120
T=${1:?tag}; O=gpurun_out/$T; mkdir -p $O
export SNAPGPU_LIB=$PWD/snap-rnaseq_amd/snapgpu/libsnapgpu_${2:?lib}.so
for i in 1 2; do
  for o in 0 1; do
    SNAPGPU_ORDER_LONG=$o timeout -k 10 300 python -u tools/rna_probe.py 100000 > $O/probe_o${o}_$i.txt 2> $O/probe_o${o}_$i.err || { tail $O/probe_o${o}_$i.err; exit 1; }
    echo "order=$o run $i: $(tail -c 1500 $O/probe_o${o}_$i.txt)" | cut -c1-1500
  done
done
SNAPGPU_ORDER_LONG=1 timeout -k 10 400 python -u tools/rna_tail_probe.py > $O/tail_o1.txt 2> $O/tail_o1.err || { tail $O/tail_o1.err; exit 1; }
tail -12 $O/tail_o1.txt
