#!/bin/bash
# Alternating A/B of library builds on one box: bash tools/gpu/ab_lib.sh <script.py args> -- lib1 lib2 ...
# (each lib path relative to snap-rnaseq_amd/snapgpu/), 2 rounds; output gpurun_out/ablib_<k>_<i>.log
mkdir -p gpurun_out
CMD=()
while [ "$1" != "--" ]; do CMD+=("$1"); shift; done
shift
for i in 1 2; do
  k=0
  for lib in "$@"; do
    k=$((k+1))
    SNAPGPU_LIB=$PWD/snap-rnaseq_amd/snapgpu/$lib timeout -k 10 200 python3 "${CMD[@]}" > gpurun_out/ablib_${k}_$i.log 2>&1 || exit $?
  done
done
k=0
for lib in "$@"; do k=$((k+1)); echo "== $lib"; cat gpurun_out/ablib_${k}_1.log gpurun_out/ablib_${k}_2.log | grep -v "^\[" ; done
