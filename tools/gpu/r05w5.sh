#!/bin/bash
# 5 waves/SIMD for align_kernel<256> (libsnapgpu_w5.so: 96 VGPRs + 60 B/lane scratch for the plain
# twin) against the 4-wave build, on the RNA leg (tools/rna_sub_probe.py, 1 and 2 sub-batches,
# alternating); first the new statistics test.
export TMPDIR=/tmp SNAPGPU_TIMEOUT_S=120
T=${1:?tag}; O=gpurun_out/$T; mkdir -p $O
L=$PWD/snap-rnaseq_amd/snapgpu
timeout -k 10 300 python -u -m pytest tests/test_gpu_edges.py tests/test_rna_paired.py -x -v -m gpu --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  for v in cur w5; do
    if [ $v = cur ]; then lib=$L/libsnapgpu.so; else lib=$L/libsnapgpu_$v.so; fi
    echo "== $v $i"
    SNAPGPU_LIB=$lib timeout -k 10 300 python -u tools/rna_sub_probe.py 100000 1,2 2> $O/probe_${v}_$i.err || { tail $O/probe_${v}_$i.err; exit 1; }
  done
done
