#!/bin/bash
# Round 4 A/B: the Elem64 build (e64) and its 5-waves/SIMD twin (e64w5) against the current library:
# parity first (golden digests, parity, multi-hit, long reads), then C2 bench and C3 resident timings.
set -o pipefail
O=gpurun_out/r04b; mkdir -p $O
export SNAPGPU_TIMEOUT_S=90
L=$PWD/snap-rnaseq_amd/snapgpu
SNAPGPU_LIB=$L/libsnapgpu_e64.so timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread \
  tests/test_gpu_golden.py tests/test_gpu_parity.py tests/test_multihit.py tests/test_long_reads.py tests/test_gpu_edges.py \
  tests/test_rna_paired.py > $O/e64_tests.log 2>&1 || { tail -30 $O/e64_tests.log; exit 1; }
tail -1 $O/e64_tests.log
SNAPGPU_LIB=$L/libsnapgpu_e64w5.so timeout -k 10 300 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread \
  tests/test_gpu_golden.py tests/test_gpu_parity.py > $O/e64w5_tests.log 2>&1 || { tail -30 $O/e64w5_tests.log; exit 1; }
tail -1 $O/e64w5_tests.log
timeout -k 10 900 bash tools/abn.sh e64 e64w5 > $O/abn.txt 2>&1 || { tail -20 $O/abn.txt; exit 1; }
cat $O/abn.txt
timeout -k 10 300 python tools/ab_c3.py build > $O/c3_build.log 2>&1 || { tail $O/c3_build.log; exit 1; }
for r in 1 2; do for v in libsnapgpu libsnapgpu_e64 libsnapgpu_e64w5; do
  SNAPGPU_LIB=$L/$v.so timeout -k 10 300 python tools/ab_c3.py run >> $O/c3_ab.txt 2>&1 || { tail $O/c3_ab.txt; rm -f /dev/shm/snapgpu_ab_c3.bin; exit 1; }
done; done
rm -f /dev/shm/snapgpu_ab_c3.bin
cat $O/c3_ab.txt
