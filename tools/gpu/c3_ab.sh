#!/bin/bash
# C3 A/B of library variants (one bench run each, no extras, oracle parity of 300k reads), after the
# GPU tests of the long-read ordering paths on the current library.
#   gpurun -- bash tools/gpu/c3_ab.sh <tag> v1 v2 ...
export TMPDIR=/tmp SNAPGPU_TIMEOUT_S=120
T=${1:?tag}; shift
O=gpurun_out/$T; mkdir -p $O
L=$PWD/snap-rnaseq_amd/snapgpu
timeout -k 10 600 python -u -m pytest tests/test_order_long.py tests/test_long_reads.py tests/test_paired.py tests/test_rna_paired.py \
  -x -v -m gpu --timeout 200 --timeout-method thread > $O/order_tests.log 2>&1 || { tail -30 $O/order_tests.log; exit 1; }
tail -1 $O/order_tests.log
cp $L/libsnapgpu.so $L/libsnapgpu_cur.so
for v in cur "$@" cur; do
  SNAPGPU_LIB=$L/libsnapgpu_$v.so timeout -k 10 400 python bench.py --workload c3 --steps 5 --warmup 1 --no-extras \
    --cpu-sample 300000 > $O/c3_$v.json 2> $O/c3_$v.err || { tail -5 $O/c3_$v.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/c3_$v.json').readline()); print('$v', round(d['value']/1e6,3), 'M reads/s', round(d['roofline']['kernel_ms_per_launch'],3), 'ms/launch', 'mismatches', d['parity']['mismatches'])"
done
