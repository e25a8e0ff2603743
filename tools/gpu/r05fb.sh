#!/bin/bash
# The chimeric fallback of a sparse batch as one packed single-end batch (paired.hip) against the
# build before (two batches): the paired / RNA tests, then the paired leg of the bench alternating.
export TMPDIR=/tmp SNAPGPU_TIMEOUT_S=120
T=${1:?tag}; O=gpurun_out/$T; mkdir -p $O
L=$PWD/snap-rnaseq_amd/snapgpu
timeout -k 10 600 python -u -m pytest tests/test_paired.py tests/test_rna_paired.py tests/test_c3_scale.py -x -v -m gpu \
  --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  for v in cur prev; do
    if [ $v = cur ]; then lib=$L/libsnapgpu.so; else lib=$L/libsnapgpu_prev.so; fi
    SNAPGPU_LIB=$lib timeout -k 10 400 python bench.py --no-cpu-baseline --rna-pairs 0 --steps 5 > $O/b_${v}_$i.json 2> $O/b_${v}_$i.err || { tail $O/b_${v}_$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/b_${v}_$i.json').readline()); p=d['paired']; print('$v', 'paired', round(p['value']/1e6,3), 'M reads/s', round(p['ms_per_batch'],2), 'ms/batch; intersect', round(p['intersect_only_ms'],2), 'mismatches', p['parity'].get('mismatches') if isinstance(p['parity'], dict) else p['parity'])"
  done
done
