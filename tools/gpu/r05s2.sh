#!/bin/bash
# Writer threads building their output in local strings (sam.cpp, single.cpp, rna_paired.cpp):
# the record-writing tests, then the default bench line (SAM-format and RNA legs) alternating the
# current library and libsnapgpu_prev.so.
export TMPDIR=/tmp SNAPGPU_TIMEOUT_S=120
T=${1:?tag}; O=gpurun_out/$T; mkdir -p $O
L=$PWD/snap-rnaseq_amd/snapgpu
timeout -k 10 500 python -u -m pytest tests/test_cigar.py tests/test_single.py tests/test_rna_paired.py tests/test_sorted.py \
  tests/test_contamination.py -x -v -m gpu --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  for v in cur prev; do
    if [ $v = cur ]; then lib=$L/libsnapgpu.so; else lib=$L/libsnapgpu_prev.so; fi
    SNAPGPU_LIB=$lib timeout -k 10 400 python bench.py --no-cpu-baseline --paired-pairs 0 > $O/b_${v}_$i.json 2> $O/b_${v}_$i.err || { tail $O/b_${v}_$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/b_${v}_$i.json').readline()); s=d['sam_records']; r=d['rna_paired']; print('$v', 'sam_format', round(s['sam_format_reads_per_s']/1e6,2), 'M lines/s; rna', round(r['value']/1e6,3), 'M reads/s', r['stage_ms'])"
  done
done
