#!/bin/bash
# Stream host tail without false sharing: record-path tests, then the default C2 line (no extras)
# alternating the current library and libsnapgpu_prev.so; ms/step, kernel busy, host tail per step.
export TMPDIR=/tmp SNAPGPU_TIMEOUT_S=90
T=${1:?tag}; O=gpurun_out/$T; mkdir -p $O
L=$PWD/snap-rnaseq_amd/snapgpu
timeout -k 10 400 python -u -m pytest tests/test_capi.py tests/test_gpu_golden.py tests/test_gpu_edges.py tests/test_single.py tests/test_rna_paired.py \
  -x -v -m gpu --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2 3; do
  for v in cur prev; do
    if [ $v = cur ]; then lib=$L/libsnapgpu.so; else lib=$L/libsnapgpu_prev.so; fi
    SNAPGPU_LIB=$lib timeout -k 10 300 python bench.py --no-extras --no-cpu-baseline > $O/b_${v}_$i.json 2> $O/b_${v}_$i.err || { tail $O/b_${v}_$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/b_${v}_$i.json').readline()); r=d['roofline']; print('$v', round(d['value']/1e6,3), 'M reads/s', round(d['ms_per_step'],3), 'ms/step; busy', round(r['kernel_busy_ms_per_step'],3), 'tail', round(d['config'].get('host_tail_ms_per_step'),2))"
  done
done
