#!/bin/bash
# Host tail of the stream path (one pass per record, up to 16 threads): the record-path GPU tests,
# then the default bench line twice.
export TMPDIR=/tmp SNAPGPU_TIMEOUT_S=90
T=${1:?tag}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_capi.py tests/test_gpu_golden.py tests/test_gpu_parity.py tests/test_gpu_edges.py \
  tests/test_watchdog.py -x -v -m gpu --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-extras --no-cpu-baseline > $O/bench$i.json 2> $O/bench$i.err || { tail $O/bench$i.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bench$i.json').readline()); r=d['roofline']; print('bench', round(d['value']/1e6,3), 'M reads/s', round(d['ms_per_step'],3), 'ms/step; busy', round(r['kernel_busy_ms_per_step'],3), 'tail', d['config'].get('host_tail_ms_per_step'))"
done
