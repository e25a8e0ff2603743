#!/bin/bash
# Round 4 iteration: bucket-image tests, the GPU suite, a bench with the lookup roofline and the RNA leg.
mkdir -p gpurun_out/r04a
export SNAPGPU_TIMEOUT_S=90
O=gpurun_out/r04a
timeout -k 10 300 python -u -m pytest tests/test_bucket_table.py -x -v -m gpu --timeout 120 --timeout-method thread > $O/bucket_tests.log 2>&1 || { tail -30 $O/bucket_tests.log; exit 1; }
tail -3 $O/bucket_tests.log
timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 500 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 - <<'PY'
import json; d=json.loads(open('gpurun_out/r04a/bench.json').readline())
lk=d['extras']['lookup_roofline']
print('value', round(d['value']/1e6,3), 'roofline', {k: d['roofline'].get(k) for k in ('achieved','frac','kernel_ms_per_launch')})
print('lookup', {k: lk.get(k) for k in ('kernel_ms_per_launch','achieved','frac','pass0_probes_per_read','applied_probes_per_read','probe_rate_frac_of_gather_peak','frac_of_measured_copy_peak')})
print('bucket', lk.get('bucket_image'))
r=d['extras'].get('rna_paired',{}); print('rna', r.get('value'), r.get('stages_ms') or {k:v for k,v in r.items() if 'ms' in k})
print('paired', d['extras'].get('paired',{}).get('value'))
PY
