#!/bin/bash
# Round 4: GPU suite, then C2 headline A/B against the round-3 final build (ab/r03: its own
# bench.py and library, commit 17016c4), alternating, then the full bench (RNA + paired legs).
export TMPDIR=/tmp
O=gpurun_out/r04h; mkdir -p $O
export SNAPGPU_TIMEOUT_S=90
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extras > $O/cur_$i.json 2> $O/cur_$i.err || { tail $O/cur_$i.err; exit 1; }
  (cd ab/r03 && timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extras) > $O/r03_$i.json 2> $O/r03_$i.err || { tail $O/r03_$i.err; exit 1; }
done
python3 - <<'PY'
import json
for v in ('cur', 'r03'):
    for i in (1, 2, 3):
        d = json.loads(open(f'gpurun_out/r04h/{v}_{i}.json').readline())
        r = d['roofline']
        print(v, i, round(d['value'] / 1e6, 3), 'ms/step', round(d['ms_per_step'], 2), 'kernel', round(r['kernel_ms_per_launch'], 2), 'launch', round(r['launch_duration_ms'], 2))
PY
timeout -k 10 600 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 - <<'PY'
import json; d=json.loads(open('gpurun_out/r04h/bench.json').readline())
print('value', round(d['value']/1e6,3), 'kernel_ms', round(d['roofline']['kernel_ms_per_launch'],2))
lk=d['lookup_roofline']; print('lookup', {k: lk.get(k) for k in ('kernel_ms_per_launch','achieved','frac_of_measured_copy_peak')})
r=d['rna_paired']; print('rna', round(r['value']/1e6,3), r['stage_ms'], r['parity'].get('sha256_match'))
p=d['paired']; print('paired', round(p['value']/1e6,3))
PY
