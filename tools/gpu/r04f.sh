#!/bin/bash
# Round 4: GPU suite, serialised lookup trace, full C2 bench (RNA + paired legs, no CPU baseline).
export TMPDIR=/tmp
O=gpurun_out/r04f; mkdir -p $O
export SNAPGPU_TIMEOUT_S=90
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
SNAPGPU_OVERLAP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/serial_kt -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-extras --no-cpu-baseline > $O/serial_kt.json 2> $O/serial_kt.log || exit $?
python3 - <<'PY'
import csv, glob
for f in glob.glob('gpurun_out/r04f/serial_kt/**/*kernel_stats.csv', recursive=True):
    for row in csv.DictReader(open(f)):
        if 'seed_lookup' in row['Name'] or 'align_kernel<128' in row['Name']:
            print(row['Name'][:60], row['Calls'], row['AverageNs'])
PY
timeout -k 10 600 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 - <<'PY'
import json; d=json.loads(open('gpurun_out/r04f/bench.json').readline())
print('value', round(d['value']/1e6,3), 'kernel_ms', round(d['roofline']['kernel_ms_per_launch'],2))
lk=d['lookup_roofline']; print('lookup', {k: lk.get(k) for k in ('kernel_ms_per_launch','achieved','frac_of_measured_copy_peak','probe_rate_frac_of_gather_peak')})
r=d['rna_paired']; print('rna', round(r['value']/1e6,3), r['stage_ms'], r['parity'].get('sha256_match'))
p=d['paired']; print('paired', round(p['value']/1e6,3))
PY
