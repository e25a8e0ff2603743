#!/bin/bash
# Round 4: GPU suite, serialised lookup trace, C2 A/B against the previous build.
export TMPDIR=/tmp
O=gpurun_out/r04g; mkdir -p $O
export SNAPGPU_TIMEOUT_S=90
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
SNAPGPU_OVERLAP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/serial_kt -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-extras --no-cpu-baseline > $O/serial_kt.json 2> $O/serial_kt.log || exit $?
python3 - <<'PY'
import csv, glob
for f in glob.glob('gpurun_out/r04g/serial_kt/**/*kernel_stats.csv', recursive=True):
    for row in csv.DictReader(open(f)):
        if 'seed_lookup' in row['Name'] or 'align_kernel<128' in row['Name']:
            print(row['Name'][:60], row['Calls'], row['AverageNs'])
PY
timeout -k 10 600 bash tools/abn.sh prev > $O/abn.txt 2>&1 || { tail -20 $O/abn.txt; exit 1; }
cat $O/abn.txt
