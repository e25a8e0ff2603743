#!/bin/bash
# Round 4 step: GPU suite on the current library, A/B against the previous build (C2 bench, C3
# resident), serialised kernel trace (seed_lookup_kernel duration), FETCH/WRITE of the align kernel.
export TMPDIR=/tmp
O=gpurun_out/r04e; mkdir -p $O
export SNAPGPU_TIMEOUT_S=90
L=$PWD/snap-rnaseq_amd/snapgpu
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 600 bash tools/abn.sh prev > $O/abn.txt 2>&1 || { tail -20 $O/abn.txt; exit 1; }
cat $O/abn.txt
timeout -k 10 300 python tools/ab_c3.py build > $O/c3_build.log 2>&1 || { tail $O/c3_build.log; exit 1; }
for r in 1 2; do for v in libsnapgpu libsnapgpu_prev; do
  SNAPGPU_LIB=$L/$v.so timeout -k 10 300 python tools/ab_c3.py run >> $O/c3_ab.txt 2>&1 || { tail $O/c3_ab.txt; rm -f /dev/shm/snapgpu_ab_c3.bin; exit 1; }
done; done
rm -f /dev/shm/snapgpu_ab_c3.bin
cat $O/c3_ab.txt
SNAPGPU_OVERLAP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/serial_kt -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-extras --no-cpu-baseline > $O/serial_kt.json 2> $O/serial_kt.log || exit $?
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras"
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d $O/pmc1 -o run --output-format csv -- $B > $O/pmc1.log 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d $O/pmc1w -o run --output-format csv -- $B > $O/pmc1w.log 2>&1 || exit $?
python3 - <<'PY'
import csv, glob, collections
for f in glob.glob('gpurun_out/r04e/serial_kt/**/*kernel_stats.csv', recursive=True):
    for row in csv.DictReader(open(f)):
        if 'seed_lookup' in row['Name'] or 'align_kernel<128' in row['Name']:
            print(row['Name'][:60], row['Calls'], row['AverageNs'])
for tag in ('pmc1', 'pmc1w'):
    for f in glob.glob(f'gpurun_out/r04e/{tag}/**/*counter_collection.csv', recursive=True):
        acc = collections.defaultdict(list)
        for row in csv.DictReader(open(f)):
            if 'align_kernel<128, false>' in row['Kernel_Name']:
                acc[row['Counter_Name']].append(float(row['Counter_Value']))
        for k, v in acc.items(): print(tag, k, 'per dispatch KB', sum(v) / len(v))
PY
