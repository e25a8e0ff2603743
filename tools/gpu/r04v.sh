#!/bin/bash
# Round 4: hit insertion grouped by neighbouring lanes (sorted hit lists) instead of the LDS hash table:
# the GPU suite on it, then A/B against the build before (prevnb): C2 three alternating rounds, C3 once each.
export TMPDIR=/tmp SNAPGPU_TIMEOUT_S=90
O=gpurun_out/r04v; mkdir -p $O
L=$PWD/snap-rnaseq_amd/snapgpu
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
C2="--steps 10 --warmup 2 --no-cpu-baseline --no-extras"
for i in 1 2 3; do
  timeout -k 10 300 python bench.py $C2 > $O/cur_$i.json 2> $O/cur_$i.err || exit 1
  SNAPGPU_LIB=$L/libsnapgpu_prevnb.so timeout -k 10 300 python bench.py $C2 > $O/prevnb_$i.json 2> $O/prevnb_$i.err || exit 1
done
C3="--workload c3 --steps 3 --warmup 1 --no-cpu-baseline --no-extras"
timeout -k 10 400 python bench.py $C3 > $O/c3_cur.json 2> $O/c3_cur.err || exit 1
SNAPGPU_LIB=$L/libsnapgpu_prevnb.so timeout -k 10 400 python bench.py $C3 > $O/c3_prevnb.json 2> $O/c3_prevnb.err || exit 1
python3 - <<'PY' | tee gpurun_out/r04v/ab.txt
import json
def row(n):
    d = json.loads(open(f'gpurun_out/r04v/{n}.json').readline())
    return f"{n:10s} {d['value'] / 1e6:7.3f} M reads/s  kernel {d['roofline']['kernel_ms_per_launch']:7.2f} ms/launch"
for i in (1, 2, 3):
    for n in ("cur", "prevnb"):
        print(row(f'{n}_{i}'))
for n in ("c3_cur", "c3_prevnb"):
    print(row(n))
PY
