#!/bin/bash
# Round 4: align_kernel<128> at 6 waves/SIMD (w6m: amdgpu_waves_per_eu(6), SKCAP / MIRCAP 256 -> 128,
# ELCAP 6 -> 4: 6,768 B of LDS, 80 VGPRs, 40 B/lane scratch): single-end parity on it, then A/B
# against the current build: C2 two alternating rounds, C3 once each.
export TMPDIR=/tmp SNAPGPU_TIMEOUT_S=90
O=gpurun_out/r04w; mkdir -p $O
L=$PWD/snap-rnaseq_amd/snapgpu
SNAPGPU_LIB=$L/libsnapgpu_w6m.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
C2="--steps 10 --warmup 2 --no-cpu-baseline --no-extras"
for i in 1 2; do
  timeout -k 10 300 python bench.py $C2 > $O/cur_$i.json 2> $O/cur_$i.err || exit 1
  SNAPGPU_LIB=$L/libsnapgpu_w6m.so timeout -k 10 300 python bench.py $C2 > $O/w6m_$i.json 2> $O/w6m_$i.err || exit 1
done
C3="--workload c3 --steps 3 --warmup 1 --no-cpu-baseline --no-extras"
timeout -k 10 400 python bench.py $C3 > $O/c3_cur.json 2> $O/c3_cur.err || exit 1
SNAPGPU_LIB=$L/libsnapgpu_w6m.so timeout -k 10 400 python bench.py $C3 > $O/c3_w6m.json 2> $O/c3_w6m.err || exit 1
python3 - <<'PY' | tee gpurun_out/r04w/ab.txt
import json
def row(n):
    d = json.loads(open(f'gpurun_out/r04w/{n}.json').readline())
    return f"{n:10s} {d['value'] / 1e6:7.3f} M reads/s  kernel {d['roofline']['kernel_ms_per_launch']:7.2f} ms/launch"
for i in (1, 2):
    for n in ("cur", "w6m"):
        print(row(f'{n}_{i}'))
for n in ("c3_cur", "c3_w6m"):
    print(row(n))
PY
