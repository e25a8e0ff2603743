#!/bin/bash
# Round 4: occupancy test of align_kernel<128> (verdict r3 item 3) and a bisect of 3f0aeb9's parts.
#  (a) the same library at 4, 3 and 2 resident waves per SIMD (SNAPGPU_WAVES_PER_CU 16/12/8:
#      only the persistent grid shrinks; code, registers and LDS caps are those of the build);
#  (b) ELCAP = 6 builds (LDS 8,176 B, fits 5 waves) at 4 and at 5 waves/SIMD (96 VGPRs, 44 B scratch);
#  (c) 3f0aeb9's parts: e24 (ELCAP 24) vs h32e24 (u32 chain heads, ELCAP 24); ord256 (ORDCAP 256).
# C2 alternating, three rounds; C3 for (b) and cur; the paired leg (small fallback subsets packed).
export TMPDIR=/tmp
O=gpurun_out/r04j; mkdir -p $O
export SNAPGPU_TIMEOUT_S=90
L=$PWD/snap-rnaseq_amd/snapgpu
run() {  # name lib wpc args...
  local n=$1 lib=$2 w=$3; shift 3
  SNAPGPU_LIB=$lib SNAPGPU_WAVES_PER_CU=$w timeout -k 10 400 python bench.py "$@" > $O/$n.json 2> $O/$n.err || { tail $O/$n.err; exit 1; }
}
C2="--steps 10 --warmup 2 --no-cpu-baseline --no-extras"
for i in 1 2 3; do
  for w in 16 12 8; do run cur_w$w\_$i $L/libsnapgpu.so $w $C2; done
  for v in e6w4 e6w5 e24 h32e24 ord256; do run ${v}_$i $L/libsnapgpu_$v.so 0 $C2; done
done
for v in e6w4 e6w5; do run c3_${v} $L/libsnapgpu_$v.so 0 --workload c3 --steps 3 --warmup 1 --no-cpu-baseline --no-extras; done
run c3_cur $L/libsnapgpu.so 0 --workload c3 --steps 3 --warmup 1 --no-cpu-baseline --no-extras
run cur_paired $L/libsnapgpu.so 0 --steps 2 --warmup 1 --no-cpu-baseline --rna-pairs 0
python3 - <<'PY' | tee gpurun_out/r04j/summary.txt
import json
def row(n):
    d = json.loads(open(f'gpurun_out/r04j/{n}.json').readline())
    r = d['roofline']
    return f"{n:14s} {d['value'] / 1e6:7.3f} M reads/s  kernel {r['kernel_ms_per_launch']:7.2f} ms/launch"
for i in (1, 2, 3):
    for n in ('cur_w16', 'cur_w12', 'cur_w8', 'e6w4', 'e6w5', 'e24', 'h32e24', 'ord256'):
        print(row(f'{n}_{i}'))
for n in ('c3_e6w4', 'c3_e6w5', 'c3_cur'):
    print(row(n))
d = json.loads(open('gpurun_out/r04j/cur_paired.json').readline())
p = d.get('paired') or d.get('extras', {}).get('paired')
print('cur_paired', round(p['value'] / 1e6, 3), round(p['ms_per_batch'], 1), p.get('fallback_pairs'))
PY
