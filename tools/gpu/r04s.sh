#!/bin/bash
# Round 4: a clean 4-vs-5-waves test (verdict r3 item 3).  With -mllvm -structurizecfg-skip-uniform-regions
# align_kernel<128> needs 88-92 VGPRs, so at ELCAP 6 / forced-order window 128 (LDS 8,176 B) it runs 5
# waves/SIMD with no scratch.  s5 = that build at 5 waves (SNAPGPU_WAVES_PER_CU 20) and at 4 (16): the same
# binary, registers and LDS caps; s4 = the same sources with the 4-wave attribute (92 VGPRs, also 5 waves by
# resources); su = the flag alone on the current configuration (ELCAP 32, window 256, 4 waves); cur.
export TMPDIR=/tmp SNAPGPU_TIMEOUT_S=120
O=gpurun_out/r04s; mkdir -p $O
L=$PWD/snap-rnaseq_amd/snapgpu
run() {  # name lib wpc args...
  local n=$1 lib=$2 w=$3; shift 3
  SNAPGPU_LIB=$lib SNAPGPU_WAVES_PER_CU=$w timeout -k 10 400 python bench.py "$@" > $O/$n.json 2> $O/$n.err || { tail $O/$n.err; exit 1; }
}
C2="--steps 10 --warmup 2 --no-cpu-baseline --no-extras"
for i in 1 2 3; do
  run cur_$i $L/libsnapgpu.so 0 $C2
  run su_$i $L/libsnapgpu_su.so 0 $C2
  run s5w5_$i $L/libsnapgpu_s5.so 20 $C2
  run s5w4_$i $L/libsnapgpu_s5.so 16 $C2
  run s4w5_$i $L/libsnapgpu_s4.so 0 $C2
done
C3="--workload c3 --steps 3 --warmup 1 --no-cpu-baseline --no-extras"
run c3_cur $L/libsnapgpu.so 0 $C3
run c3_s5w5 $L/libsnapgpu_s5.so 20 $C3
run c3_s5w4 $L/libsnapgpu_s5.so 16 $C3
python3 - <<'PY' | tee gpurun_out/r04s/ab.txt
import json
def row(n):
    d = json.loads(open(f'gpurun_out/r04s/{n}.json').readline())
    return f"{n:10s} {d['value'] / 1e6:7.3f} M reads/s  kernel {d['roofline']['kernel_ms_per_launch']:7.2f} ms/launch"
for i in (1, 2, 3):
    for n in ("cur", "su", "s5w5", "s5w4", "s4w5"):
        print(row(f'{n}_{i}'))
for n in ("c3_cur", "c3_s5w5", "c3_s5w4"):
    print(row(n))
PY
