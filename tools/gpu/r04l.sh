#!/bin/bash
# Round 4: match-probability factors from LDS (cur: phred / indel tables copied per wave, ELCAP 20)
# against the previous build (prev = 8c444fe), and two knockouts of cur that give the marginal cost
# of a success's parts (timing only, results not valid): kprob (no match-probability product), knear
# (no nearby element lookup).  C2, 10 steps, three alternating rounds; C3 cur vs prev.
export TMPDIR=/tmp
O=gpurun_out/r04l; mkdir -p $O
export SNAPGPU_TIMEOUT_S=120
L=$PWD/snap-rnaseq_amd/snapgpu
run() {  # name lib args...
  local n=$1 lib=$2; shift 2
  SNAPGPU_LIB=$lib timeout -k 10 400 python bench.py "$@" > $O/$n.json 2> $O/$n.err || { tail $O/$n.err; exit 1; }
}
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
C2="--steps 10 --warmup 2 --no-cpu-baseline --no-extras"
for i in 1 2 3; do
  run cur_$i $L/libsnapgpu.so $C2
  for v in prev kprob knear; do run ${v}_$i $L/libsnapgpu_$v.so $C2; done
done
for v in cur prev; do
  lib=$L/libsnapgpu_$v.so; [ $v = cur ] && lib=$L/libsnapgpu.so
  run c3_$v $lib --workload c3 --steps 3 --warmup 1 --no-cpu-baseline --no-extras
done
python3 - <<'PY' | tee gpurun_out/r04l/ab.txt
import json
def row(n):
    d = json.loads(open(f'gpurun_out/r04l/{n}.json').readline())
    return f"{n:10s} {d['value'] / 1e6:7.3f} M reads/s  kernel {d['roofline']['kernel_ms_per_launch']:7.2f} ms/launch  mismatches {d.get('parity', {}).get('mismatches', '-')}"
for i in (1, 2, 3):
    for n in ("cur", "prev", "kprob", "knear"):
        print(row(f'{n}_{i}'))
for n in ("c3_cur", "c3_prev"):
    print(row(n))
PY
