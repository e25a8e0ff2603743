#!/bin/bash
# Round 4: GPU suite; A/B of the success step's match-probability product: prev (8c444fe), fac2
# (phred / indel factors from an LDS copy per wave, a uniform per-read fallback to the global table
# when a quality byte lies outside it), cur (fac2 + the product over the non-1.0 factors only);
# C2 three alternating rounds, C3 once each; then the RNA PMC pass (tools/gpu/rna_pmc.sh r04).
export TMPDIR=/tmp
O=gpurun_out/r04m; mkdir -p $O
export SNAPGPU_TIMEOUT_S=120
L=$PWD/snap-rnaseq_amd/snapgpu
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
run() {  # name lib args...
  local n=$1 lib=$2; shift 2
  SNAPGPU_LIB=$lib timeout -k 10 400 python bench.py "$@" > $O/$n.json 2> $O/$n.err || { tail $O/$n.err; exit 1; }
}
C2="--steps 10 --warmup 2 --no-cpu-baseline --no-extras"
for i in 1 2 3; do
  run cur_$i $L/libsnapgpu.so $C2
  for v in prev fac2; do run ${v}_$i $L/libsnapgpu_$v.so $C2; done
done
run c3_cur $L/libsnapgpu.so --workload c3 --steps 3 --warmup 1 --no-cpu-baseline --no-extras
for v in prev fac2; do run c3_$v $L/libsnapgpu_$v.so --workload c3 --steps 3 --warmup 1 --no-cpu-baseline --no-extras; done
python3 - <<'PY' | tee gpurun_out/r04m/ab.txt
import json
def row(n):
    d = json.loads(open(f'gpurun_out/r04m/{n}.json').readline())
    return f"{n:10s} {d['value'] / 1e6:7.3f} M reads/s  kernel {d['roofline']['kernel_ms_per_launch']:7.2f} ms/launch"
for i in (1, 2, 3):
    for n in ("cur", "prev", "fac2"):
        print(row(f'{n}_{i}'))
for n in ("c3_cur", "c3_prev", "c3_fac2"):
    print(row(n))
PY
bash tools/gpu/rna_pmc.sh r04
