#!/bin/bash
# Round 4: GPU suite; A/B of the element LDS cap (ELCAP 6/16/24/32) and of u32 chain heads
# (h32e24 vs e24); phase split of align_kernel<128> with the success step's parts timed
# (PHASE_TIMERS build, libsnapgpu_phases.so), C2 and C3, 1M reads each.
export TMPDIR=/tmp
O=gpurun_out/r04k; mkdir -p $O
export SNAPGPU_TIMEOUT_S=120
L=$PWD/snap-rnaseq_amd/snapgpu
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
run() {  # name lib args...
  local n=$1 lib=$2; shift 2
  SNAPGPU_LIB=$lib timeout -k 10 400 python bench.py "$@" > $O/$n.json 2> $O/$n.err || { tail $O/$n.err; exit 1; }
}
C2="--steps 10 --warmup 2 --no-cpu-baseline --no-extras"
for i in 1 2 3; do
  run cur_$i $L/libsnapgpu.so $C2
  for v in e6 e16 e24 h32e24; do run ${v}_$i $L/libsnapgpu_$v.so $C2; done
done
python3 - <<'PY' | tee gpurun_out/r04k/ab.txt
import json
for i in (1, 2, 3):
    for n in ('cur', 'e6', 'e16', 'e24', 'h32e24'):
        d = json.loads(open(f'gpurun_out/r04k/{n}_{i}.json').readline())
        print(f"{n}_{i:<10} {d['value'] / 1e6:7.3f} M reads/s  kernel {d['roofline']['kernel_ms_per_launch']:7.2f} ms/launch")
PY
export SNAPGPU_PHASES=1 SNAPGPU_LIB=$L/libsnapgpu_phases.so
timeout -k 10 200 python -u tools/phase_probe.py > $O/phase_c2.json 2> $O/phase_c2.err || { tail $O/phase_c2.err; exit 1; }
timeout -k 10 500 python -u tools/phase_probe.py --genome-bases 3100000000 --contigs 25 --families 2000 > $O/phase_c3.json 2> $O/phase_c3.err || { tail $O/phase_c3.err; exit 1; }
python3 - <<'PY'
import json
for w in ("c2", "c3"):
    d = json.load(open(f"gpurun_out/r04k/phase_{w}.json"))
    c = d["cycles_per_read"]
    print(w, "kernel_ms", round(d["kernel_ms"], 1), "cyc/read", int(c["cycles_per_read_total"]),
          {k: v for k, v in d["share_of_wave_time"].items() if v > 0.01})
    print("  per success", d["cycles_per_success"], "n_succ/read", round(c["n_succ"], 2))
    print("  per pass", d["cycles_per_pass"], "overhead", d["pass_overhead_per_pass"], "n_pass/read", round(c["n_pass"], 2))
PY
