#!/bin/bash
# Per-phase cycle breakdown (PHASE_TIMERS build) on C2 and on the C3 genome (1M reads each).
mkdir -p gpurun_out
export SNAPGPU_TIMEOUT_S=120 SNAPGPU_PHASES=1 SNAPGPU_LIB=$PWD/snap-rnaseq_amd/snapgpu/libsnapgpu_phases.so
timeout -k 10 200 python -u tools/phase_probe.py > gpurun_out/phase_c2.json 2> gpurun_out/phase_c2.err || exit $?
timeout -k 10 500 python -u tools/phase_probe.py --genome-bases 3100000000 --contigs 25 --families 2000 > gpurun_out/phase_c3.json 2> gpurun_out/phase_c3.err || exit $?
python3 - <<'PY'
import json
for w in ("c2", "c3"):
    d = json.load(open(f"gpurun_out/phase_{w}.json"))
    c = d["cycles_per_read"]
    print(w, "kernel_ms", round(d["kernel_ms"], 1), "cyc/read", int(c["cycles_per_read_total"]),
          {k: v for k, v in d["share_of_wave_time"].items() if v > 0.01})
PY
