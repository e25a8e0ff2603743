#!/bin/bash
# d1-boundary bench variants on one box: kernel overlap on/off x chunk sizes (bench only).
mkdir -p gpurun_out
for i in 1 2; do
  for v in "0 262144" "1 262144" "0 131072" "0 500000" "0 1000000"; do
    set -- $v
    SNAPGPU_OVERLAP=$1 SNAPGPU_CHUNK_READS=$2 timeout -k 10 120 python bench.py --steps 20 --no-cpu-baseline --no-extras > gpurun_out/abc_$1_$2_$i.log 2>/dev/null || exit $?
  done
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/abc_*.log")):
    d = json.loads(open(f).readline())
    r = d["roofline"]
    print(f, round(d["value"] / 1e6, 3), round(d["ms_per_step"], 2), "kms/launch", round(r["kernel_ms_per_launch"], 2), "launches", r["launches_per_step"])
PY
