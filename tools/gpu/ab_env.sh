#!/bin/bash
# A/B of environment settings on one box (bench only, alternating, 2 rounds):
#   bash tools/gpu/ab_env.sh "SNAPGPU_HEAVY_FIRST=0" "SNAPGPU_HEAVY_FIRST=1" ...
mkdir -p gpurun_out
for i in 1 2; do
  k=0
  for v in "$@"; do
    k=$((k+1))
    env $v timeout -k 10 120 python bench.py --steps 20 --no-cpu-baseline --no-extras > gpurun_out/abe_${k}_$i.log 2>/dev/null || exit $?
    env $v timeout -k 10 120 python bench.py --steps 10 --resident-steps 10 --no-cpu-baseline --paired-pairs 0 > gpurun_out/abr_${k}_$i.log 2>/dev/null || exit $?
  done
done
python3 - "$@" <<'PY'
import json, sys
for k, v in enumerate(sys.argv[1:], 1):
    d1 = [json.loads(open(f"gpurun_out/abe_{k}_{i}.log").readline()) for i in (1, 2)]
    rs = [json.loads(open(f"gpurun_out/abr_{k}_{i}.log").readline())["resident"] for i in (1, 2)]
    print(v, "d1", [round(d["value"] / 1e6, 3) for d in d1], "resident", [round(r["value"] / 1e6, 3) for r in rs],
          "busy/launch", [round(d["roofline"]["kernel_ms_per_launch"], 3) for d in d1])
PY
