#!/bin/bash
# Alternating A/B/n of library variants on the headline bench (C2, stream mode, no extras):
#   bash tools/gpu/abx.sh <tag> <rounds> <variant...>   (variant "cur" = snapgpu/libsnapgpu.so,
#   else snapgpu/libsnapgpu_<v>.so); prints reads/s per variant and round.
TAG=$1; R=$2; shift 2
mkdir -p gpurun_out/$TAG
L=$PWD/snap-rnaseq_amd/snapgpu
for i in $(seq 1 $R); do
  for v in "$@"; do
    if [ "$v" = cur ]; then lib=$L/libsnapgpu.so; else lib=$L/libsnapgpu_$v.so; fi
    SNAPGPU_LIB=$lib timeout -k 10 200 python bench.py --steps 10 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/$TAG/ab_${v}_$i.json 2> gpurun_out/$TAG/ab_${v}_$i.err || { tail -5 gpurun_out/$TAG/ab_${v}_$i.err; exit 1; }
  done
done
python3 - $TAG $R "$@" <<'PY'
import json, sys
tag, R, vs = sys.argv[1], int(sys.argv[2]), sys.argv[3:]
for v in vs:
    xs = [json.loads(open(f"gpurun_out/{tag}/ab_{v}_{i}.json").readline()) for i in range(1, R + 1)]
    print(v, [round(x["value"] / 1e6, 3) for x in xs], "busy ms/launch", [round(x["roofline"]["kernel_ms_per_launch"], 2) for x in xs])
PY
