#!/bin/bash
# A/B/n of library variants on one box with parity: for the current library ("cur") and every
# snapgpu/libsnapgpu_<v>.so named, two alternating rounds of the C2 bench line (no extras) with the
# oracle parity of the first 300k reads; prints reads/s, kernel busy ms per launch and mismatches.
#   gpurun -- bash tools/gpu/ab_parity.sh <tag> v1 v2 ...
export TMPDIR=/tmp SNAPGPU_TIMEOUT_S=90
T=${1:?tag}; shift
O=gpurun_out/$T; mkdir -p $O
L=snap-rnaseq_amd/snapgpu
for i in 1 2; do
  for v in cur "$@"; do
    if [ "$v" = cur ]; then lib=$PWD/$L/libsnapgpu.so; else lib=$PWD/$L/libsnapgpu_$v.so; fi
    SNAPGPU_LIB=$lib timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-extras --cpu-sample 300000 \
      > $O/ab_${v}_$i.json 2> $O/ab_${v}_$i.err || { tail -5 $O/ab_${v}_$i.err; exit 1; }
  done
done
python3 - $O cur "$@" <<'PY'
import json, sys
o = sys.argv[1]
for v in sys.argv[2:]:
    ds = [json.loads(open(f"{o}/ab_{v}_{i}.json").readline()) for i in (1, 2)]
    print(v.ljust(8), "M reads/s", [round(d["value"] / 1e6, 3) for d in ds], "kernel ms/launch",
          [round(d["roofline"]["kernel_ms_per_launch"], 3) for d in ds], "mismatches",
          [d["parity"]["mismatches"] for d in ds])
PY
