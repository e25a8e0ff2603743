#!/bin/bash
# Alternating A/B of the current library ("cur") against snapgpu/libsnapgpu_<v>.so variants: the C2
# bench line (10 steps, no extras, oracle parity on 200k reads), R rounds -> gpurun_out/<tag>/.
#   gpurun -- bash tools/gpu/ab2.sh <tag> <rounds> v1 v2 ...
# WL=c3: the C3 per-GPU shard's index (3.1 Gb) with 1M of its reads per step instead
export TMPDIR=/tmp SNAPGPU_TIMEOUT_S=90
EXTRA=""; [ "$WL" = c3 ] && EXTRA="--workload c3 --reads 1000000"
T=${1:?tag}; R=${2:?rounds}; shift 2
O=gpurun_out/$T; mkdir -p $O
L=$PWD/snap-rnaseq_amd/snapgpu
cp $L/libsnapgpu.so $L/libsnapgpu_cur.so
for i in $(seq 1 $R); do
  for v in cur "$@"; do
    SNAPGPU_LIB=$L/libsnapgpu_$v.so timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-extras --cpu-sample 200000 $EXTRA \
      > $O/ab_${v}_$i.json 2> $O/ab_${v}_$i.err || { tail -5 $O/ab_${v}_$i.err; exit 1; }
  done
done
python3 - $O $R cur "$@" <<'PY' | tee $O/ab_summary.txt
import json, sys
o, R = sys.argv[1], int(sys.argv[2])
for v in sys.argv[3:]:
    ds = [json.loads(open(f"{o}/ab_{v}_{i}.json").readline()) for i in range(1, R + 1)]
    ks = [d["roofline"]["kernel_ms_per_launch"] for d in ds]
    print(v.ljust(7), "M reads/s", [round(d["value"] / 1e6, 3) for d in ds], "kernel ms", [round(k, 3) for k in ks],
          "mean", round(sum(ks) / len(ks), 3), "mismatches", [d["parity"]["mismatches"] for d in ds])
PY
