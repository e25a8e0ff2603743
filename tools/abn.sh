#!/bin/bash
# A/B/n on one GPU box: every snapgpu/libsnapgpu_*.so variant named on the command line
# (plus the current libsnapgpu.so as "cur"), two alternating rounds, bench only.
mkdir -p gpurun_out
L=snap-rnaseq_amd/snapgpu
for i in 1 2; do
  for v in cur "$@"; do
    if [ "$v" = cur ]; then lib=$PWD/$L/libsnapgpu.so; else lib=$PWD/$L/libsnapgpu_$v.so; fi
    SNAPGPU_LIB=$lib timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/abn_${v}_$i.log 2> gpurun_out/abn_${v}_$i.err || exit $?
  done
done
python3 - "$@" <<'PY'
import json, sys
for v in ["cur"] + sys.argv[1:]:
    xs = [json.loads(open(f"gpurun_out/abn_{v}_{i}.log").readline())["value"] for i in (1, 2)]
    print(v, [round(x / 1e6, 3) for x in xs])
PY
