#!/bin/bash
# A/B on one GPU box: A = snapgpu/libsnapgpu_base.so, B = snapgpu/libsnapgpu.so,
# alternated A B A B so box-to-box clock differences cancel.  Bench only (no parity).
mkdir -p gpurun_out
L=snap-rnaseq_amd/snapgpu
for i in 1 2; do
  SNAPGPU_LIB=$PWD/$L/libsnapgpu_base.so timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ab_A$i.log 2>&1 || exit $?
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ab_B$i.log 2>&1 || exit $?
done
python3 - <<'PY'
import json
for v in "AB":
    xs = [json.loads(open(f"gpurun_out/ab_{v}{i}.log").readline())["value"] for i in (1, 2)]
    print(v, [round(x / 1e6, 3) for x in xs])
PY
