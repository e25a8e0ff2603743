#!/bin/bash
# C2 A/B of library variants with parity, then SQ instruction counts per align_kernel<128> dispatch:
# the current library ("cur") and snapgpu/libsnapgpu_<v>.so for each named v, two alternating rounds
# of the bench line (no extras, oracle parity of 300k reads), then one rocprofv3 PMC pass each.
#   gpurun -- bash tools/gpu/ab_pmc.sh <tag> v1 v2 ...
export TMPDIR=/tmp SNAPGPU_TIMEOUT_S=90
T=${1:?tag}; shift
O=gpurun_out/$T; mkdir -p $O
L=$PWD/snap-rnaseq_amd/snapgpu
cp $L/libsnapgpu.so $L/libsnapgpu_cur.so
for i in 1 2; do
  for v in cur "$@"; do
    SNAPGPU_LIB=$L/libsnapgpu_$v.so timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-extras --cpu-sample 300000 \
      > $O/ab_${v}_$i.json 2> $O/ab_${v}_$i.err || { tail -5 $O/ab_${v}_$i.err; exit 1; }
  done
done
for v in cur "$@"; do
  SNAPGPU_LIB=$L/libsnapgpu_$v.so timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES \
    -d $O/pmc_$v -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-extras --no-cpu-baseline \
    > $O/pmc_$v.log 2>&1 || { tail -5 $O/pmc_$v.log; exit 1; }
done
python3 - $O cur "$@" <<'PY'
import csv, glob, json, sys
o = sys.argv[1]
for v in sys.argv[2:]:
    ds = [json.loads(open(f"{o}/ab_{v}_{i}.json").readline()) for i in (1, 2)]
    f = glob.glob(f"{o}/pmc_{v}/**/*counter_collection.csv", recursive=True)[0]
    acc = {}
    for r in csv.DictReader(open(f)):
        if "align_kernel<128, false>" in r["Kernel_Name"]:
            acc.setdefault(r["Counter_Name"], {}).setdefault(r["Dispatch_Id"], 0.0)
            acc[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    pm = {c: round(sum(d.values()) / len(d) / 1e6, 1) for c, d in sorted(acc.items()) if c != "SQ_WAVES"}
    print(v.ljust(7), "M reads/s", [round(d["value"] / 1e6, 3) for d in ds], "kernel ms/launch",
          [round(d["roofline"]["kernel_ms_per_launch"], 3) for d in ds], "mismatches", [d["parity"]["mismatches"] for d in ds],
          "M instr/dispatch", pm)
PY
