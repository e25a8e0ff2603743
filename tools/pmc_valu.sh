#!/bin/bash
# SQ_INSTS_VALU / SALU per align_kernel<128> launch for each library variant named
# (libsnapgpu_<name>.so; "cur" = libsnapgpu.so).  Measurement aid for A/B of code regions.
export TMPDIR=/tmp
L=$PWD/snap-rnaseq_amd/snapgpu
mkdir -p gpurun_out/pmcv
for v in "$@"; do
  if [ "$v" = cur ]; then lib=$L/libsnapgpu.so; else lib=$L/libsnapgpu_$v.so; fi
  SNAPGPU_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES -d gpurun_out/pmcv/$v -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmcv/$v.log 2>&1 || exit $?
done
python3 - "$@" <<'PY'
import csv, glob, sys
for v in sys.argv[1:]:
    f = glob.glob(f"gpurun_out/pmcv/{v}/**/run_counter_collection.csv", recursive=True) + glob.glob(f"gpurun_out/pmcv/{v}/run_counter_collection.csv")
    tot = {}
    for r in csv.DictReader(open(f[0])):
        if "align_kernel<128" in r["Kernel_Name"]:
            tot.setdefault(r["Counter_Name"], {}).setdefault(r["Dispatch_Id"], 0.0)
            tot[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    print(v, {k: round(sum(d.values()) / len(d) / 1e6, 1) for k, d in tot.items()})
PY
