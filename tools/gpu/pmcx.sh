#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of align_kernel<128> per variant (one counter pass per run):
#   bash tools/gpu/pmcx.sh <tag> <variant...>
export TMPDIR=/tmp
TAG=$1; shift
L=$PWD/snap-rnaseq_amd/snapgpu
for v in "$@"; do
  if [ "$v" = cur ]; then lib=$L/libsnapgpu.so; else lib=$L/libsnapgpu_$v.so; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    SNAPGPU_LIB=$lib timeout -s KILL 180 rocprofv3 --pmc $c -d gpurun_out/$TAG/pmc_${v}_$c -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/$TAG/pmc_${v}_$c.log 2>&1 || { tail -5 gpurun_out/$TAG/pmc_${v}_$c.log; exit 1; }
  done
done
python3 - $TAG "$@" <<'PY'
import csv, glob, sys
tag, vs = sys.argv[1], sys.argv[2:]
for v in vs:
    out = []
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        f = glob.glob(f"gpurun_out/{tag}/pmc_{v}_{c}/**/*counter_collection.csv", recursive=True)
        tot, n = 0.0, 0
        for row in csv.DictReader(open(f[0])):
            if "align_kernel<128, false>" in row.get("Kernel_Name", "") and row.get("Counter_Name") == c:
                tot += float(row["Counter_Value"]); n += 1
        out.append(f"{c} {tot / max(n, 1) / 1e6:.1f} (units as counted) per dispatch over {n} dispatch rows")
    print(v, "; ".join(out))
PY
