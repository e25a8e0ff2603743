#!/bin/bash
# Write-traffic A/B of align_kernel<128> (verdict r5 #3): the current library ("cur") against
# snapgpu/libsnapgpu_<v>.so for each named v -- two alternating bench runs each (C2, no extras,
# 300k-read oracle parity), then per variant one PMC pass of WRITE_SIZE + the SQ memory-instruction
# counters and one of FETCH_SIZE, summed over the align_kernel<128> dispatches and divided by the
# reads they aligned.  -> gpurun_out/<tag>/.
#   gpurun -- bash tools/gpu/ab_writes.sh <tag> v1 v2 ...
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
  B="python3 bench.py --steps 2 --warmup 1 --no-extras --no-cpu-baseline"
  SNAPGPU_LIB=$L/libsnapgpu_$v.so timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_FLAT SQ_WAVES \
    -d $O/pmcw_$v -o run --output-format csv -- $B > $O/pmcw_$v.log 2>&1 || { tail -5 $O/pmcw_$v.log; exit 1; }
  SNAPGPU_LIB=$L/libsnapgpu_$v.so timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE \
    -d $O/pmcf_$v -o run --output-format csv -- $B > $O/pmcf_$v.log 2>&1 || { tail -5 $O/pmcf_$v.log; exit 1; }
done
python3 - $O cur "$@" <<'PY' | tee $O/summary.txt
import csv, glob, json, sys
o = sys.argv[1]
for v in sys.argv[2:]:
    ds = [json.loads(open(f"{o}/ab_{v}_{i}.json").readline()) for i in (1, 2)]
    reads = ds[0]["roofline"]["reads_per_launch"]
    acc = {}
    for d in ("pmcw", "pmcf"):
        f = glob.glob(f"{o}/{d}_{v}/**/*counter_collection.csv", recursive=True)[0]
        for r in csv.DictReader(open(f)):
            if "align_kernel<128, false>" in r["Kernel_Name"]:
                acc.setdefault(r["Counter_Name"], {}).setdefault(r["Dispatch_Id"], 0.0)
                acc[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    # FETCH_SIZE / WRITE_SIZE are KiB per dispatch: bytes per read = KiB * 1024 / reads (uncorrected)
    per = {(c + "_B" if c.endswith("_SIZE") else c): round(sum(x.values()) / len(x) * (1024 if c.endswith("_SIZE") else 1) / reads, 2)
           for c, x in sorted(acc.items()) if c != "SQ_WAVES"}
    print(v.ljust(8), "M reads/s", [round(d["value"] / 1e6, 3) for d in ds], "kernel ms/launch",
          [round(d["roofline"]["kernel_ms_per_launch"], 3) for d in ds], "mismatches", [d["parity"]["mismatches"] for d in ds],
          "per read", per)
PY
