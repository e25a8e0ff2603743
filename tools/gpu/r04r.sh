#!/bin/bash
# Round 4: what the align kernel's 5.2 KB/read of WRITE_SIZE is made of -- PMC FETCH_SIZE / WRITE_SIZE
# and time of the headline for: cur; cur with the forced-order radix sort off (SNAPGPU_RADIX_MIN huge:
# the ranked windows instead, no sort buffers in the arena); e6 (only 6 elements per read in LDS).
export TMPDIR=/tmp SNAPGPU_TIMEOUT_S=120
O=gpurun_out/r04r; mkdir -p $O
L=$PWD/snap-rnaseq_amd/snapgpu
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras"
for v in cur norad e6; do
  lib=$L/libsnapgpu.so; [ $v = e6 ] && lib=$L/libsnapgpu_e6.so
  rm_=""; [ $v = norad ] && rm_=1000000000
  SNAPGPU_LIB=$lib SNAPGPU_RADIX_MIN=$rm_ timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extras > $O/$v.json 2> $O/$v.err || { tail $O/$v.err; exit 1; }
  SNAPGPU_LIB=$lib SNAPGPU_RADIX_MIN=$rm_ timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d $O/pf_$v -o run --output-format csv -- $B > $O/pf_$v.log 2>&1 || exit $?
  SNAPGPU_LIB=$lib SNAPGPU_RADIX_MIN=$rm_ timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d $O/pw_$v -o run --output-format csv -- $B > $O/pw_$v.log 2>&1 || exit $?
done
python3 - <<'PY' | tee gpurun_out/r04r/traffic.txt
import csv, glob, json
for v in ("cur", "norad", "e6"):
    d = json.loads(open(f"gpurun_out/r04r/{v}.json").readline())
    out = {}
    for c, p in (("FETCH_SIZE", "pf"), ("WRITE_SIZE", "pw")):
        f = glob.glob(f"gpurun_out/r04r/{p}_{v}/**/run_counter_collection.csv", recursive=True)[0]
        per = {}
        for r in csv.DictReader(open(f)):
            if "align_kernel<128, false>" in r["Kernel_Name"]:
                per[r["Dispatch_Id"]] = per.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
        out[c] = round(sum(per.values()) / len(per) * 1024 / 1e6 / 1000, 3)
    print(f"{v:6s} {d['value'] / 1e6:7.3f} M reads/s  kernel {d['roofline']['kernel_ms_per_launch']:6.2f} ms  KB per read: {out}")
PY
