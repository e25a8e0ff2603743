#!/bin/bash
# Round 5: (1) the GPU tests of the long-read paths on the longest-first build (libsnapgpu_rna.so);
# (2) C2 A/B of the forced-mode prefilter builds (fB: FKM 5, fB4: FKM 4; both 4 waves/SIMD) against
# the current build at 5 and at 4 waves/SIMD (SNAPGPU_WAVES_PER_CU=16), parity on 300k reads;
# (3) instruction counts per align_kernel<128> dispatch of each build (SQ_INSTS_VALU / SALU / LDS).
export TMPDIR=/tmp SNAPGPU_TIMEOUT_S=90
O=gpurun_out/r05h; mkdir -p $O
L=$PWD/snap-rnaseq_amd/snapgpu
SNAPGPU_LIB=$L/libsnapgpu_rna.so timeout -k 10 600 python -u -m pytest tests/test_order_long.py tests/test_long_reads.py \
  tests/test_paired.py tests/test_rna_paired.py tests/test_multihit.py -x -v -m gpu --timeout 200 --timeout-method thread > $O/rna_tests.log 2>&1 || { tail -30 $O/rna_tests.log; exit 1; }
tail -1 $O/rna_tests.log
run() {   # name lib env-prefix round
  SNAPGPU_LIB=$L/libsnapgpu_$2.so $3 timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-extras --cpu-sample 300000 \
    > $O/ab_$1_$4.json 2> $O/ab_$1_$4.err || { tail -5 $O/ab_$1_$4.err; exit 1; }
}
cp $L/libsnapgpu.so $L/libsnapgpu_cur.so
for i in 1 2; do
  run cur cur "" $i; run cur4 cur "env SNAPGPU_WAVES_PER_CU=16" $i; run fB fB "" $i; run fB4 fB4 "" $i
done
python3 - $O <<'PY'
import json, sys
o = sys.argv[1]
for v in ("cur", "cur4", "fB", "fB4"):
    ds = [json.loads(open(f"{o}/ab_{v}_{i}.json").readline()) for i in (1, 2)]
    print(v.ljust(6), "M reads/s", [round(d["value"] / 1e6, 3) for d in ds], "kernel ms/launch",
          [round(d["roofline"]["kernel_ms_per_launch"], 3) for d in ds], "mismatches", [d["parity"]["mismatches"] for d in ds])
PY
for v in cur fB fB4; do
  SNAPGPU_LIB=$L/libsnapgpu_$v.so timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES \
    -d $O/pmc_$v -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-extras --no-cpu-baseline \
    > $O/pmc_$v.log 2>&1 || { tail -5 $O/pmc_$v.log; exit 1; }
done
python3 - $O <<'PY'
import csv, glob, sys
o = sys.argv[1]
for v in ("cur", "fB", "fB4"):
    f = glob.glob(f"{o}/pmc_{v}/**/*counter_collection.csv", recursive=True)[0]
    acc = {}
    for r in csv.DictReader(open(f)):
        if "align_kernel<128, false>" in r["Kernel_Name"]:
            acc.setdefault(r["Counter_Name"], {}).setdefault(r["Dispatch_Id"], 0.0)
            acc[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    print(v.ljust(5), {c: round(sum(d.values()) / len(d) / 1e6, 2) for c, d in sorted(acc.items())}, "M per dispatch")
PY
