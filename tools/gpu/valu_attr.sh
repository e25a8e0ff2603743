#!/bin/bash
# Dynamic instruction attribution: SQ_INSTS_* of align_kernel<128,false> per read for the
# production build and for variants that execute one region twice (tools/build_variant.sh
# dprob / dlvf / dchain); the difference is that region's dynamic count.
export TMPDIR=/tmp
mkdir -p gpurun_out/va
L=$PWD/snap-rnaseq_amd/snapgpu
VARS=${*:-libsnapgpu.so libsnapgpu_dprob.so libsnapgpu_dlvf.so libsnapgpu_dchain.so}
for v in $VARS; do
  SNAPGPU_LIB=$L/$v timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES -d gpurun_out/va/$v -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/va/$v.log 2>&1 || exit $?
done
VARS="$VARS" python3 - <<'PY'
import csv, glob, collections, os
for v in os.environ["VARS"].split():
    f = glob.glob(f"gpurun_out/va/{v}/**/run_counter_collection.csv", recursive=True)[0]
    c = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        if "align_kernel<128, false>" in r["Kernel_Name"]:
            c[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    print(v, {k: round(sum(d.values()) / len(d) / 1e6, 1) for k, d in c.items()}, "per read (1M-read dispatches)")
PY
