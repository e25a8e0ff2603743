#!/bin/bash
# Round 4: seed_lookup_kernel with the seed-offset table and the seed tables' bucket ranges in LDS
# (two dependent global round trips off each lookup) -- GPU suite, A/B of the headline against the
# previous build (q8: four lanes per line, 35 VGPRs), and the serialised lookup pass
# (SNAPGPU_OVERLAP=0 kernel trace + FETCH_SIZE) of both.
export TMPDIR=/tmp SNAPGPU_TIMEOUT_S=120
O=gpurun_out/r04q; mkdir -p $O
L=$PWD/snap-rnaseq_amd/snapgpu
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
run() {  # name lib args...
  local n=$1 lib=$2; shift 2
  SNAPGPU_LIB=$lib timeout -k 10 400 python bench.py "$@" > $O/$n.json 2> $O/$n.err || { tail $O/$n.err; exit 1; }
}
C2="--steps 10 --warmup 2 --no-cpu-baseline --no-extras"
for i in 1 2 3; do
  run cur_$i $L/libsnapgpu.so $C2
  run q8_$i $L/libsnapgpu_q8.so $C2
done
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras"
for v in cur q8; do
  lib=$L/libsnapgpu_$v.so; [ $v = cur ] && lib=$L/libsnapgpu.so
  SNAPGPU_LIB=$lib SNAPGPU_OVERLAP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/skt_$v -o run --output-format csv -- $B > $O/skt_$v.log 2>&1 || exit $?
  SNAPGPU_LIB=$lib SNAPGPU_OVERLAP=0 timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d $O/spf_$v -o run --output-format csv -- $B > $O/spf_$v.log 2>&1 || exit $?
done
python3 - <<'PY' | tee gpurun_out/r04q/ab.txt
import csv, glob, json
def row(n):
    d = json.loads(open(f'gpurun_out/r04q/{n}.json').readline())
    return f"{n:9s} {d['value'] / 1e6:7.3f} M reads/s  kernel {d['roofline']['kernel_ms_per_launch']:7.2f} ms/launch"
for i in (1, 2, 3):
    for n in ("cur", "q8"):
        print(row(f'{n}_{i}'))
for v in ("cur", "q8"):
    ks = glob.glob(f"gpurun_out/r04q/skt_{v}/**/run_kernel_stats.csv", recursive=True)[0]
    ms = [float(r["AverageNs"]) / 1e6 for r in csv.DictReader(open(ks)) if "seed_lookup_kernel" in r["Name"]][0]
    f = glob.glob(f"gpurun_out/r04q/spf_{v}/**/run_counter_collection.csv", recursive=True)[0]
    per = {}
    for r in csv.DictReader(open(f)):
        if "seed_lookup_kernel" in r["Kernel_Name"]:
            per[r["Dispatch_Id"]] = per.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    fb = sum(per.values()) / len(per) * 1024
    print(v, f"serialised seed_lookup_kernel {ms:.3f} ms per 1M-read dispatch, FETCH {fb / 1e6:.0f} MB, {fb / ms / 1e6:.0f} GB/s")
PY
