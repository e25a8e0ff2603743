#!/bin/bash
# Round 4: non-temporal loads for the streaming reads of align_kernel<128> (nt: genome plane
# windows, bucket lines, read bases / qualities, seed records) so the element arena's lines stay in
# L2 longer -- A/B time (C2, three alternating rounds) and FETCH_SIZE / WRITE_SIZE per read of both;
# unib: the success step's branches on f64 comparisons made wave-uniform (readfirstlane).
export TMPDIR=/tmp SNAPGPU_TIMEOUT_S=120
O=gpurun_out/r04n; mkdir -p $O
L=$PWD/snap-rnaseq_amd/snapgpu
run() {  # name lib args...
  local n=$1 lib=$2; shift 2
  SNAPGPU_LIB=$lib timeout -k 10 400 python bench.py "$@" > $O/$n.json 2> $O/$n.err || { tail $O/$n.err; exit 1; }
}
C2="--steps 10 --warmup 2 --no-cpu-baseline --no-extras"
for i in 1 2 3; do
  run cur_$i $L/libsnapgpu.so $C2
  run nt_$i $L/libsnapgpu_nt.so $C2
  run unib_$i $L/libsnapgpu_unib.so $C2
done
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras"
for v in cur nt; do
  lib=$L/libsnapgpu_$v.so; [ $v = cur ] && lib=$L/libsnapgpu.so
  SNAPGPU_LIB=$lib timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d $O/pf_$v -o run --output-format csv -- $B > $O/pf_$v.log 2>&1 || exit $?
  SNAPGPU_LIB=$lib timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d $O/pw_$v -o run --output-format csv -- $B > $O/pw_$v.log 2>&1 || exit $?
done
python3 - <<'PY' | tee gpurun_out/r04n/ab.txt
import csv, glob, json
def row(n):
    d = json.loads(open(f'gpurun_out/r04n/{n}.json').readline())
    return f"{n:8s} {d['value'] / 1e6:7.3f} M reads/s  kernel {d['roofline']['kernel_ms_per_launch']:7.2f} ms/launch"
for i in (1, 2, 3):
    for n in ("cur", "nt", "unib"):
        print(row(f'{n}_{i}'))
for v in ("cur", "nt"):
    out = {}
    for c, p in (("FETCH_SIZE", "pf"), ("WRITE_SIZE", "pw")):
        f = glob.glob(f"gpurun_out/r04n/{p}_{v}/**/run_counter_collection.csv", recursive=True)[0]
        per = {}
        for r in csv.DictReader(open(f)):
            if "align_kernel<128, false>" in r["Kernel_Name"]:
                per[r["Dispatch_Id"]] = per.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
        out[c] = round(sum(per.values()) / len(per) * 1024 / 1e6 / 1000, 3)   # KiB per 1M-read dispatch -> KB per read
    print(v, "KB per read (1M-read dispatches):", out)
PY
