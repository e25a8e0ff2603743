#!/bin/bash
# Instruction-fetch evidence for align_kernel<128> (73.7 KB of code): the counters this pool's
# rocprofv3 offers, then one PMC pass of the SQC instruction-cache counters over the headline bench.
export TMPDIR=/tmp SNAPGPU_TIMEOUT_S=120
O=gpurun_out/icache; mkdir -p $O
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1
grep -o "SQC_ICACHE[A-Z_]*\|SQ_IFETCH[A-Z_]*\|SQ_WAIT_INST[A-Z_]*\|SQ_INST_LEVEL[A-Z_]*" $O/counters.txt | sort -u > $O/icache_counters.txt
cat $O/icache_counters.txt
C=$(grep -x "SQC_ICACHE_HITS\|SQC_ICACHE_MISSES\|SQ_IFETCH\|SQC_ICACHE_MISSES_DUPLICATE" $O/icache_counters.txt | tr '\n' ' ')
[ -n "$C" ] || { echo "no icache counters"; exit 0; }
timeout -s KILL 180 rocprofv3 --pmc $C -d $O/pmc -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/icache/pmc/**/run_counter_collection.csv", recursive=True)[0]
per = {}
for r in csv.DictReader(open(f)):
    if "align_kernel<128, false>" in r["Kernel_Name"]:
        d = per.setdefault(r["Counter_Name"], {})
        d[r["Dispatch_Id"]] = d.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
print({k: round(sum(v.values()) / len(v) / 1e6, 1) for k, v in per.items()}, "per read (1M-read dispatches)")
PY
