#!/bin/bash
# Round 6: the single-end product path's host stages (parallel FASTQ parse, allocation-free filter,
# overlapped aligners, pinned CIGARs, parallel record writes): its GPU tests and the bench leg, then
# a 4-round alternating A/B of the pass-wide match probabilities (libsnapgpu_pgrp.so) -> gpurun_out/r06e/.
export TMPDIR=/tmp SNAPGPU_TIMEOUT_S=120
O=gpurun_out/r06e; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_single.py tests/test_sorted.py tests/test_contamination.py tests/test_cigar.py tests/test_capi.py -x -v -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --paired-pairs 0 --rna-pairs 0 > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench.json').readline()); s=d['single_e2e']; print('single', round(s['value']/1e6,3), s['stage_ms'], s['parity'].get('sha256_match'))"
L=$PWD/snap-rnaseq_amd/snapgpu
cp $L/libsnapgpu.so $L/libsnapgpu_cur.so
for i in 1 2 3 4; do
  for v in cur pgrp; do
    SNAPGPU_LIB=$L/libsnapgpu_$v.so timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-extras --cpu-sample 200000 \
      > $O/ab_${v}_$i.json 2> $O/ab_${v}_$i.err || { tail -5 $O/ab_${v}_$i.err; exit 1; }
  done
done
python3 - $O <<'PY' | tee $O/ab_summary.txt
import json, sys
o = sys.argv[1]
for v in ("cur", "pgrp"):
    ds = [json.loads(open(f"{o}/ab_{v}_{i}.json").readline()) for i in (1, 2, 3, 4)]
    ks = [d["roofline"]["kernel_ms_per_launch"] for d in ds]
    print(v.ljust(6), "M reads/s", [round(d["value"] / 1e6, 3) for d in ds], "kernel ms", [round(k, 3) for k in ks],
          "mean", round(sum(ks) / len(ks), 3), "mismatches", [d["parity"]["mismatches"] for d in ds])
PY
