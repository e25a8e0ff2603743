#!/bin/bash
# Round 4: C3 chunk size (SNAPGPU_CHUNK_READS: reads per align launch; the C3 step is 6.25M reads, so
# 1M-read chunks give ~7 launches per step and as many persistent-kernel tails) and a compiler
# variant (noatomopt: -amdgpu-atomic-optimizer-strategy=None), C2 three alternating rounds.
export TMPDIR=/tmp SNAPGPU_TIMEOUT_S=120
O=gpurun_out/r04t; mkdir -p $O
L=$PWD/snap-rnaseq_amd/snapgpu
C3="--workload c3 --steps 3 --warmup 1 --no-cpu-baseline --no-extras"
for ch in 1048576 2097152 3200000; do
  SNAPGPU_CHUNK_READS=$ch timeout -k 10 400 python bench.py $C3 > $O/c3_ch$ch.json 2> $O/c3_ch$ch.err || { tail $O/c3_ch$ch.err; exit 1; }
done
C2="--steps 10 --warmup 2 --no-cpu-baseline --no-extras"
for i in 1 2 3; do
  timeout -k 10 300 python bench.py $C2 > $O/cur_$i.json 2> $O/cur_$i.err || exit 1
  SNAPGPU_LIB=$L/libsnapgpu_noatomopt.so timeout -k 10 300 python bench.py $C2 > $O/noatomopt_$i.json 2> $O/noatomopt_$i.err || exit 1
done
python3 - <<'PY' | tee gpurun_out/r04t/ab.txt
import json
def row(n):
    d = json.loads(open(f'gpurun_out/r04t/{n}.json').readline())
    return f"{n:14s} {d['value'] / 1e6:7.3f} M reads/s  kernel {d['roofline']['kernel_ms_per_launch']:7.2f} ms/launch  ms/step {d['ms_per_step']:.1f}"
for ch in (1048576, 2097152, 3200000):
    print(row(f'c3_ch{ch}'))
for i in (1, 2, 3):
    for n in ("cur", "noatomopt"):
        print(row(f'{n}_{i}'))
PY
