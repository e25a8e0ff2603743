#!/bin/bash
# Round 4 bisect of the align-kernel time: the round-3 build and three round-4 commits (ab/<commit>:
# each with its own bench.py and library) against the current tree, C2 headline, alternating;
# then the paired leg of the current tree and of 3043e8d (before reads views).
export TMPDIR=/tmp
O=gpurun_out/r04i; mkdir -p $O
export SNAPGPU_TIMEOUT_S=90
run() {  # name dir args...
  local n=$1 d=$2; shift 2
  (cd $d && timeout -k 10 300 python bench.py "$@") > $O/$n.json 2> $O/$n.err || { tail $O/$n.err; exit 1; }
}
for i in 1 2; do
  run cur_$i . --steps 10 --warmup 2 --no-cpu-baseline --no-extras
  for c in r03 7cacbce 3f0aeb9 3043e8d; do run ${c}_$i ab/$c --steps 10 --warmup 2 --no-cpu-baseline --no-extras; done
done
run cur_paired . --steps 2 --warmup 1 --no-cpu-baseline --rna-pairs 0
run old_paired ab/3043e8d --steps 2 --warmup 1 --no-cpu-baseline --rna-pairs 0
python3 - <<'PY'
import json
for v in ('cur', 'r03', '7cacbce', '3f0aeb9', '3043e8d'):
    for i in (1, 2):
        d = json.loads(open(f'gpurun_out/r04i/{v}_{i}.json').readline())
        r = d['roofline']
        print(v, i, round(d['value'] / 1e6, 3), 'ms/step', round(d['ms_per_step'], 2), 'kernel', round(r['kernel_ms_per_launch'], 2), 'launch', round(r['launch_duration_ms'], 2))
for v in ('cur_paired', 'old_paired'):
    d = json.loads(open(f'gpurun_out/r04i/{v}.json').readline())
    p = d.get('paired') or d.get('extras', {}).get('paired')
    print(v, round(p['value'] / 1e6, 3), round(p['ms_per_batch'], 1), p.get('fallback_pairs'))
PY
