#!/bin/bash
# Round 4: GPU suite, a short C2 bench (headline + lookup roofline), then the rocprofv3 evidence
# (tools/gpu/prof.sh r04: kernel trace + PMC passes -> profiles/r04/summary.json).
O=gpurun_out/r04d; mkdir -p $O
export SNAPGPU_TIMEOUT_S=90
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --rna-pairs 0 --paired-pairs 0 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 - <<'PY'
import json; d=json.loads(open('gpurun_out/r04d/bench.json').readline())
lk=d['lookup_roofline']
print('value', round(d['value']/1e6,3), 'kernel_ms', round(d['roofline']['kernel_ms_per_launch'],2))
print('lookup', {k: lk.get(k) for k in ('kernel_ms_per_launch','achieved','frac','pass0_probes_per_read','probe_rate_frac_of_gather_peak','frac_of_measured_copy_peak')})
PY
bash tools/gpu/prof.sh r04 && python3 -c "
import json; d=json.load(open('profiles/r04/summary.json')); print(json.dumps(d)[:3000])"
