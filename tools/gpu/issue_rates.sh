#!/bin/bash
# Issue capacity of the CU's pipes (tools/gpu/issue_rates.hip, built in-tree as tools/gpu/issue_rates):
# -> gpurun_out/issue_rates.json (committed as profiles/r05/issue_rates.json)
mkdir -p gpurun_out
[ -x tools/gpu/issue_rates ] || hipcc --offload-arch=gfx950 -O3 -o tools/gpu/issue_rates tools/gpu/issue_rates.hip || exit 1
timeout -k 10 120 tools/gpu/issue_rates > gpurun_out/issue_rates.json || exit $?
python3 -c "
import json; d = json.load(open('gpurun_out/issue_rates.json'))
for r in d['rates']: print(r['instruction'][:40].ljust(40), ' '.join('%s %.2f/%.2f' % (k, v['cycles_per_instr_per_wave'], v['cycles_per_instr_per_cu']) for k, v in r.items() if k.startswith('wpc')))"
