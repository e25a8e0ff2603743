#!/bin/bash
# Round 6: the default bench line (with the new single_e2e leg and the RNA roofline in slot-probe
# units) and the C3 line with its RNA leg (configs[4] at C3 scale, builder-run rate) -> gpurun_out/r06c/.
export TMPDIR=/tmp SNAPGPU_TIMEOUT_S=120
O=gpurun_out/r06c; mkdir -p $O
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench.json').readline()); s=d['single_e2e']; r=d['rna_paired']; print('bench', round(d['value']/1e6,3), 'single', round(s['value']/1e6,3), s['stage_ms'], s['parity'].get('sha256_match'), 'rna', round(r['value']/1e6,3), r['roofline']['frac'], r['roofline']['per_read'])"
timeout -k 10 900 python bench.py --workload c3 --steps 3 --warmup 1 --paired-pairs 0 --single-reads 0 --rna-pairs 100000 > $O/c3_rna_bench.json 2> $O/c3_rna_bench.err || { tail $O/c3_rna_bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/c3_rna_bench.json').readline()); r=d['rna_paired']; print('c3', round(d['value']/1e6,3), 'upload_s', d['config']['index_upload_s'], 'rna', round(r['value']/1e6,3), r['stage_ms'], r['records'])"
