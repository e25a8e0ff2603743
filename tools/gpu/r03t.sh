#!/bin/bash
# The RNA paired product path at human-genome scale: bench.py --workload c3 with its extras (the RNA leg
# builds its 2,000-gene GTF and transcriptome on the 3.1 Gb / 25-contig C3 genome); no reference digest
# exists at this scale (the compiled reference needs more RAM than the build container has)
mkdir -p gpurun_out/r03t
export SNAPGPU_TIMEOUT_S=120
timeout -k 10 900 python bench.py --workload c3 --steps 2 --warmup 1 --paired-pairs 0 --no-cpu-baseline > gpurun_out/r03t/c3_rna.json 2> gpurun_out/r03t/c3_rna.err || { tail -5 gpurun_out/r03t/c3_rna.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/r03t/c3_rna.json').readline()); r=d['rna_paired']; print('c3', round(d['value']/1e6,3), 'rna', round(r['value']/1e6,3), r['stage_ms'], r['records'], r['parity'])"
