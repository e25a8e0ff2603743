#!/bin/bash
# Round 6: the N-rank launch on one GPU (2 ranks share GPU 0: the self-launch, one index build per
# node through /dev/shm, the host thread budget split by LOCAL_WORLD_SIZE) -> gpurun_out/r06n/.
export TMPDIR=/tmp SNAPGPU_TIMEOUT_S=120
O=gpurun_out/r06n; mkdir -p $O
timeout -k 10 600 python bench.py --gpus 2 --steps 5 --warmup 1 --no-cpu-baseline --paired-pairs 0 --rna-pairs 0 --single-reads 0 > $O/bench_g2.json 2> $O/bench_g2.err || { tail -20 $O/bench_g2.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench_g2.json').readline()); print('n_gpus', d['n_gpus'], 'value', round(d['value']/1e6,3), [ (r['rank'], round(r['reads_per_s']/1e6,3), r['index_upload_s'], r['index_built_here'], r['index_attached']) for r in d['config']['per_rank']])"
