#!/bin/bash
# rocprofv3 evidence for the RNA paired leg (verdict r3 item 5): kernel trace, FETCH_SIZE,
# WRITE_SIZE, SQ wave state and instruction mix of align_kernel<256,*> and paired_kernel<256>,
# each pass its own run over tools/rna_pmc_probe.py (100k 2x150 pairs, 3 calls); then
# tools/rna_pmc_summary.py -> profiles/<tag>/rna/summary.json.
#   gpurun -- bash tools/gpu/rna_pmc.sh <tag>
export TMPDIR=/tmp SNAPGPU_TIMEOUT_S=120
TAG=${1:-r04}
OUT=gpurun_out/rnapmc_$TAG
mkdir -p $OUT
P="python3 tools/rna_pmc_probe.py 100000 3"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- $P > $OUT/kt.json 2> $OUT/kt.log || exit $?
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc1 -o run --output-format csv -- $P > $OUT/pmc1.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc1w -o run --output-format csv -- $P > $OUT/pmc1w.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -d $OUT/pmc2 -o run --output-format csv -- $P > $OUT/pmc2.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_THREAD_CYCLES_VALU -d $OUT/pmc3 -o run --output-format csv -- $P > $OUT/pmc3.log 2>&1 || exit $?
python3 tools/rna_pmc_summary.py $OUT profiles/$TAG/rna && echo RNA_PMC_DONE
