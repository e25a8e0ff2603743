#!/bin/bash
# rocprofv3 passes for the bench workload: kernel trace + stats, then PMC passes
# (FETCH_SIZE; SQ wave-state; instruction mix), each in its own run.
export TMPDIR=/tmp
OUT=gpurun_out/prof_${1:-r01}
mkdir -p $OUT
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- $B > $OUT/kt.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc1 -o run --output-format csv -- $B > $OUT/pmc1.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc1w -o run --output-format csv -- $B > $OUT/pmc1w.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -d $OUT/pmc2 -o run --output-format csv -- $B > $OUT/pmc2.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH -d $OUT/pmc3 -o run --output-format csv -- $B > $OUT/pmc3.log 2>&1 || exit $?
echo PROF_DONE
