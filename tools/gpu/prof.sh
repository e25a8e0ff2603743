#!/bin/bash
# rocprofv3 evidence for the bench workload, each pass in its own run:
#   kt   kernel trace + stats of the headline bench (bench.py --no-extras: every align_kernel<128>
#        dispatch is a timed-region one, so rocprof's average duration is the bench's launch
#        duration; the extras legs launch the same kernel on small chimeric-fallback batches)
#   pmc* FETCH_SIZE / WRITE_SIZE / SQ wave state / SQ instruction mix (one counter group per run,
#        headline only, so per-dispatch counters / reads per dispatch is per read)
# then tools/pmc_summary.py folds them into profiles/<tag>/summary.json + profiles/pmc_traffic.json.
#   gpurun -- bash tools/gpu/prof.sh <tag> [bench args...]
export TMPDIR=/tmp
TAG=${1:-r03}; shift
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 bench.py --no-extras --no-cpu-baseline "$@" > $OUT/bench_kt.json 2> $OUT/kt.log || exit $?
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras $*"
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc1 -o run --output-format csv -- $B > $OUT/pmc1.log 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc1w -o run --output-format csv -- $B > $OUT/pmc1w.log 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -d $OUT/pmc2 -o run --output-format csv -- $B > $OUT/pmc2.log 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_THREAD_CYCLES_VALU -d $OUT/pmc3 -o run --output-format csv -- $B > $OUT/pmc3.log 2>&1 || exit $?
# seed_lookup_kernel with the two streams' pass sets serialised (SNAPGPU_OVERLAP=0): its dispatch
# durations are its own, so FETCH_SIZE / duration is a clean HBM rate for the lookups
SNAPGPU_OVERLAP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/serial_kt -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-extras --no-cpu-baseline "$@" > $OUT/serial_kt.json 2> $OUT/serial_kt.log || exit $?
SNAPGPU_OVERLAP=0 timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d $OUT/serial_pmc -o run --output-format csv -- $B > $OUT/serial_pmc.log 2>&1 || exit $?
python3 tools/pmc_summary.py $OUT profiles/$TAG && echo PROF_DONE
