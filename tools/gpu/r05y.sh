#!/bin/bash
# Multi-block order sort (order_long.h): the tests of the ordered paths, the RNA sub-batch probe,
# then a kernel trace of the RNA leg (tools/rna_pmc_probe.py).
export TMPDIR=/tmp SNAPGPU_TIMEOUT_S=120
T=${1:?tag}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_order_long.py tests/test_paired.py tests/test_long_reads.py tests/test_rna_paired.py \
  tests/test_multihit.py -x -v -m gpu --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python -u tools/rna_sub_probe.py > $O/rna_sub.txt 2> $O/rna_sub.err || { tail $O/rna_sub.err; exit 1; }
cat $O/rna_sub.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 tools/rna_pmc_probe.py 100000 3 > $O/kt.json 2> $O/kt.log || exit 1
grep -E "order_|paired_kernel<256>|align_kernel<256, true>" $O/kt/run_kernel_stats.csv | cut -c1-160
