#!/bin/bash
# The failing configuration of final_r04c (wave-history tests: two single-end tests, then the paired
# ones, one pytest process) twice, then the paired history test alone; outcomes only, no retry of a
# GPU fault (these are result comparisons).
export TMPDIR=/tmp SNAPGPU_TIMEOUT_S=90
O=gpurun_out/repro_hist; mkdir -p $O
for i in 1 2; do
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_paired.py -v -m gpu -k independent --timeout 200 --timeout-method thread > $O/both_$i.log 2>&1
  echo "both_$i rc=$?"; grep -E "PASSED|FAILED|Error" $O/both_$i.log | cut -c1-160
done
timeout -k 10 300 python -u -m pytest tests/test_paired.py -v -m gpu -k independent --timeout 200 --timeout-method thread > $O/paired_only.log 2>&1
echo "paired_only rc=$?"; grep -E "PASSED|FAILED|Error" $O/paired_only.log | cut -c1-160
exit 0
