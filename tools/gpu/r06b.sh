#!/bin/bash
# Round 6: the C3 module (index upload with the wave-reduced bucket placement, the configs[4] RNA
# test at C3 scale) and the bucket-image tests -> gpurun_out/r06b/.
export TMPDIR=/tmp SNAPGPU_TIMEOUT_S=120
O=gpurun_out/r06b; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests/test_c3_scale.py tests/test_bucket_table.py -x -v -s -m gpu --timeout 900 --timeout-method thread > $O/c3_tests.log 2>&1 || { tail -40 $O/c3_tests.log; exit 1; }
grep -E "PASSED|FAILED|\[c3" $O/c3_tests.log | tail -30
