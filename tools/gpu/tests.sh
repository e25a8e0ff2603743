#!/bin/bash
# CIGAR / SAM GPU tests (tests/test_cigar.py), then the whole GPU suite.  Run from the repo root.
mkdir -p gpurun_out
export SNAPGPU_TIMEOUT_S=90
timeout -k 10 300 python -u -m pytest tests/test_cigar.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/cigar_tests.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit $?
