#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_fast.py -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r4_fast_tests_v3.log 2>&1 || { tail -40 gpurun_out/r4_fast_tests_v3.log; exit 1; }
tail -2 gpurun_out/r4_fast_tests_v3.log
R=3 bash tools/ab_var.sh r4v3 w4 v3 || exit 1
