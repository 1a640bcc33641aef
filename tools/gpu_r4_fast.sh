#!/bin/bash
# GPU call: fast-mode tests, then the fast pyramid's stage time (product build).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_fast.py -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r4_fast_tests.log 2>&1 || { tail -40 gpurun_out/r4_fast_tests.log; exit 1; }
tail -3 gpurun_out/r4_fast_tests.log
for i in 1 2 3; do
  timeout -k 10 120 python3 tools/stage_bench.py --fast --reps 5 --tag tri4_$i || exit 1
done
