#!/bin/bash
# Iteration check: the -m gpu suite, then exact- and fast-mode stage timings.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 120 python tools/stage_bench.py --tag exact > gpurun_out/stage_exact.log 2>&1 &&
timeout -k 10 120 python tools/stage_bench.py --fast --tag fast > gpurun_out/stage_fast.log 2>&1
rc=$?
echo "exit $rc"
exit $rc
