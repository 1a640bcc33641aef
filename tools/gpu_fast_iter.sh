#!/bin/bash
# Fast-pyramid iteration: fast-mode tests, then stage timings and a kernel trace.
set -o pipefail
mkdir -p gpurun_out/pf
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gpu_fast.py -x -q -s --timeout 200 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/fast.log 2>&1 &&
timeout -k 10 120 python tools/stage_bench.py --fast --tag fast > gpurun_out/stage_fast.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pf/trace -o run --output-format csv -- \
  python3 tools/stage_bench.py --fast --reps 2 > gpurun_out/pf/trace.log 2>&1
rc=$?
echo "exit $rc"
exit $rc
