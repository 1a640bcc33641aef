#!/bin/bash
# Parity suite + per-stage timing (no CPU baseline): the inner-loop GPU check.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 180 python tools/stage_bench.py --tag quick "$@" > gpurun_out/stage.log 2>&1
rc=$?
echo "exit $rc"
exit $rc
