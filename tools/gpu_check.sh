#!/bin/bash
# One GPU session: smoke -> parity tests -> short bench.  Each GPU step has its
# own time limit; the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 600 python bench.py --steps 5 --warmup 2 > gpurun_out/bench.log 2>&1
rc=$?
echo "exit $rc"
exit $rc
