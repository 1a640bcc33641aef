#!/bin/bash
# Fast-mode bring-up on one GPU: new-kernel tests first, then the whole GPU
# suite, then the bench.  Each GPU step has its own limit; stop at the first failure.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gpu_fast.py -x -v -s --timeout 200 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/fast.log 2>&1 &&
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/bench.log 2>&1
rc=$?
echo "exit $rc"
exit $rc
