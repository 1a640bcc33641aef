#!/bin/bash
# Fast-pyramid ablation timings (diagnostic builds via SIFT_FAST_ABLATE).
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_fast.py -x -q --timeout 200 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/fast.log 2>&1 || exit 1
for a in 0 1 2 4 8 6 7 15; do
  SIFT_FAST_ABLATE=$a timeout -k 10 120 python tools/stage_bench.py --fast --tag abl$a >> gpurun_out/ablate.log 2>&1 || exit 1
done
echo done
