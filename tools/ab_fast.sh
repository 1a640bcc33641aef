#!/bin/bash
# A/B of the fast pyramids (pyramid_fast2.hip default vs SIFT_HIP_FAST_V1=1):
# tests/test_gpu_fast.py, then per-kernel times under rocprofv3 --kernel-trace
# and tools/stage_bench.py --fast for each.  Run on the GPU box.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_fast.py \
  > gpurun_out/fast2_test.log 2>&1 || { tail -30 gpurun_out/fast2_test.log; exit 1; }
for v in 0 1; do
  SIFT_HIP_FAST_V1=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -T -d gpurun_out/pf_v$v -o run \
    --output-format csv -- python3 tools/stage_bench.py --fast --reps 3 > gpurun_out/pf_v$v.log 2>&1 || exit 1
done
for v in 1 0 1 0; do
  SIFT_HIP_FAST_V1=$v timeout -k 10 120 python3 tools/stage_bench.py --fast --reps 5 --tag v1=$v || exit 1
done > gpurun_out/fast2_ab.txt 2>&1
