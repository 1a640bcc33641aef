#!/bin/bash
# GPU call: full -m gpu suite, then one-image latency with the bucketed
# orientation (default) vs orient_kernel (SIFT_HIP_ORIENT_SLOTS=1), then a
# kernel trace of the one-image loop.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r4_gpu_tests.log 2>&1 || { tail -40 gpurun_out/r4_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r4_gpu_tests.log
for r in 1 2 3; do
  for v in 5 1; do
    echo -n "slots=$v " >> gpurun_out/r4_orient_ab.txt
    SIFT_HIP_ORIENT_SLOTS=$v timeout -k 10 120 python3 tools/single_trace.py --reps 200 >> gpurun_out/r4_orient_ab.txt 2>/dev/null || exit 1
  done
done
cat gpurun_out/r4_orient_ab.txt
timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace --stats -T -d gpurun_out/r4_single -o run --output-format csv -- \
  python3 tools/single_trace.py --reps 20 > gpurun_out/r4_single.log 2>&1 || exit 1
python3 tools/trace_summary.py $(ls gpurun_out/r4_single/*kernel_trace.csv gpurun_out/r4_single/*/*kernel_trace.csv 2>/dev/null | head -1) > gpurun_out/r4_single_summary.txt; head -30 gpurun_out/r4_single_summary.txt
