#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r4_gpu_tests_b.log 2>&1 || { tail -40 gpurun_out/r4_gpu_tests_b.log; exit 1; }
tail -2 gpurun_out/r4_gpu_tests_b.log
R=3 bash tools/ab_single.sh r4dsplit dbase dsplit || exit 1
timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace --stats -T -d gpurun_out/r4_single_c -o run --output-format csv -- \
  python3 tools/single_trace.py --reps 20 > gpurun_out/r4_single_c.log 2>&1 || exit 1
python3 tools/trace_summary.py gpurun_out/r4_single_c/run_kernel_trace.csv | head -8
