#!/bin/bash
# Kernel trace (no counters) of the exact-mode stage bench; per-kernel averages
# land in gpurun_out/te/summary.txt.
set -o pipefail
mkdir -p gpurun_out/te
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/te/trace -o run --output-format csv -- \
  python3 tools/stage_bench.py --reps 2 "$@" > gpurun_out/te/trace.log 2>&1 &&
python3 tools/trace_summary.py gpurun_out/te/trace/run_kernel_trace.csv > gpurun_out/te/summary.txt
