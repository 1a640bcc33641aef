#!/bin/bash
# Per-kernel times of the fast pyramid under SIFT_HIP_ABL settings (see
# tools/abl_fast2.sh), pyramid only.  usage: tools/abl_trace.sh m1 m2 ...
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for m in "$@"; do
  SIFT_HIP_PYR_ONLY=1 SIFT_HIP_ABL=$m timeout -k 10 200 rocprofv3 --kernel-trace --stats -T -d gpurun_out/abl_$m -o run \
    --output-format csv -- python3 tools/stage_bench.py --fast --reps 3 --ignore-status > gpurun_out/abl_$m.log 2>&1 || exit 1
done
