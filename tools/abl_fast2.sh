#!/bin/bash
# Phase ablation of pyramid_fast2.hip's scale kernel (SIFT_HIP_ABL bits: 1 row
# passes, 2 column-pass compute, 4 plane stores, 8 source fetch, 16 stage
# fill, unused by the DMA kernel), pyramid only (SIFT_HIP_PYR_ONLY=1: no detection on ablated planes).
set -o pipefail
mkdir -p gpurun_out
for m in 0 1 2 3 4 7 8 12 15 0; do
  echo "== $m"
  SIFT_HIP_PYR_ONLY=1 SIFT_HIP_ABL=$m timeout -k 10 120 python3 tools/stage_bench.py --fast --reps 5 --ignore-status \
    --tag abl$m || exit 1
done
