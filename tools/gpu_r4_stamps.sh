#!/bin/bash
# GPU call: product fast-pyramid time, then the stamps build's per-role split.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python3 tools/stage_bench.py --fast --reps 5 --tag product > gpurun_out/r4_stamps_product.txt 2>&1 || { tail -20 gpurun_out/r4_stamps_product.txt; exit 1; }
timeout -k 10 180 python3 -u tools/tri_stamps.py --reps 5 --json gpurun_out/r4_tri_stamps.json > gpurun_out/r4_tri_stamps.txt 2>&1 || { tail -20 gpurun_out/r4_tri_stamps.txt; exit 1; }
cat gpurun_out/r4_stamps_product.txt gpurun_out/r4_tri_stamps.txt
