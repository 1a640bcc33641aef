#!/bin/bash
# Descriptor-kernel iteration: parity tests that cover it, then the stage
# times of the exact path (tools/stage_bench.py) twice.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_batch.py > gpurun_out/desc_test.log 2>&1 || { tail -30 gpurun_out/desc_test.log; exit 1; }
tail -2 gpurun_out/desc_test.log
for r in 1 2; do
  timeout -k 10 120 python3 tools/stage_bench.py --reps 5 --tag run$r || exit 1
done
