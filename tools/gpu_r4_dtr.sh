#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batch.py -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r4_gpu_tests_dtr.log 2>&1 || { tail -40 gpurun_out/r4_gpu_tests_dtr.log; exit 1; }
tail -2 gpurun_out/r4_gpu_tests_dtr.log
MODE=exact R=3 bash tools/ab_var.sh r4dtr dbase dtr || exit 1
for r in 1 2; do
  for v in 2 5; do
    SIFT_HIP_ORIENT_SLOTS=$v timeout -k 10 120 python3 tools/stage_bench.py --reps 3 --tag slots$v >> gpurun_out/r4_orient_batch_ab.txt 2>&1 || exit 1
  done
done
grep -h "^{" gpurun_out/r4_orient_batch_ab.txt | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['tag'], d['total_ms'], d['stages_ms']['refine_orient'])"
