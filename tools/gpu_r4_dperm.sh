#!/bin/bash
# Round 4: descriptor bin bytes generated in owner-slot order by v_perm byte
# tables, invalid corners carried as +0.0 (dperm) vs the committed kernel (base).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
L=sift-gpu_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batch.py -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/r4_dperm_tests.log 2>&1 || { tail -30 gpurun_out/r4_dperm_tests.log; exit 1; }
tail -1 gpurun_out/r4_dperm_tests.log
MODE=exact R=2 bash tools/ab_var.sh r4dperm base dperm || exit 1
R=2 bash tools/ab_bench_lib.sh base dperm 2>&1 | tee gpurun_out/r4_dperm_bench.txt || exit 1
