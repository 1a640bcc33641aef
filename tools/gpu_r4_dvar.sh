#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
L=sift-gpu_amd/lib
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "descriptor" \
    > gpurun_out/r4_dvar3.log 2>&1 || { tail -30 gpurun_out/r4_dvar3.log; exit 1; }
echo "dperm3: $(tail -1 gpurun_out/r4_dvar3.log)"
MODE=exact R=2 bash tools/ab_var.sh r4dvar3 base dmicro dperm2 dperm3 || exit 1
R=2 bash tools/ab_bench_lib.sh base dperm2 dperm3 2>&1 | tee gpurun_out/r4_dvar3_bench.txt || exit 1
