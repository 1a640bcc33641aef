#!/bin/bash
# exact scatter blur: two source rows per loop step for w = 12, 18 (br2) vs one (bref); parity of the blur planes first
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
L=sift-gpu_amd/lib
cp $L/libsift_hip.so $L/libsift_hip_keep0.so
cp $L/libsift_hip_br2.so $L/libsift_hip.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batch.py -x -q --timeout 120 --timeout-method thread -k "blur or headline or scatter" \
    > gpurun_out/r4_br2.log 2>&1 || { tail -30 gpurun_out/r4_br2.log; cp $L/libsift_hip_keep0.so $L/libsift_hip.so; exit 1; }
echo "br2: $(tail -1 gpurun_out/r4_br2.log)"
cp $L/libsift_hip_keep0.so $L/libsift_hip.so
MODE=exact R=2 bash tools/ab_var.sh r4br2 bref br2 || exit 1
R=2 bash tools/ab_bench_lib.sh bref br2 2>&1 | tee gpurun_out/r4_br2_bench.txt || exit 1
