#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
L=sift-gpu_amd/lib
cp $L/libsift_hip.so $L/libsift_hip_keep0.so
cp $L/libsift_hip_o24.so $L/libsift_hip.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batch.py -x -q --timeout 200 --timeout-method thread \
    > gpurun_out/r4_o24.log 2>&1 || { tail -30 gpurun_out/r4_o24.log; cp $L/libsift_hip_keep0.so $L/libsift_hip.so; exit 1; }
echo "o24: $(tail -1 gpurun_out/r4_o24.log)"
cp $L/libsift_hip_keep0.so $L/libsift_hip.so
MODE=exact R=2 bash tools/ab_var.sh r4o24 base o24 || exit 1
R=3 bash tools/ab_bench_lib.sh base o24 2>&1 | tee gpurun_out/r4_o24_bench.txt || exit 1
R=2 bash tools/ab_single.sh base o24 || exit 1
