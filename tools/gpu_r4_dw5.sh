#!/bin/bash
# descriptor: 5 waves per SIMD on the batch path (96 VGPRs, spills outside the sample loop) vs 4
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
L=sift-gpu_amd/lib
cp $L/libsift_hip.so $L/libsift_hip_keep0.so
cp $L/libsift_hip_dw5.so $L/libsift_hip.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batch.py -x -q --timeout 120 --timeout-method thread -k "descriptor or headline" \
    > gpurun_out/r4_dw5.log 2>&1 || { tail -30 gpurun_out/r4_dw5.log; cp $L/libsift_hip_keep0.so $L/libsift_hip.so; exit 1; }
echo "dw5: $(tail -1 gpurun_out/r4_dw5.log)"
cp $L/libsift_hip_keep0.so $L/libsift_hip.so
MODE=exact R=2 bash tools/ab_var.sh r4dw5 dw4 dw5 || exit 1
R=2 bash tools/ab_bench_lib.sh dw4 dw5 2>&1 | tee gpurun_out/r4_dw5_bench.txt || exit 1
