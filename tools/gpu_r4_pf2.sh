#!/bin/bash
# descriptor: gathers two batches ahead on the batch path (PF = 2) at 4 / 3 waves per SIMD vs the default
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
L=sift-gpu_amd/lib
cp $L/libsift_hip.so $L/libsift_hip_keep0.so
cp $L/libsift_hip_pf2w4.so $L/libsift_hip.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batch.py -x -q --timeout 120 --timeout-method thread -k "descriptor or headline" \
    > gpurun_out/r4_pf2.log 2>&1 || { tail -30 gpurun_out/r4_pf2.log; cp $L/libsift_hip_keep0.so $L/libsift_hip.so; exit 1; }
echo "pf2w4: $(tail -1 gpurun_out/r4_pf2.log)"
cp $L/libsift_hip_keep0.so $L/libsift_hip.so
MODE=exact R=2 bash tools/ab_var.sh r4pf2 dbase pf2w4 pf2w3 || exit 1
R=2 bash tools/ab_bench_lib.sh dbase pf2w4 pf2w3 2>&1 | tee gpurun_out/r4_pf2_bench.txt || exit 1
