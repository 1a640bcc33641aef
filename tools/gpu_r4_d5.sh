#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
L=sift-gpu_amd/lib
cp $L/libsift_hip.so $L/libsift_hip_keep0.so
cp $L/libsift_hip_dperm5.so $L/libsift_hip.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "descriptor" \
    > gpurun_out/r4_d5.log 2>&1 || { tail -30 gpurun_out/r4_d5.log; cp $L/libsift_hip_keep0.so $L/libsift_hip.so; exit 1; }
echo "dperm5: $(tail -1 gpurun_out/r4_d5.log)"
cp $L/libsift_hip_keep0.so $L/libsift_hip.so
MODE=exact R=2 bash tools/ab_var.sh r4d5 dperm4 dperm5 || exit 1
R=2 bash tools/ab_bench_lib.sh dperm4 dperm5 2>&1 | tee gpurun_out/r4_d5_bench.txt || exit 1
R=2 bash tools/ab_single.sh dperm4 dperm5 || exit 1
