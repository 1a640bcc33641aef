#!/bin/bash
# descriptor: PF = 2 loop unrolled by two (Loc buffers swap, no copies; no ballot) vs the committed form
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
L=sift-gpu_amd/lib
cp $L/libsift_hip.so $L/libsift_hip_keep0.so
cp $L/libsift_hip_dunr.so $L/libsift_hip.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batch.py -x -q --timeout 120 --timeout-method thread -k "descriptor or headline" \
    > gpurun_out/r4_dunr.log 2>&1 || { tail -30 gpurun_out/r4_dunr.log; cp $L/libsift_hip_keep0.so $L/libsift_hip.so; exit 1; }
echo "dunr: $(tail -1 gpurun_out/r4_dunr.log)"
cp $L/libsift_hip_keep0.so $L/libsift_hip.so
MODE=exact R=2 bash tools/ab_var.sh r4dunr dcur dunr || exit 1
R=2 bash tools/ab_bench_lib.sh dcur dunr 2>&1 | tee gpurun_out/r4_dunr_bench.txt || exit 1
R=2 bash tools/ab_single.sh dcur dunr || exit 1
