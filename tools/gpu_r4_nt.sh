#!/bin/bash
# Round 4: non-temporal plane stores (fast pyramid: ntst; exact blur: ntblur)
# and padded plane pitch (pad32 / pad64) against the committed library (base).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
L=sift-gpu_amd/lib
cp $L/libsift_hip_ntst.so $L/libsift_hip.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_fast.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r4_nt_fast.log 2>&1 || { tail -30 gpurun_out/r4_nt_fast.log; cp $L/libsift_hip_base.so $L/libsift_hip.so; exit 1; }
echo "ntst: $(tail -1 gpurun_out/r4_nt_fast.log)"
cp $L/libsift_hip_base.so $L/libsift_hip.so
R=3 bash tools/ab_var.sh r4nt base ntst pad64 || exit 1
R=2 bash tools/ab_bench_lib.sh base pad32 pad64 ntblur 2>&1 | tee gpurun_out/r4_nt_bench.txt || exit 1
