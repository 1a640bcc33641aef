#!/bin/bash
# Round 4: the fast pyramid's column passes on v_mfma_f32_16x16x4_f32 vs the VALU scatter (base).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
L=sift-gpu_amd/lib
cp $L/libsift_hip.so $L/libsift_hip_keep0.so
for V in $VARS; do
  cp $L/libsift_hip_$V.so $L/libsift_hip.so
  timeout -k 10 300 python -u -m pytest tests/test_gpu_fast.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/r4_mfma_fast_$V.log 2>&1; rc=$?
  cp $L/libsift_hip_keep0.so $L/libsift_hip.so
  echo "$V: $(tail -1 gpurun_out/r4_mfma_fast_$V.log)"
  [ $rc -eq 0 ] || { tail -30 gpurun_out/r4_mfma_fast_$V.log; exit 1; }
done
R=3 bash tools/ab_var.sh r4mfma base $VARS || exit 1
