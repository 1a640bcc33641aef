#!/bin/bash
# Round 4: pyramid lazy window loads (lazy vs w4, fast mode) and the
# descriptor's speculative bin reads (dspec vs lazy, exact mode).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
L=sift-gpu_amd/lib
timeout -k 10 300 python -u -m pytest tests/test_gpu_fast.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r4_spec_fast.log 2>&1 || { tail -30 gpurun_out/r4_spec_fast.log; exit 1; }
tail -1 gpurun_out/r4_spec_fast.log
cp $L/libsift_hip.so $L/libsift_hip_keep0.so
for v in dspec8 dspec4 dspec2; do
  cp $L/libsift_hip_$v.so $L/libsift_hip.so
  timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "descriptor" \
    > gpurun_out/r4_spec_desc_$v.log 2>&1 || { tail -30 gpurun_out/r4_spec_desc_$v.log; cp $L/libsift_hip_keep0.so $L/libsift_hip.so; exit 1; }
  echo "$v: $(tail -1 gpurun_out/r4_spec_desc_$v.log)"
done
cp $L/libsift_hip_keep0.so $L/libsift_hip.so
R=3 bash tools/ab_var.sh r4lazy w4 lazy pad32 || exit 1
MODE=exact R=2 bash tools/ab_var.sh r4dspec lazy dspec8 dspec4 dspec2 pad32 || exit 1
