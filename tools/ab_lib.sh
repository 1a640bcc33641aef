#!/bin/bash
# Same-box A/B of two builds of libsift_hip.so: lib/libsift_hip_base.so (A)
# against the current lib/libsift_hip.so (B), tools/stage_bench.py alternating.
set -o pipefail
L=sift-gpu_amd/lib
cp $L/libsift_hip.so $L/libsift_hip_new.so
for r in 1 2 3; do
  for v in base new; do
    cp $L/libsift_hip_$v.so $L/libsift_hip.so
    timeout -k 10 120 python3 tools/stage_bench.py --reps 5 --tag $v || exit 1
  done
done
cp $L/libsift_hip_new.so $L/libsift_hip.so
