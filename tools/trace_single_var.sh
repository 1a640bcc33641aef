#!/bin/bash
# one-image kernel traces of lib/libsift_hip_<name>.so variants (tools/rocpd_kernels.py reads them)
# usage: bash tools/trace_single_var.sh <name>...
set -e
L=sift-gpu_amd/lib
cp $L/libsift_hip.so $L/libsift_hip_keep.so
for n in "$@"; do
  cp $L/libsift_hip_$n.so $L/libsift_hip.so
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/ot_$n -o run -- python3 tools/single_trace.py --reps 50 > gpurun_out/ot_$n.log 2>&1
  grep latency gpurun_out/ot_$n.log
done
cp $L/libsift_hip_keep.so $L/libsift_hip.so
