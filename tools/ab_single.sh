#!/bin/bash
# One-image latency (tools/single_trace.py) of each lib/libsift_hip_<name>.so,
# alternating, R rounds (default 3).
# usage: tools/ab_single.sh <tag> <name>...
set -o pipefail
TAG=$1; shift
L=sift-gpu_amd/lib
O=gpurun_out/single_$TAG
mkdir -p $O
cp $L/libsift_hip.so $L/libsift_hip_keep.so
for r in $(seq ${R:-3}); do
  for n in "$@"; do
    cp $L/libsift_hip_$n.so $L/libsift_hip.so
    echo -n "$n " >> $O/ab.txt
    timeout -k 10 120 python3 tools/single_trace.py --reps 200 >> $O/ab.txt 2>> $O/stderr.txt || { echo "var $n failed"; tail -5 $O/ab.txt; cp $L/libsift_hip_keep.so $L/libsift_hip.so; exit 1; }
  done
done
cp $L/libsift_hip_keep.so $L/libsift_hip.so
cat $O/ab.txt
