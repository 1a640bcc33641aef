#!/bin/bash
# Times the SIFT_FLAG_FAST pyramid of each lib/libsift_hip_abl<N>.so
# (tools/build_abl.sh), twice each, alternating.  usage: tools/ab_abl.sh tag N...
set -o pipefail
TAG=$1; shift
L=sift-gpu_amd/lib
O=gpurun_out/abl_$TAG
mkdir -p $O
cp $L/libsift_hip.so $L/libsift_hip_keep.so
for r in 1 2; do
  for n in "$@"; do
    cp $L/libsift_hip_abl$n.so $L/libsift_hip.so
    timeout -k 10 120 python3 tools/stage_bench.py --fast --reps 3 --ignore-status --tag abl$n >> $O/ab.txt 2>&1 || { echo "abl $n failed"; cp $L/libsift_hip_keep.so $L/libsift_hip.so; exit 1; }
  done
done
cp $L/libsift_hip_keep.so $L/libsift_hip.so
grep -h "^{" $O/ab.txt | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['tag'], d['stages_ms'].get('pyramid_fast'))"
