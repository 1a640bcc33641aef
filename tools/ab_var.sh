#!/bin/bash
# Times the SIFT_FLAG_FAST pyramid (or, with MODE=exact, every stage) of each
# lib/libsift_hip_<name>.so, alternating, R rounds (default 2).
# usage: tools/ab_var.sh <tag> <name>...
set -o pipefail
TAG=$1; shift
L=sift-gpu_amd/lib
O=gpurun_out/var_$TAG
mkdir -p $O
FL=--fast; [ "$MODE" = exact ] && FL=
cp $L/libsift_hip.so $L/libsift_hip_keep.so
for r in $(seq ${R:-2}); do
  for n in "$@"; do
    cp $L/libsift_hip_$n.so $L/libsift_hip.so
    timeout -k 10 120 python3 tools/stage_bench.py $FL --reps 3 --ignore-status --tag $n >> $O/ab.txt 2>&1 || { echo "var $n failed"; tail -5 $O/ab.txt; cp $L/libsift_hip_keep.so $L/libsift_hip.so; exit 1; }
  done
done
cp $L/libsift_hip_keep.so $L/libsift_hip.so
grep -h "^{" $O/ab.txt | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['tag'], d['total_ms'], json.dumps(d['stages_ms']))"
