#!/bin/bash
# SIFT_FLAG_FAST pyramid variants on one box: pyramid_tri (default),
# pyramid_pair (SIFT_HIP_FAST_PAIR=1), pyramid_fast (SIFT_HIP_FAST_V1=1),
# R rounds (default 2) of tools/stage_bench.py --fast.
# usage: tools/fast_ab.sh <tag> [variants...]
set -o pipefail
TAG=$1; shift
V=${@:-tri pair}
O=gpurun_out/fab_$TAG
mkdir -p $O
for r in $(seq ${R:-2}); do
  for v in $V; do
    unset SIFT_HIP_FAST_PAIR SIFT_HIP_FAST_V1
    [ $v = pair ] && export SIFT_HIP_FAST_PAIR=1
    [ $v = v1 ] && export SIFT_HIP_FAST_V1=1
    timeout -k 10 120 python3 tools/stage_bench.py --fast --reps 3 --tag $v >> $O/ab.txt 2>&1 || { echo "$v failed"; tail -5 $O/ab.txt; exit 1; }
  done
done
unset SIFT_HIP_FAST_PAIR SIFT_HIP_FAST_V1
grep -h "^{" $O/ab.txt | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['tag'], d['total_ms'], d['stages_ms'].get('pyramid_fast'), d['keypoints'])"
