#!/bin/bash
# configs[4] (one 8K image) under library builds (lib/libsift_hip_<name>.so, "cur" = current), alternating, R rounds:
#   tools/ab8k_lib.sh <tag> <name>...
set -o pipefail
TAG=$1; shift
L=sift-gpu_amd/lib
O=gpurun_out/ab8kl_$TAG
mkdir -p $O
cp $L/libsift_hip.so $L/libsift_hip_ab8kkeep.so
trap 'cp $L/libsift_hip_ab8kkeep.so $L/libsift_hip.so' EXIT
for r in $(seq ${R:-2}); do
  for v in "$@"; do
    if [ "$v" = cur ]; then cp $L/libsift_hip_ab8kkeep.so $L/libsift_hip.so; else cp $L/libsift_hip_$v.so $L/libsift_hip.so; fi
    timeout -k 10 200 python3 bench.py --only 8k --steps 5 --warmup 2 > $O/${v}_$r.json 2> $O/${v}_$r.err \
      || { echo "8k $v failed"; tail -3 $O/${v}_$r.err; exit 1; }
    python3 -c "
import json, sys
e = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['image_8k']
r = e['roofline']['fast_pyramid']
print(sys.argv[2], 'fast_pyr_ms', r['ms_per_image'], 'frac', r['frac'], 'exact_ms', e['latency_ms'], 'verified', e['output_verified'])" $O/${v}_$r.json "$v"
  done
done
