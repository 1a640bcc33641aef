#!/bin/bash
# bench.py's one-image leg (configs[1]) with each lib/libsift_hip_<name>.so, alternating, R rounds.
set -o pipefail
mkdir -p gpurun_out
L=sift-gpu_amd/lib
cp $L/libsift_hip.so $L/libsift_hip_keep.so
for r in $(seq ${R:-2}); do for n in "$@"; do
  cp $L/libsift_hip_$n.so $L/libsift_hip.so
  timeout -k 10 300 python3 bench.py --only single --steps 20 --warmup 5 > gpurun_out/abs_${n}_${r}.json 2>/dev/null || { cp $L/libsift_hip_keep.so $L/libsift_hip.so; exit 1; }
  python3 -c "
import json;d=json.loads(open('gpurun_out/abs_${n}_${r}.json').read().strip().splitlines()[-1])
s=d.get('single_image') or {}
print('$n', s.get('latency_ms'), s.get('device_no_graph_ms'), 'verified', s.get('output_verified'))"
done; done
cp $L/libsift_hip_keep.so $L/libsift_hip.so
