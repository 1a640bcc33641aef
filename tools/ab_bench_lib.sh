#!/bin/bash
# bench.py's exact headline leg with each lib/libsift_hip_<name>.so, alternating, R rounds.
set -o pipefail
mkdir -p gpurun_out
L=sift-gpu_amd/lib
cp $L/libsift_hip.so $L/libsift_hip_keep.so
for r in $(seq ${R:-2}); do for n in "$@"; do
  cp $L/libsift_hip_$n.so $L/libsift_hip.so
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-single --no-8k --no-match --no-fast \
    --steps 10 > gpurun_out/abb_${n}_${r}.json 2>/dev/null || { cp $L/libsift_hip_keep.so $L/libsift_hip.so; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/abb_${n}_${r}.json').read().strip().splitlines()[-1]);print('$n', d['value'], d['ms_per_step'])"
done; done
cp $L/libsift_hip_keep.so $L/libsift_hip.so
