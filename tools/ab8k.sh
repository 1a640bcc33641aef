#!/bin/bash
# configs[4] (one 8K image, exact) under environment variants, alternating, R rounds:
#   tools/ab8k.sh <tag> "<VAR=val ...>" ["<VAR=val ...>" ...]   ("-" = no variables)
set -o pipefail
TAG=$1; shift
O=gpurun_out/ab8k_$TAG
mkdir -p $O
for r in $(seq ${R:-2}); do
  for v in "$@"; do
    ENVS=$v; [ "$v" = "-" ] && ENVS=""
    f=$O/$(echo "$v" | tr ' =,/' '___-')_$r
    env $ENVS timeout -k 10 200 python3 bench.py --only 8k --steps 5 --warmup 2 > $f.json 2> $f.err \
      || { echo "8k $v failed"; tail -3 $f.err; exit 1; }
    python3 -c "
import json, sys
e = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['image_8k']
print(sys.argv[2], 'latency_ms', e['latency_ms'], 'blur_ms', e['roofline']['exact_blur_octave']['ms_per_image'],
      'verified', e['output_verified'])" $f.json "$v"
  done
done
