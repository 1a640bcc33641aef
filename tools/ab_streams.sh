#!/bin/bash
# bench.py's headline leg at several stream splits, same box, alternating.
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do for s in 1 2 3 4; do
  timeout -k 10 300 python3 bench.py --streams $s --no-cpu-baseline --no-single --no-8k --no-match --no-fast \
    --steps 10 > gpurun_out/streams_${s}_${r}.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/streams_${s}_${r}.json'));print('streams', $s, d['value'], d['ms_per_step'])"
done; done
