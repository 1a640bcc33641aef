#!/bin/bash
# exact headline leg with 1, 2, 3, 4 streams (sub-batches), alternating, 2 rounds
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do for s in 2 4 3 1; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-single --no-8k --no-match --no-fast --streams $s --steps 10 \
    > gpurun_out/streams_${s}_${r}.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/streams_${s}_${r}.json').read().strip().splitlines()[-1]);print('streams $s', d['value'], d['ms_per_step'])"
done; done
