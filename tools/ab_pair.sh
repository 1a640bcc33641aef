#!/bin/bash
# bench.py's exact leg with and without pyramid turns (sift_ctx_pair), same box, alternating.
set -o pipefail
mkdir -p gpurun_out
for r in $(seq ${R:-3}); do for p in 0 1; do
  timeout -k 10 300 python3 bench.py --pair $p --no-cpu-baseline --no-single --no-8k --no-match --no-fast \
    --steps 10 > gpurun_out/pair_${p}_${r}.json 2>gpurun_out/pair_${p}_${r}.err || { tail -5 gpurun_out/pair_${p}_${r}.err; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/pair_${p}_${r}.json').read().strip().splitlines()[-1]);print('pair', $p, d['value'], d['ms_per_step'], d['output_verified'])"
done; done
