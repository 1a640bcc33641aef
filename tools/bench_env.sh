#!/bin/bash
# bench.py's exact leg once per library environment setting (same box).
# usage: tools/bench_env.sh "VAR=val ..." ...   (extra bench args in BENCH_ARGS)
set -o pipefail
mkdir -p gpurun_out
for setting in "$@"; do
  env $setting timeout -k 10 300 python3 bench.py --only exact --no-cpu-baseline $BENCH_ARGS > gpurun_out/be.json 2> gpurun_out/be.err \
    || { echo "bench failed: $setting"; tail -5 gpurun_out/be.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/be.json')); print(sys.argv[1], d['value'], d['ms_per_step'], d['serial_leg']['ms_per_step'], d['output_verified'], {k: v for k, v in d['stages_ms_per_step'].items() if 'blur' in k})" "$setting"
done
