#!/bin/bash
# A/B of library environment switches on the same box: tools/stage_bench.py
# once per setting.  usage: tools/ab_env.sh "VAR=val ..." "VAR=val ..." ...
set -o pipefail
mkdir -p gpurun_out
for setting in "$@"; do
  echo "== $setting"
  env $setting timeout -k 10 300 python3 tools/stage_bench.py --reps 3 --tag "$setting" || exit 1
done
