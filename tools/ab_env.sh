#!/bin/bash
# usage: tools/ab_env.sh "ENV=V ..." "ENV=V ..." ...   -- one stage_bench per env set
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
: > gpurun_out/ab.log
for e in "$@"; do
  env $e timeout -k 10 180 python tools/stage_bench.py --tag "$e" >> gpurun_out/ab.log 2>&1 || exit 1
done
echo done
