#!/bin/bash
# Same-box A/B of library variants selected by an environment switch:
#   tools/env_ab.sh <tag> <VAR> <value>... -- runs the -m gpu suite once, then
#   tools/stage_bench.py with VAR=value for each value, three rounds alternating.
set -o pipefail
TAG=$1; VAR=$2; shift 2
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_$TAG.log
for r in 1 2 3; do
  for v in "$@"; do
    env $VAR=$v timeout -k 10 120 python3 tools/stage_bench.py --reps 5 --tag "$VAR=$v" \
      >> gpurun_out/ab_$TAG.log 2>&1 || { tail -20 gpurun_out/ab_$TAG.log; exit 1; }
  done
done
cat gpurun_out/ab_$TAG.log
