#!/bin/bash
# GPU-box check for round 2: the -m gpu suite, then one bench run.
# usage: tools/gpu_r2.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-r2}; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_$TAG.log 2>&1 &&
timeout -k 10 600 python -u bench.py "$@" > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?
tail -3 gpurun_out/pytest_$TAG.log
echo "exit $rc"
exit $rc
