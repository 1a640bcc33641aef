#!/bin/bash
# -m gpu suite on the current build, then tools/ab_lib.sh (base vs current),
# printing per-stage ms of each run.
set -o pipefail
TAG=${1:-lib}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_$TAG.log
bash tools/ab_lib.sh > gpurun_out/ab_$TAG.log 2>&1 || { tail -20 gpurun_out/ab_$TAG.log; exit 1; }
grep -h stages_ms gpurun_out/ab_$TAG.log | python3 -c "
import sys,json
for l in sys.stdin:
  d=json.loads(l); s=d['stages_ms']; print(d['tag'], d['total_ms'], {k: s[k] for k in ('extrema','refine_orient','descriptor')})"
