#!/bin/bash
# rocprofv3 passes over one bench configuration (run on the GPU box):
#   1. --kernel-trace --stats          per-kernel durations
#   2. --pmc FETCH_SIZE (own pass)     HBM read (gfx950: reads are half the bytes of wide streams)
#   3. --pmc WRITE_SIZE (own pass)     HBM write
# usage: tools/profile.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-r1}; shift
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
ARGS="$@"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d $OUT/trace -o run --output-format csv -- \
  python3 bench.py --no-cpu-baseline $ARGS > $OUT/trace.log 2>&1 &&
timeout -k 10 600 rocprofv3 --kernel-trace --pmc FETCH_SIZE -T -d $OUT/fetch -o run --output-format csv -- \
  python3 bench.py --no-cpu-baseline --steps 1 --warmup 1 $ARGS > $OUT/fetch.log 2>&1 &&
timeout -k 10 600 rocprofv3 --kernel-trace --pmc WRITE_SIZE -T -d $OUT/write -o run --output-format csv -- \
  python3 bench.py --no-cpu-baseline --steps 1 --warmup 1 $ARGS > $OUT/write.log 2>&1
rc=$?
echo "profile exit $rc"
exit $rc
