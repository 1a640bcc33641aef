#!/bin/bash
# GPU-box check for round 3: -m gpu suite, same-box A/B of lib/libsift_hip_base.so
# against the current library (tools/stage_bench.py), the descriptor's LDS
# counters for both, then one bench run.
# usage: tools/gpu_r3.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-r3}; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
L=sift-gpu_amd/lib
O=gpurun_out/$TAG
mkdir -p $O
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
fi
cp $L/libsift_hip.so $L/libsift_hip_new.so
for r in 1 2; do
  for v in base new; do
    cp $L/libsift_hip_$v.so $L/libsift_hip.so
    timeout -k 10 180 python3 tools/stage_bench.py --reps 5 --tag $v >> $O/ab.txt 2>&1 || { cp $L/libsift_hip_new.so $L/libsift_hip.so; exit 1; }
  done
done
for v in base new; do
  cp $L/libsift_hip_$v.so $L/libsift_hip.so
  timeout -k 10 -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES \
    -T --kernel-include-regex "descriptor_kernel" -d $O/pmc_$v -o run --output-format csv -- \
    python3 tools/stage_bench.py --reps 1 > $O/pmc_$v.log 2>&1 || { cp $L/libsift_hip_new.so $L/libsift_hip.so; echo "pmc $v failed"; tail -5 $O/pmc_$v.log; exit 1; }
done
cp $L/libsift_hip_new.so $L/libsift_hip.so
for r in 1 2; do
  for v in pair v1; do
    if [ $v = v1 ]; then export SIFT_HIP_FAST_V1=1; else unset SIFT_HIP_FAST_V1; fi
    timeout -k 10 180 python3 tools/stage_bench.py --fast --reps 5 --tag fast_$v >> $O/ab.txt 2>&1 || exit 1
  done
done
unset SIFT_HIP_FAST_V1
grep -h "^{" $O/ab.txt | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['tag'], d['total_ms'], d['stages_ms'])" || true
timeout -k 10 600 python -u bench.py "$@" > $O/bench.json 2> $O/bench.err
rc=$?
echo "bench exit $rc"
exit $rc
