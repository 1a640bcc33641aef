#!/bin/bash
# Round-4 closing run on one GPU box: -m gpu suite, same-box A/Bs of the last
# variants (lib/libsift_hip_<name>.so), the bench line, the rocprofv3 passes.
# usage: tools/final_r3.sh <tag> "<fast A/B libs>" "<exact A/B libs>"
set -o pipefail
TAG=$1
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -2 $O/pytest.log
[ $rc -eq 0 ] || exit 1
[ -n "$2" ] && { R=3 bash tools/ab_var.sh ${TAG}f $2 || exit 1; }
[ -n "$3" ] && { MODE=exact R=2 bash tools/ab_var.sh ${TAG}x $3 || exit 1; }
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
tail -c 200 $O/bench.json
bash tools/profile_r3.sh $TAG || exit 1
echo "final $TAG done"
