#!/bin/bash
# One-image (configs[1]) kernel times per library build: rocprofv3 --kernel-trace
# --stats over tools/single_trace.py, top kernels by total time, then SQ
# counters (PMC=1) of the kernels matching PMC_RE, default "descriptor" (tools/pmc.sh with PROG).
# usage: tools/r6_one.sh <tag> <variant>...   (variant: cur | lib/libsift_hip_<name>.so)
set -o pipefail
export TMPDIR=/tmp
TAG=$1; shift
L=sift-gpu_amd/lib
cp $L/libsift_hip.so $L/libsift_hip_keep1.so
trap 'cp $L/libsift_hip_keep1.so $L/libsift_hip.so' EXIT
for v in "$@"; do
  [ $v = cur ] && cp $L/libsift_hip_keep1.so $L/libsift_hip.so || cp $L/libsift_hip_$v.so $L/libsift_hip.so
  O=gpurun_out/one_${TAG}_$v
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O -o run --output-format csv -- python3 tools/single_trace.py --reps 10 > $O.log 2>&1 || { echo "trace $v failed"; tail $O.log; exit 1; }
  echo "== $v $(grep latency_ms $O.log | tail -1)"
  python3 - $O <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:6]:
    print("%-60s %6s %9.1f us" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
done
cp $L/libsift_hip_keep1.so $L/libsift_hip.so
[ -n "$PMC" ] && PROG="tools/single_trace.py --reps 3" bash tools/pmc.sh one_$TAG "${PMC_RE:-descriptor}" "$@"
exit 0
