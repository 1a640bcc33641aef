#!/bin/bash
# One-image (configs[1]) kernel times per library build: rocprofv3 --kernel-trace
# --stats over tools/single_trace.py, top kernels by total time, then SQ
# counters (PMC=1) of the kernels matching PMC_RE, default "descriptor" (tools/pmc.sh with PROG).
# usage: tools/r6_one.sh <tag> <variant>...   (variant: cur | lib/libsift_hip_<name>.so)
#        ARGS="--rows 4320 --cols 7680 --octaves 5 --cap 400000": configs[4] instead
set -o pipefail
export TMPDIR=/tmp
TAG=$1; shift
L=sift-gpu_amd/lib
cp $L/libsift_hip.so $L/libsift_hip_keep1.so
trap 'cp $L/libsift_hip_keep1.so $L/libsift_hip.so' EXIT
for v in "$@"; do
  [ $v = cur ] && cp $L/libsift_hip_keep1.so $L/libsift_hip.so || cp $L/libsift_hip_$v.so $L/libsift_hip.so
  O=gpurun_out/one_${TAG}_$v
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O -o run --output-format csv -- python3 tools/single_trace.py --reps 10 $ARGS > $O.log 2>&1 || { echo "trace $v failed"; tail $O.log; exit 1; }
  echo "== $v $(grep latency_ms $O.log | tail -1)"
  python3 - $O <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:6]:
    print("%-60s %6s %9.1f us" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3))
if len(sys.argv) > 1:  # the last iteration's launches in order (start, end, duration in us)
    t = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
    ks = sorted(csv.DictReader(open(t)), key=lambda r: int(r["Start_Timestamp"]))
    first = [i for i, r in enumerate(ks) if "blur_plane_kernel" in r["Kernel_Name"] or "blur_sym_base" in r["Kernel_Name"]]
    if len(first) >= 2:
        t0 = int(ks[first[-2]]["Start_Timestamp"])
        for r in ks[first[-2]:first[-1]]:
            a, b = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
            print("   %8.1f %8.1f %7.1f  %s" % (a / 1e3, b / 1e3, (b - a) / 1e3, r["Kernel_Name"][:60]))
PY
done
cp $L/libsift_hip_keep1.so $L/libsift_hip.so
[ -n "$PMC" ] && PROG="tools/single_trace.py --reps 3" bash tools/pmc.sh one_$TAG "${PMC_RE:-descriptor}" "$@"
exit 0
