#!/bin/bash
# FETCH_SIZE of the exact scatter blur with and without the XCD-contiguous
# wave order (SIFT_HIP_SYM_XCD): one rocprofv3 counter pass per
# setting over tools/stage_bench.py (exact path), kernel-trace only beside the
# counter; prints KB fetched per launch of blur_sym_kernel for each.
set -o pipefail
OUT=gpurun_out/xcd_fetch
mkdir -p $OUT
export TMPDIR=/tmp
for x in 0 1; do
  SIFT_HIP_SYM_XCD=$x timeout -k 5 -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -T \
    --kernel-include-regex "blur_sym_kernel" -d $OUT/x$x -o run --output-format csv -- \
    python3 tools/stage_bench.py --reps 1 > $OUT/x$x.log 2>&1 || { echo "pass x$x failed"; tail -5 $OUT/x$x.log; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
for x in (0, 1):
    f = glob.glob(f"{sys.argv[1]}/x{x}/**/run_counter_collection.csv", recursive=True)[0]
    per = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "blur_sym_kernel" in r["Kernel_Name"] and r["Counter_Name"] == "FETCH_SIZE":
            per[int(r["Grid_Size"])].append(float(r["Counter_Value"]))
    print(f"SIFT_HIP_SYM_XCD={x}: " + ", ".join(f"grid {g}: {sum(v)/len(v)/1024:.0f} MiB/launch (raw FETCH_SIZE)" for g, v in sorted(per.items(), reverse=True)))
PY
