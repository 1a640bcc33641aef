"""Per-kernel (and per-grid) average durations from a rocprofv3 kernel trace CSV.

    python tools/trace_summary.py gpurun_out/pf/trace/run_kernel_trace.csv [name-regex]
"""
import collections
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else '.')
d = collections.defaultdict(list)
for r in rows:
    if pat.search(r['Kernel_Name']):
        key = (r['Kernel_Name'][:70], r['Grid_Size_X'], r['Grid_Size_Y'], r['Grid_Size_Z'])
        d[key].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1]) / len(kv[1])):
    print('%8.1f us  x%-3d %s grid %sx%sx%s' % (sum(v) / len(v), len(v), k[0], k[1], k[2], k[3]))
