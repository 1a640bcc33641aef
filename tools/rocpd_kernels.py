#!/usr/bin/env python3
"""Median kernel durations from rocprofv3 rocpd databases (run_results.db).
  python3 tools/rocpd_kernels.py gpurun_out/ot_a/run_results.db [...]"""
import collections
import sqlite3
import sys

for path in sys.argv[1:]:
    cur = sqlite3.connect(path).cursor()
    cols = [r[1] for r in cur.execute("pragma table_info(kernels)")]
    ni = cols.index("name") if "name" in cols else cols.index("kernel_name")
    s, e = cols.index("start"), cols.index("end")
    d = collections.defaultdict(list)
    for r in cur.execute("select * from kernels"):
        d[r[ni].split("(")[0]].append((r[e] - r[s]) / 1e3)
    print(path)
    for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
        if k.startswith("sift::") or "sift::" in k:
            v = sorted(v)
            print(f"  {k[:48]:48s} {len(v):4d} med {v[len(v) // 2]:8.1f} us")
