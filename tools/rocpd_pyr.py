#!/usr/bin/env python3
"""Per-launch median durations of the fast-pyramid kernels (pyr_*) in
rocprofv3 rocpd databases, one line per (kernel, grid): octave launches.
  python3 tools/rocpd_pyr.py gpurun_out/<trace>/run_results.db [...]"""
import collections
import sqlite3
import sys

for path in sys.argv[1:]:
    cur = sqlite3.connect(path).cursor()
    d = collections.defaultdict(list)
    for name, grid, s, e in cur.execute("select name, grid_x, start, end from kernels"):
        if "pyr_" in name:
            d[(name.split("(")[0].split("::")[-1], grid)].append((e - s) / 1e3)
    print(path)
    tot = 0.0
    for (k, g), v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
        v = sorted(v)
        med = v[len(v) // 2]
        tot += med
        print(f"  {k:32s} grid {g:8d} n {len(v):3d} med {med:8.1f} us")
    print(f"  sum of medians {tot:.1f} us")
