#!/usr/bin/env python3
"""Two-stream overlap of a kernel trace (rocprofv3 --kernel-trace CSV).

  python tools/trace_overlap.py <run_kernel_trace.csv>

For the timed-looking tail of the trace (the last half of the dispatches), per
kernel family: total busy time, and how much of each family's time runs beside
a dispatch of each other family on another queue (pairwise overlap in ms).
"""
import collections
import csv
import sys


def fam(name):
    n = name.split("(")[0]
    for k in ("blur_sym_kernel", "descriptor_kernel", "orient_slots_kernel", "extrema_walk_kernel",
              "refine_kernel", "blur_sym_base_kernel", "decimate_kernel", "blur_octave_kernel"):
        if n.startswith(k) or ("::" + k) in n or n.endswith(k):
            return k
    return "other"


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    ev = []
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        q = r.get("Queue_Id") or r.get("Stream_Id") or "0"
        ev.append((s, e, q, fam(r["Kernel_Name"])))
    ev.sort()
    ev = ev[len(ev) // 2:]
    t0, t1 = ev[0][0], max(e for _, e, _, _ in ev)
    busy = collections.defaultdict(float)
    ov = collections.defaultdict(float)
    for i, (s, e, q, f) in enumerate(ev):
        busy[f] += (e - s) * 1e-6
        for s2, e2, q2, f2 in ev:
            if q2 == q or s2 >= e or e2 <= s:
                continue
            ov[(f, f2)] += (min(e, e2) - max(s, s2)) * 1e-6
    print(f"window {(t1 - t0) * 1e-6:.2f} ms, {len(ev)} dispatches")
    for f in sorted(busy, key=lambda k: -busy[k]):
        parts = ", ".join(f"{f2} {v:.2f}" for (a, f2), v in sorted(ov.items(), key=lambda kv: -kv[1]) if a == f and v > 0.05)
        print(f"{f:24s} busy {busy[f]:8.2f} ms; beside: {parts}")


if __name__ == "__main__":
    main()
