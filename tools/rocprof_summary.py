#!/usr/bin/env python3
"""Summarise a tools/profile.sh run into profiles/<tag>_*.

  python tools/rocprof_summary.py <tag>   (reads gpurun_out/prof_<tag>/)

Writes profiles/<tag>_kernel_stats.csv (rocprofv3 --stats, verbatim) and
profiles/<tag>_summary.md: per-kernel average duration and HBM bytes per
launch from the separate FETCH_SIZE / WRITE_SIZE passes, corrected as
MI355X_MICROARCH.md prescribes (FETCH_SIZE/WRITE_SIZE are KiB; gfx950
FETCH_SIZE counts half the bytes of wide coalesced reads, so reads are x2).
"""
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def counter(path):
    agg = {}
    if not os.path.exists(path):
        return agg
    for r in csv.DictReader(open(path)):
        agg.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r1"
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    out = os.path.join(ROOT, "profiles")
    os.makedirs(out, exist_ok=True)
    stats_csv = os.path.join(src, "trace", "run_kernel_stats.csv")
    shutil.copy(stats_csv, os.path.join(out, f"{tag}_kernel_stats.csv"))
    stats = list(csv.DictReader(open(stats_csv)))
    fetch = counter(os.path.join(src, "fetch", "run_counter_collection.csv"))
    write = counter(os.path.join(src, "write", "run_counter_collection.csv"))
    bench = None
    for line in open(os.path.join(src, "trace.log")):
        if line.startswith("{"):
            bench = json.loads(line)
    lines = [f"# rocprofv3 summary `{tag}`", ""]
    if bench:
        lines += [f"bench: {bench['value']} {bench['unit']}, {bench['ms_per_step']} ms/step, "
                  f"{bench['keypoints_per_s']:.0f} keypoints/s, config `{bench['config']['workload']}` "
                  f"(under the profiler)", ""]
    lines += ["| kernel | calls | avg ms | % time | HBM read MB/launch (FETCH x2) | HBM write MB/launch | GB/s |",
              "|---|---|---|---|---|---|---|"]
    summary = {}
    for r in stats:
        name = r["Name"]
        avg_ms = float(r["AverageNs"]) / 1e6
        rd = fetch.get(name, 0.0) * 1024 * 2 / 1e6
        wr = write.get(name, 0.0) * 1024 / 1e6
        gbs = (rd + wr) / 1e3 / (avg_ms / 1e3) if avg_ms else 0
        summary[name] = dict(calls=int(r["Calls"]), avg_ms=avg_ms, read_MB=rd, write_MB=wr)
        lines.append(f"| {name} | {r['Calls']} | {avg_ms:.4f} | {float(r['Percentage']):.2f} | {rd:.1f} | {wr:.1f} | {gbs:.0f} |")
    with open(os.path.join(out, f"{tag}_summary.md"), "w") as f:
        f.write("\n".join(lines) + "\n")
    with open(os.path.join(out, f"{tag}_summary.json"), "w") as f:
        json.dump({"bench": bench, "kernels": summary}, f, indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main()
