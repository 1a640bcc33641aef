#!/usr/bin/env python3
"""Summarise a tools/profile.sh run into profiles/<tag>_*.

  python tools/rocprof_summary.py <tag>   (reads gpurun_out/prof_<tag>/)

Writes
  profiles/<tag>_kernel_stats.csv  rocprofv3 --stats of the bench, verbatim;
  profiles/<tag>_summary.md/.json  per kernel: calls, average duration, HBM bytes
                                   per launch, GB/s; SQ counter ratios for the
                                   profiled kernels;
  profiles/traffic.json            per-launch HBM bytes that bench.py puts into
                                   roofline.traffic.

HBM bytes.  FETCH_SIZE / WRITE_SIZE are KiB.  tools/fetch_calib moves known
byte counts through a 1 GiB buffer in the same profile run; on gfx950 it shows
FETCH_SIZE = 0.5 x the bytes of coalesced streaming reads at 4, 8 and 16 B
per lane (MI355X_MICROARCH.md states it for 16 B) and WRITE_SIZE = 1.0 x the
bytes of streaming writes.  So:
  * STREAMING kernels (coalesced row reads: the blurs, the separable pyramid,
    the extrema tiles, decimation, DoG): read = FETCH_SIZE x the calibrated
    factor (2);
  * GATHER kernels (descriptor, orientation, refinement, emit, matcher):
    read = FETCH_SIZE raw -- a random 8-B gather reports 64 B per request in
    the calibration run and the line size behind it is not observable here, so
    the raw figure is a lower bound on their traffic.
"""
import csv
import json
import os
import re
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STREAMING = re.compile(r"blur_octave_kernel|blur_plane_kernel|blur_sym_kernel|blur_sym_base_kernel|pyr_pc_kernel|dog_extrema_kernel|extrema_walk_kernel|decimate_kernel|"
                       r"dog_kernel|blur1d|synth_kernel|grad_kernel|mask_count|mask_expand|bgr8_gray")


def counters(path):
    """{kernel: {counter: mean value per dispatch}}"""
    agg = defaultdict(lambda: defaultdict(list))
    if not os.path.exists(path):
        return {}
    for r in csv.DictReader(open(path)):
        agg[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in agg.items()}


def calibration(src):
    f = counters(os.path.join(src, "cal_f", "run_counter_collection.csv"))
    w = counters(os.path.join(src, "cal_w", "run_counter_collection.csv"))
    gib = float(1 << 30)
    out = {}
    for k, v in f.items():
        m = re.match(r"void rd<(float|HIP_vector_type<float, (\d)u> )>", k)
        if m:
            width = 4 * int(m.group(2) or 1)
            out[f"read_{width}B_per_lane"] = v["FETCH_SIZE"] * 1024 / gib
        if k.startswith("gather8"):
            out["gather_8B_reported_bytes_per_request"] = v["FETCH_SIZE"] * 1024 / (1 << 24)
    for k, v in w.items():
        m = re.match(r"void wr<(float|HIP_vector_type<float, (\d)u> )>", k)
        if m:
            width = 4 * int(m.group(2) or 1)
            out[f"write_{width}B_per_lane"] = v["WRITE_SIZE"] * 1024 / gib
    return out


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r2"
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    out = os.path.join(ROOT, "profiles")
    os.makedirs(out, exist_ok=True)
    stats_csv = os.path.join(src, "trace", "run_kernel_stats.csv")
    shutil.copy(stats_csv, os.path.join(out, f"{tag}_kernel_stats.csv"))
    stats = list(csv.DictReader(open(stats_csv)))
    fetch = counters(os.path.join(src, "fetch", "run_counter_collection.csv"))
    write = counters(os.path.join(src, "write", "run_counter_collection.csv"))
    cal = calibration(src)
    rf = 1.0 / min(cal.get("read_4B_per_lane", 0.5), cal.get("read_8B_per_lane", 0.5))
    wf = 1.0 / cal.get("write_4B_per_lane", 1.0)
    bench = None
    for line in open(os.path.join(src, "trace.log")):
        if line.startswith("{"):
            bench = json.loads(line)
    lines = [f"# rocprofv3 summary `{tag}`", ""]
    if bench:
        lines += [f"bench under the profiler: {bench['value']} {bench['unit']}, {bench['ms_per_step']} ms/step "
                  f"(exact), fast mode {bench.get('fast_mode', {}).get('value')} Mpix/s; config "
                  f"`{bench['config']['workload']}`", ""]
    lines += ["FETCH/WRITE calibration (tools/fetch_calib, reported / true bytes): " +
              ", ".join(f"{k} {v:.4f}" for k, v in sorted(cal.items())), "",
              f"read bytes = FETCH_SIZE x {rf:g} for streaming kernels (S), FETCH_SIZE raw for gather kernels "
              f"(G, a lower bound); write bytes = WRITE_SIZE x {wf:g}.", "",
              "| kernel | kind | calls | avg ms | % time | HBM read MB/launch | HBM write MB/launch | GB/s |",
              "|---|---|---|---|---|---|---|---|"]
    summary, traffic = {}, {}
    for r in stats:
        name = r["Name"]
        avg_ms = float(r["AverageNs"]) / 1e6
        streaming = bool(STREAMING.search(name))
        rd_raw = fetch.get(name, {}).get("FETCH_SIZE", 0.0) * 1024
        rd = rd_raw * (rf if streaming else 1.0)
        wr = write.get(name, {}).get("WRITE_SIZE", 0.0) * 1024 * wf
        gbs = (rd + wr) / 1e9 / (avg_ms / 1e3) if avg_ms else 0
        summary[name] = dict(calls=int(r["Calls"]), avg_ms=avg_ms, kind="streaming" if streaming else "gather",
                             read_bytes=rd, read_bytes_raw=rd_raw, write_bytes=wr, GBs=gbs)
        traffic[name] = {"read_bytes": round(rd), "write_bytes": round(wr), "kind": summary[name]["kind"]}
        lines.append(f"| {name} | {'S' if streaming else 'G'} | {r['Calls']} | {avg_ms:.4f} | "
                     f"{float(r['Percentage']):.2f} | {rd / 1e6:.1f} | {wr / 1e6:.1f} | {gbs:.0f} |")
    # SQ groups
    sq = defaultdict(dict)
    for grp in ("sq1", "sq2", "sq3", "sqF1", "sqF2", "sqF3"):
        for k, v in counters(os.path.join(src, grp, "run_counter_collection.csv")).items():
            sq[k].update(v)
    # shader clock per kernel: GRBM_GUI_ACTIVE (summed over the 8 XCDs) / 8 /
    # the dispatch's duration in the same counter pass
    clock = {}
    for grp in ("sq3", "sqF3"):
        path = os.path.join(src, grp, "run_kernel_trace.csv")
        if not os.path.exists(path):
            continue
        durs = defaultdict(list)
        for r in csv.DictReader(open(path)):
            durs[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        for k, ds in durs.items():
            g = sq.get(k, {}).get("GRBM_GUI_ACTIVE")
            if g and ds:
                clock[k] = g / 8 / (sum(ds) / len(ds))
    if sq:
        lines += ["", "## SQ counters (tools/stage_bench.py, one step of the 64 x 1080p batch)", "",
                  "Per dispatch, averaged over the dispatches of a kernel.  SQ_WAVE_CYCLES / SQ_WAIT_* / "
                  "SQ_ACTIVE_INST_* count quad-cycles (MI355X_MICROARCH.md), so their ratios are fractions of "
                  "wave time; VALU issue util = SQ_ACTIVE_INST_VALU x 4 / (SQ_BUSY_CYCLES x 4 SIMDs ... see "
                  "json); clock = GRBM_GUI_ACTIVE / 8 XCDs / duration.", "",
                  "| kernel | waves | VALU instr/wave | LDS instr/wave | wait (s_waitcnt/barrier) | issue stall | "
                  "active | LDS bank-conflict cycles / LDS active | L2 hit | clock GHz |",
                  "|---|---|---|---|---|---|---|---|---|---|"]
        for k, v in sorted(sq.items()):
            if "SQ_WAVES" not in v:
                continue
            wc = v.get("SQ_WAVE_CYCLES", 0) or 1
            hit = v.get("TCC_HIT_sum", 0)
            miss = v.get("TCC_MISS_sum", 0)
            lds_act = v.get("SQ_ACTIVE_INST_LDS", 0) or 1
            lines.append(
                f"| {k} | {v['SQ_WAVES']:.0f} | {v.get('SQ_INSTS_VALU', 0) / v['SQ_WAVES']:.0f} | "
                f"{v.get('SQ_INSTS_LDS', 0) / v['SQ_WAVES']:.0f} | {v.get('SQ_WAIT_ANY', 0) / wc:.2f} | "
                f"{v.get('SQ_WAIT_INST_ANY', 0) / wc:.2f} | {v.get('SQ_ACTIVE_INST_ANY', 0) / wc:.2f} | "
                f"{v.get('SQ_LDS_BANK_CONFLICT', 0) / lds_act:.2f} | "
                f"{hit / (hit + miss) if hit + miss else 0:.2f} | "
                f"{clock[k]:.2f} |" if k in clock else
                f"| {k} | {v['SQ_WAVES']:.0f} | {v.get('SQ_INSTS_VALU', 0) / v['SQ_WAVES']:.0f} | "
                f"{v.get('SQ_INSTS_LDS', 0) / v['SQ_WAVES']:.0f} | {v.get('SQ_WAIT_ANY', 0) / wc:.2f} | "
                f"{v.get('SQ_WAIT_INST_ANY', 0) / wc:.2f} | {v.get('SQ_ACTIVE_INST_ANY', 0) / wc:.2f} | "
                f"{v.get('SQ_LDS_BANK_CONFLICT', 0) / lds_act:.2f} | "
                f"{hit / (hit + miss) if hit + miss else 0:.2f} | - |")
    with open(os.path.join(out, f"{tag}_summary.md"), "w") as f:
        f.write("\n".join(lines) + "\n")
    with open(os.path.join(out, f"{tag}_summary.json"), "w") as f:
        json.dump({"bench": bench, "calibration": cal, "kernels": summary, "sq": sq, "clock_GHz": clock}, f,
                  indent=1)
    # VALU / LDS wave-instructions per dispatch (SQ pass over tools/stage_bench.py,
    # the same 64 x 1080p batch): bench.py's VALU-issue rooflines
    for name, v in sq.items():
        if name in traffic and "SQ_INSTS_VALU" in v:
            traffic[name]["valu_insts"] = round(v["SQ_INSTS_VALU"])
            traffic[name]["lds_insts"] = round(v.get("SQ_INSTS_LDS", 0))
            traffic[name]["waves"] = round(v.get("SQ_WAVES", 0))
    with open(os.path.join(out, "traffic.json"), "w") as f:
        json.dump({"source": f"profiles/{tag}_summary.json (rocprofv3 FETCH_SIZE / WRITE_SIZE passes over "
                             f"bench.py, calibrated by tools/fetch_calib; SQ_INSTS_* from the SQ pass over "
                             f"tools/stage_bench.py)", "kernels": traffic}, f, indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main()
