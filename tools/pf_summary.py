"""Per-dispatch summary of a tools/prof_fast.sh run: duration (kernel trace),
counters per dispatch, derived: VALU issue rate, waits, clock, HBM bytes.
usage: python tools/pf_summary.py gpurun_out/pf_<tag> [kernel-substring]"""
import csv
import glob
import os
import sys
from collections import defaultdict

d = sys.argv[1]
ks = sys.argv[2] if len(sys.argv) > 2 else "pyr_"
trace = list(csv.DictReader(open(glob.glob(os.path.join(d, "trace", "*kernel_trace.csv"))[0])))
rows = [r for r in trace if ks in r["Kernel_Name"]]
print("kernel trace:", len(rows), "dispatches")
byname = defaultdict(list)
for r in rows:
    key = (r["Kernel_Name"][:60], int(r.get("Grid_Size", r.get("Grid_Size_X", 0)) or 0))
    byname[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(byname.items(), key=lambda kv: -sum(kv[1])):
    print(f"  {k[0]:60s} grid {k[1]:9d}  n {len(v)}  avg {sum(v)/len(v):9.1f} us")
counters = defaultdict(dict)   # (pass, dispatch) -> name -> value
meta = {}
for p in ("sq1", "sq2", "gr", "fe", "wr", "ic"):
    f = glob.glob(os.path.join(d, p, "*counter_collection.csv"))
    if not f:
        continue
    for r in csv.DictReader(open(f[0])):
        if ks not in r["Kernel_Name"]:
            continue
        key = (p, int(r["Dispatch_Id"]))
        counters[key][r["Counter_Name"]] = counters[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        meta[key] = (int(r["Grid_Size"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, r["VGPR_Count"],
                     r["LDS_Block_Size"])
# group per grid size (octave) and pass: average
agg = defaultdict(lambda: defaultdict(list))
for (p, disp), cs in counters.items():
    g, dur, vg, lds = meta[(p, disp)]
    agg[g]["dur_" + p].append(dur)
    agg[g]["vgpr"] = [vg]
    agg[g]["lds"] = [lds]
    for n, v in cs.items():
        agg[g][n].append(v)
for g in sorted(agg, reverse=True):
    a = {n: (sum(v) / len(v) if isinstance(v[0], float) else v[0]) for n, v in agg[g].items()}
    dur = a.get("dur_sq1", 0)
    out = {"grid": g, "vgpr": a.get("vgpr"), "lds": a.get("lds"), "us": round(dur, 1)}
    if "SQ_WAVE_CYCLES" in a:
        wc = a["SQ_WAVE_CYCLES"]
        out["valu_per_wave"] = round(a["SQ_INSTS_VALU"] / a["SQ_WAVES"], 1)
        out["vmem_wr_per_wave"] = round(a["SQ_INSTS_VMEM_WR"] / a["SQ_WAVES"], 1)
        out["lds_per_wave"] = round(a["SQ_INSTS_LDS"] / a["SQ_WAVES"], 1)
        # wave64 VALU instructions per second vs 1228.8 G/s at 2.4 GHz
        out["valu_issue_frac_2.4GHz"] = round(a["SQ_INSTS_VALU"] / (dur * 1e-6) / 1228.8e9, 3)
    if "SQ_WAIT_ANY" in a:
        tot = a["SQ_WAIT_ANY"] + a["SQ_WAIT_INST_ANY"] + a["SQ_ACTIVE_INST_ANY"]
        out["wait_any"] = round(a["SQ_WAIT_ANY"] / tot, 3)
        out["wait_inst"] = round(a["SQ_WAIT_INST_ANY"] / tot, 3)
        out["active"] = round(a["SQ_ACTIVE_INST_ANY"] / tot, 3)
        out["active_valu"] = round(a["SQ_ACTIVE_INST_VALU"] / tot, 3)
        out["lds_conflict_ratio"] = round(a["SQ_LDS_BANK_CONFLICT"] / max(a["SQ_ACTIVE_INST_LDS"], 1), 3)
    if "GRBM_GUI_ACTIVE" in a:
        out["clock_GHz"] = round(a["GRBM_GUI_ACTIVE"] / 8 / (a["dur_gr"][0] if isinstance(a["dur_gr"], list) else a["dur_gr"]) / 1e3, 3)
    if "FETCH_SIZE" in a:
        out["fetch_MB_x2"] = round(2 * a["FETCH_SIZE"] / 1e3, 1)   # KB -> MB, x2 gfx950 streaming calibration
    if "WRITE_SIZE" in a:
        out["write_MB"] = round(a["WRITE_SIZE"] / 1e3, 1)
    if "SQC_ICACHE_MISSES" in a:
        out["icache_miss_frac"] = round(a["SQC_ICACHE_MISSES"] / max(a["SQC_ICACHE_HITS"] + a["SQC_ICACHE_MISSES"], 1), 4)
    print(out)
