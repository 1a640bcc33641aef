#!/usr/bin/env python3
"""Per-launch counter table from rocprofv3 --pmc passes (tools/pmc.sh).

  python tools/pmc_table.py gpurun_out/pmc_<tag>

Reads every p*/run_counter_collection.csv under the directory, groups the
dispatches by (kernel, grid size) -- one group per octave of the pyramid --
averages each counter over the group's dispatches and prints the raw values
with a few ratios:
  clock     GRBM_GUI_ACTIVE / 8 XCDs / duration (dispatches of >= 0.3 ms)
  valu      SQ_INSTS_VALU / (duration x clock x 1024 SIMDs / 2 cycles per wave64 VALU)
  lds_act   SQ_ACTIVE_INST_LDS / SQ_WAVE_CYCLES   (both in quad-cycles)
  valu_act  SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES
  wait      SQ_WAIT_ANY / SQ_WAVE_CYCLES, issue stall SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES
  conflict  SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
Durations are the profiled dispatches' own (counters slow the clock a little).
"""
import collections
import csv
import glob
import os
import sys


def main():
    d = sys.argv[1]
    groups = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for f in sorted(glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True)):
        seen = set()
        for r in csv.DictReader(open(f)):
            key = (r["Kernel_Name"].split("(")[0][:40], int(r["Grid_Size"]))
            groups[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
            did = (f, r["Dispatch_Id"])
            if did not in seen:
                seen.add(did)
                dur[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    for key in sorted(groups, key=lambda k: -k[1]):
        c = {k: sum(v) / len(v) for k, v in groups[key].items()}
        t = sum(dur[key]) / len(dur[key])
        print(f"{key[0]} grid {key[1]}: {t * 1e3:.3f} ms (mean of {len(dur[key])} profiled dispatches)")
        for k in sorted(c):
            print(f"    {k:34s} {c[k]:16.1f}")
        wc = c.get("SQ_WAVE_CYCLES")
        ratios = {}
        if "GRBM_GUI_ACTIVE" in c:
            clk = c["GRBM_GUI_ACTIVE"] / 8 / t
            ratios["clock_GHz"] = clk / 1e9
            if "SQ_INSTS_VALU" in c:
                ratios["valu_issue_frac"] = c["SQ_INSTS_VALU"] / (t * clk * 1024 / 2)
        if wc:
            for k, name in (("SQ_ACTIVE_INST_LDS", "lds_act"), ("SQ_ACTIVE_INST_VALU", "valu_act"),
                            ("SQ_WAIT_ANY", "wait"), ("SQ_WAIT_INST_ANY", "issue_stall"),
                            ("SQ_ACTIVE_INST_ANY", "active"), ("SQ_ACTIVE_INST_VMEM", "vmem_act"),
                            ("SQ_WAIT_INST_LDS", "lds_issue_stall")):
                if k in c:
                    ratios[name] = c[k] / wc
        if c.get("SQ_LDS_IDX_ACTIVE"):
            ratios["lds_conflict"] = c.get("SQ_LDS_BANK_CONFLICT", 0) / c["SQ_LDS_IDX_ACTIVE"]
        if c.get("SQ_WAVES"):
            for k in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_WR"):
                if k in c:
                    ratios[k.lower() + "_per_wave"] = c[k] / c["SQ_WAVES"]
        print("    " + "  ".join(f"{k}={v:.3f}" for k, v in ratios.items()))


if __name__ == "__main__":
    main()
