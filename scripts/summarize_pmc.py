#!/usr/bin/env python3
"""Summarise a counter-only rocprofv3 run (--pmc ... --kernel-trace, csv) per kernel:
mean counters per dispatch, kernel ms, effective clock (GRBM_GUI_ACTIVE / 8 XCDs / time) and
MFMA-pipe utilisation (SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)).

  python scripts/summarize_pmc.py gpurun_out/pmc_dir [--match assign16]"""
import argparse
import csv
import glob
import os
import statistics
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--match", default="")
    a = ap.parse_args()
    cc = glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True)
    kt = glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True)
    dur = {}
    for f in kt:
        for r in csv.DictReader(open(f)):
            dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
    vals = defaultdict(lambda: defaultdict(float))   # (kernel, dispatch) -> counter -> sum
    for f in cc:
        for r in csv.DictReader(open(f)):
            k = r.get("Kernel_Name", "?")
            if a.match and a.match not in k:
                continue
            vals[(k, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    per = defaultdict(list)
    for (k, d), c in vals.items():
        c = dict(c)
        c["ms"] = dur.get(d, float("nan"))
        per[k].append(c)
    for k, rows in per.items():
        keys = sorted({n for r in rows for n in r})
        mean = {n: statistics.mean(r[n] for r in rows if n in r) for n in keys}
        print(f"## {k[:110]}  ({len(rows)} dispatches)")
        for n in keys:
            print(f"  {n:28s} {mean[n]:.6g}")
        if "GRBM_GUI_ACTIVE" in mean and mean.get("ms", 0) > 0:
            clk = mean["GRBM_GUI_ACTIVE"] / 8 / (mean["ms"] * 1e-3) / 1e6
            print(f"  effective clock              {clk:.0f} MHz")
            if "SQ_VALU_MFMA_BUSY_CYCLES" in mean:
                util = mean["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * mean["GRBM_GUI_ACTIVE"] / 8)
                print(f"  MFMA pipe busy               {100 * util:.1f} %")


if __name__ == "__main__":
    main()
