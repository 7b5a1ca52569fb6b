#!/usr/bin/env python3
"""Summarise rocprofv3 CSV outputs (kernel stats, PMC counters) into markdown for profiles/.

usage: summarize_prof.py <rocprof output dir> [--title T] [--clock-kernel NAME]
"""
import argparse
import csv
import glob
import os
import sys
from collections import defaultdict


def kernel_stats(d, limit=20):
    fs = sorted(glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True), key=os.path.getmtime)
    if not fs:
        return None
    rows = list(csv.DictReader(open(fs[-1])))
    out = ["| kernel | calls | avg ms | total ms | % |", "|---|---:|---:|---:|---:|"]
    for r in rows[:limit] if limit else rows:
        out.append(f"| `{r['Name'][:90]}` | {r['Calls']} | {float(r['AverageNs'])/1e6:.3f} | "
                   f"{float(r['TotalDurationNs'])/1e6:.2f} | {float(r['Percentage']):.2f} |")
    return "\n".join(out)


def pmc(d):
    fs = sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True), key=os.path.getmtime)
    if not fs:
        return None
    agg = defaultdict(lambda: defaultdict(float))
    calls = defaultdict(set)
    for f in fs:
        for r in csv.DictReader(open(f)):
            k = r.get("Kernel_Name", r.get("Kernel-Name", "?"))[:70]
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            calls[k].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
    out = []
    for k, cs in agg.items():
        n = max(1, len(calls[k]))
        out.append(f"**`{k}`** ({n} dispatches, per-dispatch means)\n")
        out.append("| counter | value |\n|---|---:|")
        for c, v in sorted(cs.items()):
            out.append(f"| {c} | {v / n:.4g} |")
        out.append("")
    return "\n".join(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--title", default="rocprofv3 summary")
    ap.add_argument("--all", action="store_true", help="every kernel, not the top 20")
    a = ap.parse_args()
    parts = [f"# {a.title}\n"]
    ks = kernel_stats(a.dir, 0 if a.all else 20)
    if ks:
        parts += ["## Kernel time (rocprofv3 --kernel-trace --stats)\n", ks, ""]
    pm = pmc(a.dir)
    if pm:
        parts += ["## PMC counters\n", pm]
    print("\n".join(parts))


if __name__ == "__main__":
    sys.exit(main())
