#!/usr/bin/env python3
"""Concurrency in a rocprofv3 kernel trace: over the last N dispatches of the named kernel
family, the GPU's busy time (union of kernel intervals), its idle gaps, and how much of each
kernel's time overlapped another kernel (side-stream work such as the blob generator's
prefetch hiding under the M-step).

usage: trace_overlap.py <rocprof output dir> [--last-steps 10] [--step-kernel assign16_kernel]
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def short(name: str) -> str:
    n = name.split("(")[0]
    base = n.split("<")[0].split("::")[-1].split()[-1] if n else n
    for key in ("assign16_kernel", "update_ks_kernel", "update_kernel", "bounds_update_kernel", "blobs_kernel",
                "reduce_kernel", "finalize_kernel", "sample_index_kernel", "col_absmax_kernel",
                "row_sqnorm_kernel", "label_delta_rows_kernel", "label_delta_kernel"):
        if base == key:
            return key
    return n.split("::")[-1][:40]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--last-steps", type=int, default=10)
    ap.add_argument("--step-kernel", default="assign16_kernel")
    a = ap.parse_args()
    fs = sorted(glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True), key=os.path.getmtime)
    rows = list(csv.DictReader(open(fs[-1])))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), int(r["Queue_Id"]))
                 for r in rows), key=lambda x: x[0])
    steps = [k for k in ks if k[2] == a.step_kernel]
    if len(steps) < a.last_steps + 1:
        raise SystemExit(f"only {len(steps)} {a.step_kernel} dispatches")
    t0, t1 = steps[-a.last_steps - 1][0], steps[-1][0]     # whole steps between two step kernels
    win = [(max(s, t0), min(e, t1), n, q) for s, e, n, q in ks if e > t0 and s < t1]
    # union busy time
    busy, cur_s, cur_e = 0, None, None
    for s, e, _, _ in sorted(win):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    per = defaultdict(lambda: {"ms": 0.0, "overlapped_ms": 0.0, "calls": 0})
    for i, (s, e, n, q) in enumerate(win):
        ov = 0
        for j, (s2, e2, n2, q2) in enumerate(win):
            if j != i:
                ov = max(ov, min(e, e2) - max(s, s2))
        p = per[n]
        p["ms"] += (e - s) / 1e6 / a.last_steps
        p["overlapped_ms"] += max(0, ov) / 1e6 / a.last_steps
        p["calls"] += 1
    span = (t1 - t0) / 1e6 / a.last_steps
    out = {"steps": a.last_steps, "ms_per_step": round(span, 4), "busy_ms_per_step": round(busy / 1e6 / a.last_steps, 4),
           "idle_ms_per_step": round(span - busy / 1e6 / a.last_steps, 4),
           "kernels": {n: {k: round(v, 4) if isinstance(v, float) else v for k, v in p.items()}
                       for n, p in sorted(per.items(), key=lambda x: -x[1]["ms"])},
           "queues": sorted({q for *_, q in win})}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
