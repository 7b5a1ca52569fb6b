#!/usr/bin/env python3
"""Time the on-device blob generator (csrc/kpp.hip blobs_kernel) at the cfg5 batch shape.

usage: blobs_bench.py [--n N] [--d D] [--k K] [--reps R]
Prints one JSON line: ms per batch with and without fused row norms, and the write rate."""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mikmeans.data.blobs import blob_centers, make_blobs  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 24)
    ap.add_argument("--d", type=int, default=256)
    ap.add_argument("--k", type=int, default=512)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--tpr", default="", help="comma list of lanes-per-row A/B arms (variant blobs_tpr)")
    a = ap.parse_args()
    dev = torch.device("cuda")
    c = blob_centers(a.k, a.d, 10.0, 0, device=dev)
    X = torch.empty((a.n, a.d), dtype=torch.bfloat16, device=dev)
    xn = torch.empty(a.n, dtype=torch.float32, device=dev)
    res = {"n": a.n, "d": a.d, "k": a.k}
    for name, norms in (("plain", None), ("norms", xn)):
        ts = []
        for r in range(a.reps + 2):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            make_blobs(a.n, a.d, a.k, seed=r, i0=r * a.n, dtype=torch.bfloat16, device=dev, centers=c, out=X,
                       norms=norms)
            e1.record()
            torch.cuda.synchronize()
            if r >= 2:
                ts.append(e0.elapsed_time(e1))
        ms = statistics.median(ts)
        res[name] = {"median_ms": round(ms, 4), "min_ms": round(min(ts), 4),
                     "write_TBps": round(X.numel() * 2 / (ms * 1e-3) / 1e12, 3)}
    if a.tpr:
        from mikmeans.ops import native

        ref = X.clone()
        for tv in [int(t) for t in a.tpr.split(",")]:
            native.set_variant("blobs_tpr", tv)
            ts = []
            for r in range(a.reps + 2):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                make_blobs(a.n, a.d, a.k, seed=a.reps + 1, i0=(a.reps + 1) * a.n, dtype=torch.bfloat16,
                           device=dev, centers=c, out=X, norms=xn)
                e1.record()
                torch.cuda.synchronize()
                if r >= 2:
                    ts.append(e0.elapsed_time(e1))
            res[f"tpr{tv}"] = {"median_ms": round(statistics.median(ts), 4), "same_rows": bool(torch.equal(X, ref))}
        native.set_variant("blobs_tpr", -1)
    # the write floor: torch's vectorised fill of the same bytes
    ts = []
    for r in range(a.reps + 2):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        X.fill_(float(r))
        e1.record()
        torch.cuda.synchronize()
        if r >= 2:
            ts.append(e0.elapsed_time(e1))
    ms = statistics.median(ts)
    res["fill"] = {"median_ms": round(ms, 4), "write_TBps": round(X.numel() * 2 / (ms * 1e-3) / 1e12, 3)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
