#!/usr/bin/env python3
"""HBM ceilings beside the fit's one-time passes, at the headline's X (N=1e8, D=128, bf16,
25.6 GB): what a plain write (torch fill_ / zero_), a read + write (copy_) and a read-only
reduction reach on this box, next to the blob generator (writes X + labels + norms), the row
norms, and the column-statistics pass in its four forms (max only / + norms / + statistics /
+ both).  Device events, median of --reps after one warm call.

usage: hbm_ceiling.py [--n N] [--d D] [--reps R]"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from mikmeans import ops  # noqa: E402
from mikmeans.data.blobs import blob_centers, make_blobs  # noqa: E402


def timed(fn, reps):
    ts = []
    for _ in range(reps + 1):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return statistics.median(ts[1:])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100_000_000)
    ap.add_argument("--d", type=int, default=128)
    ap.add_argument("--k", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda")
    C = blob_centers(a.k, a.d, 10.0, 0, device=dev)
    X = make_blobs(a.n, a.d, a.k, seed=0, dtype=torch.bfloat16, device=dev, centers=C)
    gb = X.numel() * X.element_size() / 1e9
    xn = torch.empty(a.n, dtype=torch.float32, device=dev)
    res = {"n": a.n, "d": a.d, "X_GB": round(gb, 2)}

    def put(name, ms, gbytes):
        res[name] = {"ms": round(ms, 3), "TBps": round(gbytes / (ms * 1e-3) / 1e3, 2)}
        print(json.dumps({name: res[name]}), flush=True)

    Y = torch.empty_like(X)
    put("fill_write", timed(lambda: Y.fill_(1.0), a.reps), gb)
    put("zero_write", timed(lambda: Y.zero_(), a.reps), gb)
    put("copy_read_write", timed(lambda: Y.copy_(X), a.reps), 2 * gb)
    del Y
    Xi = X.view(torch.int16)
    put("amax_read_torch", timed(lambda: Xi.amax(), a.reps), gb)
    put("blobs_write", timed(lambda: make_blobs(a.n, a.d, a.k, seed=0, dtype=torch.bfloat16, device=dev,
                                                centers=C, out=X), a.reps), gb)
    put("blobs_write_norms", timed(lambda: make_blobs(a.n, a.d, a.k, seed=0, dtype=torch.bfloat16, device=dev,
                                                      centers=C, out=X, norms=xn), a.reps), gb)
    put("row_sqnorm", timed(lambda: ops.row_sqnorm(X), a.reps), gb)
    put("colmax", timed(lambda: ops.col_stats(X, stats=False), a.reps), gb)
    put("colmax_norms", timed(lambda: ops.col_stats(X, stats=False, xn=xn), a.reps), gb)
    put("colstats", timed(lambda: ops.col_stats(X), a.reps), gb)
    put("colstats_norms", timed(lambda: ops.col_stats(X, xn=xn), a.reps), gb)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
