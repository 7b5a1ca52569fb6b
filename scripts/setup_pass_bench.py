#!/usr/bin/env python3
"""The fit's setup passes over X at the headline shape (N=1e8, D=128, bf16): row norms, the
column statistics alone, and the fused statistics + row norms pass (csrc/finalize.hip), each
timed with device events; and the LloydEngine constructor end to end.

usage: setup_pass_bench.py [--n N] [--d D] [--reps R]"""
import argparse
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from mikmeans import ops  # noqa: E402
from mikmeans.data.blobs import blob_centers, make_blobs  # noqa: E402
from mikmeans.models.lloyd import LloydEngine  # noqa: E402


def timed(fn, reps):
    ts = []
    for _ in range(reps + 1):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    ts = ts[1:]
    return {"median_ms": round(statistics.median(ts), 3), "min_ms": round(min(ts), 3)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100_000_000)
    ap.add_argument("--d", type=int, default=128)
    ap.add_argument("--k", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--blocks", default="", help="comma list of statistics-grid block caps to A/B")
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda")
    X = make_blobs(a.n, a.d, a.k, seed=0, dtype=torch.bfloat16, device=dev,
                   centers=blob_centers(a.k, a.d, 10.0, 0, device=dev))
    xn = torch.empty(a.n, dtype=torch.float32, device=dev)
    gb = X.numel() * X.element_size() / 1e9
    res = {"n": a.n, "d": a.d, "X_GB": round(gb, 2)}
    res["row_sqnorm"] = timed(lambda: ops.row_sqnorm(X), a.reps)
    res["col_stats"] = timed(lambda: ops.col_stats(X), a.reps)
    res["col_stats_fused_norms"] = timed(lambda: ops.col_stats(X, xn=xn), a.reps)
    for k in ("row_sqnorm", "col_stats", "col_stats_fused_norms"):
        res[k]["TBps"] = round(gb / (res[k]["median_ms"] * 1e-3) / 1e3, 2)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng = LloydEngine(X, a.k)
    torch.cuda.synchronize()
    res["engine_init_s"] = round(time.perf_counter() - t0, 4)
    res["fused_norms_equal_row_sqnorm"] = bool(torch.equal(eng.xn, ops.row_sqnorm(X)))
    if a.blocks:   # A/B of the statistics grid's block cap (switch colstat_blocks), interleaved
        from mikmeans.ops import native

        arms = [int(b) for b in a.blocks.split(",")]
        ts = {b: [] for b in arms}
        for _ in range(a.rounds):
            for b in arms:
                with native.variant("colstat_blocks", b):
                    ts[b].append(timed(lambda: ops.col_stats(X, xn=xn), a.reps)["median_ms"])
        res["blocks_ab"] = {str(b): round(statistics.median(v), 3) for b, v in ts.items()}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
