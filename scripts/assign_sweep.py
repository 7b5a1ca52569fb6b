#!/usr/bin/env python3
"""Throughput map of the full assign pass (the E-step) and the M-step over shapes: for each
(D, K, dtype) at a fixed row count, the median time of the assign kernel over its data (a few
Lloyd steps in, so the centres are realistic) and of the M-step pass, as TF/s (2 N K D) and
TB/s (X bytes).  A table for choosing shapes, not a benchmark of record.

usage: assign_sweep.py [--n 10000000] [--d 32,64,128,256,512] [--k 64,256,1024,4096] [--dtypes bf16,f32]"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from mikmeans.data.blobs import blob_centers, make_blobs  # noqa: E402
from mikmeans.models.init import init_random  # noqa: E402
from mikmeans.models.lloyd import LloydEngine  # noqa: E402
from mikmeans.parallel import Comm  # noqa: E402


def timed(fn, reps=5):
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
    ap.add_argument("--n", type=int, default=10_000_000)
    ap.add_argument("--d", default="32,64,128,256,512")
    ap.add_argument("--k", default="64,256,1024,4096")
    ap.add_argument("--dtypes", default="bf16,f32")
    ap.add_argument("--what", default="both", choices=["both", "assign", "mstep"],
                    help="time one kernel only (a counter run over one of them)")
    a = ap.parse_args()
    dev = torch.device("cuda")
    comm = Comm.local(dev)
    rows = []
    for dts in a.dtypes.split(","):
        dt = torch.bfloat16 if dts == "bf16" else torch.float32
        for d in [int(v) for v in a.d.split(",")]:
            X = None
            for k in [int(v) for v in a.k.split(",")]:
                n = a.n if dts == "bf16" else a.n // 4      # (f32: 16x fewer MFMA FLOP/s; keep it short)
                if X is None or X.shape[0] != n:
                    X = make_blobs(n, d, 64, seed=d, dtype=dt, device=dev,
                                   centers=blob_centers(64, d, 10.0, 0, device=dev))
                eng = LloydEngine(X, k, comm=comm, incremental=False).set_centers(
                    init_random(X, d, k, n, 0, comm, 0))
                for _ in range(2):
                    eng.step()
                ta = tm = float("nan")
                if a.what != "mstep":
                    ta = timed(lambda: eng.pk.assign(eng.X, eng.xn, eng.labels, eng.mind, eng.slots, True))
                if a.what != "assign":
                    tm = timed(lambda: eng._C.update(eng.X, eng.labels, eng.K, eng.slab, eng.cnt_slab, eng.n_chunks,
                                                     eng.weights, eng.col_exp, eng.cnt_exp, False))
                xb = X.numel() * X.element_size()
                r = {"dtype": dts, "n": n, "d": d, "k": k, "assign_ms": round(ta, 4),
                     "assign_tflops": round(2.0 * n * k * d / (ta * 1e-3) / 1e12, 1),
                     "mstep_ms": round(tm, 4), "mstep_TBps": round(xb / (tm * 1e-3) / 1e12, 2),
                     "it_per_s_estimate": round(1e3 / (ta + tm), 1) if a.what == "both" else None}
                rows.append(r)
                print(json.dumps(r), flush=True)
                del eng
    print(json.dumps({"sweep": rows}), flush=True)


if __name__ == "__main__":
    main()
