#!/usr/bin/env python3
"""Per-kernel timing of one Lloyd step's phases on the bench's own data (one process).

usage: kbench.py [--n N] [--d D] [--k K] [--dtype bf16|f32] [--reps R]
Prints one JSON line: median / min ms of assign, update, reduce and the whole step,
plus the assign's MFMA TF/s.  Centres are a few Lloyd iterations in (like the bench's
timed steps), so the argmin sees realistic score distributions.
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from mikmeans.data.blobs import blob_centers, make_blobs
from mikmeans.models.init import init_random
from mikmeans.models.lloyd import LloydEngine
from mikmeans.parallel import Comm


def timed(fn, reps):
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return {"median_ms": round(statistics.median(ts), 4), "min_ms": round(min(ts), 4)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=20_000_000)
    ap.add_argument("--d", type=int, default=128)
    ap.add_argument("--k", type=int, default=1024)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--warm-iters", type=int, default=3)
    ap.add_argument("--slice-probe", action="store_true")
    a = ap.parse_args()
    dt = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    dev = torch.device("cuda")
    comm = Comm.local(dev)
    X = make_blobs(a.n, a.d, a.k, seed=0, dtype=dt, device=dev, centers=blob_centers(a.k, a.d, 10.0, 0, device=dev))
    eng = LloydEngine(X, a.k, comm=comm).set_centers(init_random(X, a.d, a.k, a.n, 0, comm, 0))
    for _ in range(a.warm_iters):
        eng.step()
    C = eng._C
    res = {"n": a.n, "d": a.d, "k": a.k, "dtype": a.dtype}
    res["assign"] = timed(lambda: eng.pk.assign(eng.X, eng.xn, eng.labels, eng.mind, eng.slots, True), a.reps)
    res["update"] = timed(lambda: C.update(eng.X, eng.labels, eng.K, eng.slab, eng.cnt_slab, eng.n_chunks, None,
                                           eng.col_exp, eng.cnt_exp, False), a.reps)
    res["reduce"] = timed(lambda: C.reduce(eng.slab, eng.cnt_slab, eng.n_chunks, eng.K, eng.Dp, eng.slots,
                                           eng.packed, eng.col_exp, eng.cnt_exp), a.reps)
    from mikmeans.ops import col_stats
    res["col_absmax"] = timed(lambda: col_stats(eng.X, stats=False), a.reps)   # streaming-read reference
    if a.slice_probe and a.d == 128:
        # EXPERIMENT: the same bytes as contiguous 64-B "rows" (what a slice-blocked layout of
        # X would give the M-step): X viewed as [4n, 32], random labels
        X4 = eng.X.reshape(-1, 32)
        lab4 = torch.randint(0, a.k, (X4.shape[0],), dtype=torch.int32, device=dev)
        nc4 = C.update_n_chunks(eng.dt, a.k, 32, X4.shape[0], False)
        slab4 = torch.empty(nc4 * a.k * 32, dtype=torch.int64, device=dev)
        cnt4 = torch.empty(nc4 * a.k, dtype=torch.int64, device=dev)
        ce4 = eng.col_exp[:32].contiguous()
        res["update_contig64"] = timed(lambda: C.update(X4, lab4, a.k, slab4, cnt4, nc4, None, ce4, 0, False), a.reps)
    res["step"] = timed(eng.step, a.reps)
    res["assign_tflops"] = round(2.0 * a.n * a.k * a.d / (res["assign"]["median_ms"] * 1e-3) / 1e12, 1)
    res["update_GBps"] = round(X.numel() * X.element_size() / (res["update"]["median_ms"] * 1e-3) / 1e9, 1)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
