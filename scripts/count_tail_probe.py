#!/usr/bin/env python3
"""What the device-counted gathered assign (the bounded E-step's launch) pays for its grid:
the host cannot know how many rows the compaction kept, so the grid covers every row and the
workgroups past the device count leave at once.  This times the same gathered assign of m rows
(bounds, per-row seed offsets, scatter -- as lloyd.py launches it) with the grid sized for N
rows and the count on the device, against the grid sized for exactly m rows.

usage: count_tail_probe.py [--n 100000000] [--m 11000000,5000000,30000000]"""
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
    ap.add_argument("--n", type=int, default=100_000_000)
    ap.add_argument("--d", type=int, default=128)
    ap.add_argument("--k", type=int, default=1024)
    ap.add_argument("--m", default="11000000,5000000,30000000")
    a = ap.parse_args()
    dev = torch.device("cuda")
    comm = Comm.local(dev)
    X = make_blobs(a.n, a.d, a.k, seed=0, dtype=torch.bfloat16, device=dev,
                   centers=blob_centers(a.k, a.d, 10.0, 0, device=dev))
    eng = LloydEngine(X, a.k, comm=comm).set_centers(init_random(X, a.d, a.k, a.n, 0, comm, 0))
    for _ in range(3):
        eng.step()
    pk = eng.pk
    oseed = pk.seed_offsets(eng.xn)
    g = torch.Generator(device=dev).manual_seed(1)
    out = {"n": a.n, "d": a.d, "k": a.k}
    for m in [int(v) for v in a.m.split(",")]:
        rows = torch.randperm(a.n, device=dev, generator=g)[:m].sort().values
        buf = torch.zeros(a.n, dtype=torch.int64, device=dev)
        buf[:m] = rows
        cnt = torch.tensor([m], dtype=torch.int64, device=dev)
        res = {}
        for tag, r, c in (("grid_N_count_on_device", buf, cnt), ("grid_m", rows, None)):
            lab = eng.labels.clone()
            ub = torch.empty(a.n, dtype=torch.float32, device=dev)
            lb = torch.empty(a.n, dtype=torch.float32, device=dev)
            slots = torch.zeros_like(eng.slots)

            def call(r=r, c=c, lab=lab, ub=ub, lb=lb, slots=slots):
                pk.assign(X, eng.xn, lab, None, slots, True, rows=r, ub=ub, lb=lb, scatter=True, count=c,
                          oseed=oseed)
            res[tag] = {"ms": round(timed(call), 4)}
            res[tag]["labels"] = lab
        res["labels_equal"] = bool(torch.equal(res["grid_N_count_on_device"].pop("labels"),
                                               res["grid_m"].pop("labels")))
        out[f"m={m}"] = res
        print(json.dumps({f"m={m}": res}), flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
