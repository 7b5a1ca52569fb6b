#!/usr/bin/env python3
"""A/B of assign-kernel variants (mikmeans.ops.native.set_variant) in one process, interleaved
rounds, on the bench's blob data a few Lloyd iterations in.

usage: assign_ab.py [--n N] [--d D] [--k K] [--dtype bf16|f32] [--rounds R] [--reps M]
                    --arms "assign_persist=0;assign_persist=1;assign_geom=4,assign_persist=1"
Prints one JSON line per shape: median / min ms per arm, TF/s, and whether every arm's labels
equal the first arm's (bitwise).
"""
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
from mikmeans.ops import native  # noqa: E402
from mikmeans.parallel import Comm  # noqa: E402


def parse_arm(spec: str) -> dict:
    out = {}
    for kv in filter(None, spec.split(",")):
        if kv.strip() in ("default", "-"):
            continue
        k, v = kv.split("=")
        out[k.strip()] = int(v)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=20_000_000)
    ap.add_argument("--d", type=int, default=128)
    ap.add_argument("--k", type=int, default=1024)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--arms", default="assign_persist=0;assign_persist=1")
    ap.add_argument("--gather", type=int, default=0,
                    help="> 0: time the gathered assign of this many random rows (the mini-batch "
                         "resident path: X[rows] read in place, norms from the fragments)")
    a = ap.parse_args()
    dt = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    dev = torch.device("cuda")
    comm = Comm.local(dev)
    X = make_blobs(a.n, a.d, a.k, seed=0, dtype=dt, device=dev, centers=blob_centers(a.k, a.d, 10.0, 0, device=dev))
    eng = LloydEngine(X, a.k, comm=comm).set_centers(init_random(X, a.d, a.k, a.n, 0, comm, 0))
    for _ in range(3 if not a.gather else 1):
        eng.step()
    if a.gather:
        g = torch.Generator(device=dev).manual_seed(5)
        rows = torch.randint(0, a.n, (a.gather,), device=dev, generator=g)
        glab = torch.empty(a.gather, dtype=torch.int32, device=dev)

        def call():
            eng.pk.assign(eng.X, None, glab, None, eng.slots, False, rows=rows)
    else:
        def call():
            eng.pk.assign(eng.X, eng.xn, eng.labels, eng.mind, eng.slots, True)
    arms = [parse_arm(s) for s in a.arms.split(";")]
    names = [s or "default" for s in a.arms.split(";")]
    labels = {}
    times = {n: [] for n in names}
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]

    def run(arm):
        old = {k: native.get_variant(k) for k in arm}
        for k, v in arm.items():
            native.set_variant(k, v)
        try:
            call()   # warm / attributes
            ev[0].record()
            for _ in range(a.reps):
                call()
            ev[1].record()
            torch.cuda.synchronize()
            return ev[0].elapsed_time(ev[1]) / a.reps, (glab if a.gather else eng.labels).clone()
        finally:
            for k, v in old.items():
                native.set_variant(k, v)

    for rd in range(a.rounds):
        order = list(zip(names, arms)) if rd % 2 == 0 else list(zip(names, arms))[::-1]
        for n, arm in order:
            t, lab = run(arm)
            times[n].append(t)
            labels.setdefault(n, lab)
    ref = labels[names[0]]
    res = {"n": a.n, "d": a.d, "k": a.k, "dtype": a.dtype, "rounds": a.rounds, "reps": a.reps,
           "gathered_rows": a.gather}
    m = a.gather or a.n
    for n in names:
        med = statistics.median(times[n])
        res[n] = {"median_ms": round(med, 4), "min_ms": round(min(times[n]), 4),
                  "tflops": round(2.0 * m * a.k * a.d / (med * 1e-3) / 1e12, 1),
                  "labels_equal": bool(torch.equal(labels[n], ref))}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
