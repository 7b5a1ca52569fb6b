#!/usr/bin/env python3
"""Where the bounded E-step's gathered assign spends its extra time per row (vs the full pass):
the same m rows assigned as lloyd.py's bounded step does (bounds ub/lb = TOP2 epilogue, per-row
seed offsets, scattered outputs) and with one feature removed at a time, plus contiguous rows
and the full pass over all N for the per-row baseline.

usage: gathered_assign_probe.py [--n 100000000] [--m 11000000]"""
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
    return round(statistics.median(ts[1:]), 4)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100_000_000)
    ap.add_argument("--d", type=int, default=128)
    ap.add_argument("--k", type=int, default=1024)
    ap.add_argument("--m", type=int, default=11_000_000)
    a = ap.parse_args()
    dev = torch.device("cuda")
    comm = Comm.local(dev)
    X = make_blobs(a.n, a.d, a.k, seed=0, dtype=torch.bfloat16, device=dev,
                   centers=blob_centers(a.k, a.d, 10.0, 0, device=dev))
    eng = LloydEngine(X, a.k, comm=comm).set_centers(init_random(X, a.d, a.k, a.n, 0, comm, 0))
    for _ in range(3):
        eng.step()
    pk, xn = eng.pk, eng.xn
    oseed = pk.seed_offsets(xn)
    g = torch.Generator(device=dev).manual_seed(1)
    rows = torch.randperm(a.n, device=dev, generator=g)[: a.m].sort().values
    contig = torch.arange(a.m, device=dev, dtype=torch.int64)
    lab = eng.labels.clone()
    mind = torch.empty(a.n, dtype=torch.float32, device=dev)
    ub = torch.empty(a.n, dtype=torch.float32, device=dev)
    lb = torch.empty(a.n, dtype=torch.float32, device=dev)
    slots = torch.zeros_like(eng.slots)
    res = {"n": a.n, "m": a.m}
    res["full_pass_all_rows"] = timed(lambda: pk.assign(X, xn, lab, mind, slots, True))
    res["full_pass_per_m_rows"] = round(res["full_pass_all_rows"] * a.m / a.n, 4)
    arms = {
        "bounded_as_lloyd_py": dict(rows=rows, ub=ub, lb=lb, scatter=True, oseed=oseed),
        "no_bounds_(keys_epilogue)": dict(rows=rows, scatter=True, oseed=oseed),
        "no_seed_offsets": dict(rows=rows, ub=ub, lb=lb, scatter=True),
        "no_scatter": dict(rows=rows, ub=ub[: a.m], lb=lb[: a.m], oseed=oseed),
        "contiguous_rows": dict(rows=contig, ub=ub, lb=lb, scatter=True, oseed=oseed),
    }
    for name, kw in arms.items():
        mm = mind if kw.get("scatter") else mind[: a.m]
        ll = lab if kw.get("scatter") else lab[: a.m].clone()
        res[name] = timed(lambda kw=kw, mm=mm, ll=ll: pk.assign(X, xn, ll, None, slots, True, **kw))
        print(json.dumps({name: res[name]}), flush=True)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
