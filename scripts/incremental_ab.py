#!/usr/bin/env python3
"""Full vs incremental M-step, iteration by iteration, on the headline data (one GPU).

Two engines share X and start from the same centres; each iteration is timed with
events for both, and the centres must stay bitwise equal.  Prints one JSON line per
iteration: n_changed, full_ms, incr_ms.
"""
import argparse
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100_000_000)
    ap.add_argument("--d", type=int, default=128)
    ap.add_argument("--k", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--cap", type=float, default=0.125)
    a = ap.parse_args()
    from mikmeans.data.blobs import blob_centers, make_blobs
    from mikmeans.models.init import init_random
    from mikmeans.models.lloyd import LloydEngine
    from mikmeans.parallel import Comm

    comm = Comm.local("cuda")
    cen = blob_centers(a.k, a.d, 10.0, 0, device="cuda")
    X = make_blobs(a.n, a.d, a.k, seed=0, dtype=torch.bfloat16, device="cuda", centers=cen)
    C0 = init_random(X, a.d, a.k, a.n, 0, comm, 0)
    full = LloydEngine(X, a.k, comm=comm).set_centers(C0)
    inc = LloydEngine(X, a.k, comm=comm, incremental=True, delta_cap=a.cap).set_centers(C0)
    for it in range(a.iters):
        row = {"iter": it}
        for name, eng in (("full", full), ("incr", inc)):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            eng.step()
            e1.record()
            torch.cuda.synchronize()
            row[f"{name}_ms"] = round(e0.elapsed_time(e1), 3)
        row["n_changed"] = full.last_stats().n_changed
        row["equal"] = bool(torch.equal(full.centers, inc.centers))
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
