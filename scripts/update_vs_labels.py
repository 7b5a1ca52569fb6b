#!/usr/bin/env python3
"""M-step time on the headline data: Lloyd labels vs uniform random vs shuffled Lloyd labels.

Separates label-distribution effects (skewed cluster sizes -> hot-label flushes) from
everything else around the update kernel in bench.py.
"""
import argparse
import json
import statistics
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100_000_000)
    ap.add_argument("--iters", type=int, default=8)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    from mikmeans.data.blobs import blob_centers, make_blobs
    from mikmeans.models.init import init_random
    from mikmeans.models.lloyd import LloydEngine
    from mikmeans.parallel import Comm

    comm = Comm.local("cuda")
    D, K = 128, 1024
    cen = blob_centers(K, D, 10.0, 0, device="cuda")
    X = make_blobs(a.n, D, K, seed=0, dtype=torch.bfloat16, device="cuda", centers=cen)
    eng = LloydEngine(X, K, comm=comm).set_centers(init_random(X, D, K, a.n, 0, comm, 0))
    for _ in range(a.iters):
        eng.step()
    torch.cuda.synchronize()
    C = eng._C
    lab = eng.labels.clone()
    cnt = torch.bincount(lab.long(), minlength=K)
    variants = {
        "lloyd": lab,
        "uniform": torch.randint(0, K, (a.n,), device="cuda", dtype=torch.int32),
        "shuffled": lab[torch.randperm(a.n, device="cuda")].contiguous(),
    }
    out = {"count_max_over_mean": float(cnt.max()) / float(cnt.float().mean()),
           "empty": int((cnt == 0).sum())}
    for name, l in variants.items():
        C.update(eng.X, l, K, eng.slab, eng.cnt_slab, eng.n_chunks, None, eng.col_exp, 0, False)
        ts = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            C.update(eng.X, l, K, eng.slab, eng.cnt_slab, eng.n_chunks, None, eng.col_exp, 0, False)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        out[name] = round(statistics.median(ts), 4)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
