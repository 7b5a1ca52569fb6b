#!/usr/bin/env python3
"""A/B k-means++ seeding with and without triangle-inequality pruning (one process).

Both arms must give bitwise-identical centres; prints the seeding wall time of each.
    python scripts/ab_kpp_prune.py --n 10000000 --d 64 --k 4096     # BASELINE config 4
"""
import argparse
import json
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=10_000_000)
    ap.add_argument("--d", type=int, default=64)
    ap.add_argument("--k", type=int, default=4096)
    ap.add_argument("--rounds", type=int, default=2)
    a = ap.parse_args()
    from mikmeans.data.blobs import make_blobs
    from mikmeans.models import init as I
    from mikmeans.parallel import Comm

    X = make_blobs(a.n, a.d, a.k, seed=0, dtype=torch.bfloat16, device="cuda")
    comm = Comm.local("cuda")
    res = {"full": [], "prune": []}
    ref = None
    for _ in range(a.rounds):
        for arm in ("full", "prune"):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            C = I.init_kmeanspp(X, a.d, a.k, a.n, 0, comm, seed=0, prune=(arm == "prune"))
            torch.cuda.synchronize()
            res[arm].append(round(time.perf_counter() - t0, 4))
            if ref is None:
                ref = C
            assert torch.equal(C, ref), f"{arm} changed the centres"
            print(arm, res[arm][-1], flush=True)
    print(json.dumps({"n": a.n, "d": a.d, "k": a.k, "bitwise_equal": True,
                      **{k: {"min_s": min(v), "all_s": v} for k, v in res.items()}}))


if __name__ == "__main__":
    main()
