#!/usr/bin/env python3
"""The bounded (Hamerly) E-step + incremental M-step -- the library's default path
(KMeans(algorithm="auto")) -- on the headline data, alone in a process so a kernel trace
shows only its steps: the same start as bench.py (blobs, random rows as centres), W warm-up
steps then S timed ones (graph replay like the bench), ms per step and rows re-assigned.

usage: bounded_profile.py [--n 100000000] [--d 128] [--k 1024] [--steps 20] [--warmup 5]"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from mikmeans.data.blobs import blob_centers, make_blobs  # noqa: E402
from mikmeans.models.init import init_random  # noqa: E402
from mikmeans.models.lloyd import LloydEngine  # noqa: E402
from mikmeans.parallel import Comm  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100_000_000)
    ap.add_argument("--d", type=int, default=128)
    ap.add_argument("--k", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--bounded", action=argparse.BooleanOptionalAction, default=True,
                    help="--no-bounded: the full E-step with the incremental M-step (algorithm='lloyd')")
    a = ap.parse_args()
    dev = torch.device("cuda")
    comm = Comm.local(dev)
    X = make_blobs(a.n, a.d, a.k, seed=0, dtype=torch.bfloat16, device=dev,
                   centers=blob_centers(a.k, a.d, 10.0, 0, device=dev))
    C0 = init_random(X, a.d, a.k, a.n, 0, comm, 0)
    eng = LloydEngine(X, a.k, comm=comm, incremental=True, bounded=a.bounded).set_centers(C0)
    eng.capture()
    per = []
    for i in range(a.warmup + a.steps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.step()
        torch.cuda.synchronize()
        if i >= a.warmup:
            per.append({"ms": round((time.perf_counter() - t0) * 1e3, 3),
                        "reassigned": int(eng.reassigned) if a.bounded else a.n})
    tot = sum(p["ms"] for p in per)
    print(json.dumps({"n": a.n, "d": a.d, "k": a.k, "steps": a.steps, "ms_per_step": round(tot / a.steps, 3),
                      "it_per_s": round(1e3 * a.steps / tot, 1), "per_step": per}), flush=True)


if __name__ == "__main__":
    main()
