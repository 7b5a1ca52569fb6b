#!/usr/bin/env python3
"""A/B the overlapped M-step (segments x slice width) against the serial step, one process."""
import argparse
import json
import statistics
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=20_000_000)
    ap.add_argument("--d", type=int, default=128)
    ap.add_argument("--k", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--configs", default="1:0,2:8,4:8,8:8,4:4,4:16,8:16")
    a = ap.parse_args()
    from mikmeans.data.blobs import make_blobs
    from mikmeans.models.lloyd import LloydEngine

    X = make_blobs(a.n, a.d, a.k, seed=0, dtype=torch.bfloat16, device="cuda")
    C0 = X[: a.k].float()
    engines = {}
    for cfg in a.configs.split(","):
        seg, sw = (int(v) for v in cfg.split(":"))
        engines[cfg] = LloydEngine(X, a.k, segments=seg, overlap_sw=sw).set_centers(C0)
    ref = None
    res = {c: [] for c in engines}
    for _ in range(a.rounds):
        for c, eng in engines.items():
            eng.set_centers(C0)
            eng.step()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.steps):
                eng.step()
            e1.record()
            torch.cuda.synchronize()
            res[c].append(e0.elapsed_time(e1) / a.steps)
            cen = eng.centers.clone()
            if ref is None:
                ref = cen
            assert torch.equal(cen, ref), f"config {c} changed the result"
    print(json.dumps({c: {"median_ms": statistics.median(v), "min_ms": min(v)} for c, v in res.items()},
                     indent=1))


if __name__ == "__main__":
    main()
