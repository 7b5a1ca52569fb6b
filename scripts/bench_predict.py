#!/usr/bin/env python3
"""Serving latency / throughput of KMeans.predict on one GPU (K=1024, D=128 bf16 by default).

    python scripts/bench_predict.py [--k 1024 --d 128 --calls 50]

Per batch size: median wall time of one synchronised predict() call with the packed
centres cached on the model (default) and rebuilt per call (the pre-cache path), and
the MFMA assign kernel alone.
"""
import argparse
import json
import statistics
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=1024)
    ap.add_argument("--d", type=int, default=128)
    ap.add_argument("--calls", type=int, default=50)
    ap.add_argument("--batches", default="1024,16384,262144,4194304")
    a = ap.parse_args()

    import mikmeans
    from mikmeans import ops

    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    km = mikmeans.KMeans(a.k, dtype="bfloat16")
    km.cluster_centers_ = torch.randn(a.k, a.d, device=dev, generator=g)
    km.n_features_in_ = a.d
    out = {"k": a.k, "d": a.d, "dtype": "bf16", "rows": []}
    for b in [int(x) for x in a.batches.split(",")]:
        X = torch.randn(b, a.d, device=dev, generator=g).to(torch.bfloat16)

        def timed(fn):
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            ts = []
            for _ in range(a.calls):
                t0 = time.perf_counter()
                fn()
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
            return statistics.median(ts) * 1e6

        cached = timed(lambda: km.predict(X))
        fresh = timed(lambda: ops.assign(X, km.cluster_centers_, with_dist=False))
        pk = km._serving_pack(X)
        lab = torch.empty(b, dtype=torch.int32, device=dev)
        kern = timed(lambda: pk.assign(X, None, lab))
        out["rows"].append({"batch": b, "predict_us": round(cached, 1), "uncached_us": round(fresh, 1),
                            "kernel_only_us": round(kern, 1),
                            "predict_points_per_s": b / (cached * 1e-6)})
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
