#!/usr/bin/env python3
"""In-process A/B of assign variants on the bench's own data (blobs, bench init) per config.

    python scripts/ab_shapes.py --config cfg4 --variants 16g1,32p4 --rounds 5
Variants as in ab_kernels.py: 16gG (16x16 MFMA, G=1 the GT1 default path), 32pP.
"""
import argparse
import json
import statistics
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg4")
    ap.add_argument("--variants", default="16g1,32p4")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--points", type=int, default=None)
    a = ap.parse_args()
    import bench
    from mikmeans.data.blobs import blob_centers, make_blobs
    from mikmeans.models.init import init_kmeanspp, init_random
    from mikmeans.models.lloyd import LloydEngine
    from mikmeans.ops import CentroidPack, native
    from mikmeans.parallel import Comm

    C = native.require()
    cfg = dict(bench.CONFIGS[a.config])
    if a.config == "cfg5":
        cfg["n"] = 1 << 24                      # one mini-batch of the stream
    if a.points:
        cfg["n"] = a.points
    N, D, K = cfg["n"], cfg["d"], cfg["k"]
    dt = torch.bfloat16 if cfg["dtype"] == "bfloat16" else torch.float32
    comm = Comm.local("cuda")
    X = make_blobs(N, D, K, seed=0, dtype=dt, device="cuda", centers=blob_centers(K, D, 10.0, 0, device="cuda"))
    C0 = (init_kmeanspp if a.config == "cfg4" else init_random)(X, D, K, N, 0, comm, 0)
    eng = LloydEngine(X, K, comm=comm).set_centers(C0)
    for _ in range(3):
        eng.step()
    torch.cuda.synchronize()
    variants = a.variants.split(",")
    packs = {}
    for v in variants:
        lay = 16 if v.startswith("16") else 32
        if lay not in packs:
            packs[lay] = CentroidPack(K, eng.Dp, dt, "cuda", layout=lay).load(eng.C[:, : eng.Dp])
    res = {v: [] for v in variants}
    for _ in range(a.rounds):
        for v in variants:
            lay = 16 if v.startswith("16") else 32
            if lay == 32:
                C.set_assign_p(int(v.split("p")[1]))
            else:
                C.set_assign16_gt(int(v.split("g")[1]))
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(3):
                packs[lay].assign(eng.X, eng.xn, eng.labels, None, eng.slots, True)
            e1.record()
            torch.cuda.synchronize()
            res[v].append(e0.elapsed_time(e1) / 3)
    C.set_assign_p(0)
    C.set_assign16_gt(0)
    flop = 2.0 * N * K * D
    print(json.dumps({"config": a.config, "n": N, "d": D, "k": K,
                      **{v: {"median_ms": statistics.median(t), "min_ms": min(t),
                             "tflops": flop / statistics.median(t) / 1e9} for v, t in res.items()}}))


if __name__ == "__main__":
    main()
