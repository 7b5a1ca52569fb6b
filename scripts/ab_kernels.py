#!/usr/bin/env python3
"""Interleaved A/B timing of kernel variants in ONE process (cdna guide §5.4 rule 24).

    MIKMEANS_AB=1 python -m mikmeans._build   # the variant knobs need the A/B build
    python scripts/ab_kernels.py --n 20000000 --d 128 --k 1024 --dtype bf16 --rounds 5

Times the assign kernel for every points-per-wave variant and the update kernel,
reporting median / min ms and the achieved MFMA TFLOP/s of the assign.
"""
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
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--variants", default="32p2,16g2,16g1v1,16g1v2,16g2v3,16g2v4")
    a = ap.parse_args()

    from mikmeans.data.blobs import make_blobs
    from mikmeans.models.lloyd import LloydEngine
    from mikmeans.ops import native

    C = native.require()
    dt = torch.bfloat16 if a.dtype in ("bf16", "bfloat16") else torch.float32
    X = make_blobs(a.n, a.d, a.k, seed=0, dtype=dt, device="cuda")
    eng = LloydEngine(X, a.k).set_centers(X[: a.k].float())
    eng.step()
    torch.cuda.synchronize()
    # variants: "32pP" = 32x32 MFMA with P point-blocks per wave; "16gG" = 16x16 MFMA, G tiles/epilogue
    from mikmeans.ops import CentroidPack

    variants = a.variants.split(",")
    packs = {}
    for v in variants:
        lay = 116 if v.startswith("res") else (16 if v.startswith("16") else 32)
        if lay not in packs:
            packs[lay] = CentroidPack(a.k, eng.Dp, dt, "cuda", layout=lay).load(eng.C[:, : eng.Dp])
    res = {f"assign_{v}": [] for v in variants}
    res["update"] = []
    res["step"] = []
    ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
    for _ in range(a.rounds):
        for v in variants:
            lay = 116 if v.startswith("res") else (16 if v.startswith("16") else 32)
            if lay == 116:
                C.set_assign_res_grid(int(v[3:]) if len(v) > 3 else 0)   # "res" or "res<grid>"
            elif lay == 32:
                C.set_assign_p(int(v.split("p")[1]))
            else:
                gpart = v.split("g")[1]
                C.set_assign16_gt(int(gpart.split("v")[0]))
                C.set_assign16_cfg(int(gpart.split("v")[1]) if "v" in gpart else 0)
            e0, e1 = ev(), ev()
            e0.record()
            packs[lay].assign(eng.X, eng.xn, eng.labels, None, eng.slots, True)
            e1.record()
            torch.cuda.synchronize()
            res[f"assign_{v}"].append(e0.elapsed_time(e1))
        C.set_assign_p(0)
        C.set_assign_res_grid(0)
        C.set_assign16_gt(0)
        C.set_assign16_cfg(0)
        e0, e1 = ev(), ev()
        e0.record()
        C.update(eng.X, eng.labels, eng.K, eng.slab, eng.cnt_slab, eng.n_chunks, None, eng.col_exp, 0, False)
        e1.record()
        torch.cuda.synchronize()
        res["update"].append(e0.elapsed_time(e1))
        e0, e1 = ev(), ev()
        e0.record()
        eng.step()
        e1.record()
        torch.cuda.synchronize()
        res["step"].append(e0.elapsed_time(e1))
    flop = 2.0 * a.n * a.k * a.d
    out = {}
    for k, v in res.items():
        out[k] = {"median_ms": statistics.median(v), "min_ms": min(v)}
        if k.startswith("assign"):
            out[k]["tflops"] = flop / (statistics.median(v) * 1e-3) / 1e12
    print(json.dumps({"n": a.n, "d": a.d, "k": a.k, "dtype": a.dtype, **out}, indent=1))


if __name__ == "__main__":
    main()
