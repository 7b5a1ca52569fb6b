"""A/B of assign-kernel variants selected by an environment switch (default: the value-only
argmin MIKMEANS_ASSIGN_VARG=1 against the packed 6-bit keys =0) in one process, interleaved rounds, on Gaussian blobs at the cfg4 shape
(N=1e7, D=64, K=4096 bf16) and optionally others: median ms, TF/s and label agreement."""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from mikmeans import ops
from mikmeans.ops import native
from mikmeans.data import blobs as B


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="10000000,64,4096;2000000,64,2048;2000000,64,1024;4000000,32,1024;4000000,32,512;4000000,32,256")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--env", default="assign_varg", help="kernel variant switched between the arms (native.set_variant)")
    ap.add_argument("--values", default="0,1", help="its values, one arm each (first = baseline)")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f32"])
    args = ap.parse_args()
    for sh in args.shapes.split(";"):
        n, d, k = (int(v) for v in sh.split(","))
        dt = torch.bfloat16 if args.dtype == "bf16" else torch.float32
        X = B.make_blobs(n, d, 256, seed=d, dtype=dt, device="cuda")
        C = X[torch.randperm(n, generator=torch.Generator().manual_seed(1))[:k].cuda()].float()
        pack = ops.pack_centers(C, d, dt, "cuda")
        xn = ops.row_sqnorm(X)
        vals = args.values.split(",")
        labels = {v: torch.empty(n, dtype=torch.int32, device="cuda") for v in vals}
        times = {v: [] for v in vals}
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        for rd in range(args.rounds):
            for v in (vals if rd % 2 == 0 else vals[::-1]):
                native.set_variant(args.env, int(v))
                pack.assign(X, xn, labels[v])            # warm
                ev[0].record()
                for _ in range(args.reps):
                    pack.assign(X, xn, labels[v])
                ev[1].record()
                torch.cuda.synchronize()
                times[v].append(ev[0].elapsed_time(ev[1]) / args.reps)
        flop = 2.0 * n * k * d
        out = {"n": n, "d": d, "k": k, "dtype": args.dtype, "env": args.env}
        base = statistics.median(times[vals[0]])
        for v in vals:
            ms = statistics.median(times[v])
            out[v] = {"median_ms": round(ms, 4), "min_ms": round(min(times[v]), 4),
                      "tflops": round(flop / ms / 1e9, 1), "speedup": round(base / ms, 4),
                      "label_mismatch": int((labels[vals[0]] != labels[v]).sum())}
        print(json.dumps(out), flush=True)
    native.set_variant(args.env, -1)


if __name__ == "__main__":
    main()
