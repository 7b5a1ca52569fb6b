"""Does the order of a gathered mini-batch matter?  One resident shard (cfg5 shape, scaled by
--shard-rows), the same sampled rows per step in Philox order and sorted ascending: median
ms of partial_fit_rows (gathered assign + M-step + reduce + finalize) per arm, interleaved."""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from mikmeans.data import blobs as B
from mikmeans.models.minibatch import MiniBatchEngine
from mikmeans.ops import col_stats, native


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shard-rows", type=int, default=60_000_000)
    ap.add_argument("--batch", type=int, default=1 << 24)
    ap.add_argument("--d", type=int, default=256)
    ap.add_argument("--k", type=int, default=512)
    ap.add_argument("--steps", type=int, default=6)
    args = ap.parse_args()
    C = native.require()
    X = B.make_blobs(args.shard_rows, args.d, args.k, seed=1, dtype=torch.bfloat16, device="cuda")
    bound = col_stats(X, stats=False).absmax
    eng = MiniBatchEngine(args.k, args.d, args.batch, dtype=torch.bfloat16, device="cuda").set_bound(bound)
    rows = torch.empty(args.batch, dtype=torch.int64, device="cuda")
    C.sample_index(args.shard_rows, args.batch, 0, 0, 0, rows)
    eng.set_centers(X[rows[: args.k]].float())
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    t = {"philox_order": [], "sorted": []}
    for s in range(args.steps):
        C.sample_index(args.shard_rows, args.batch, 0, 0, s + 1, rows)
        srt = rows.sort().values
        for name in (("philox_order", "sorted") if s % 2 == 0 else ("sorted", "philox_order")):
            r = rows if name == "philox_order" else srt
            eng.partial_fit_rows(X, r)          # warm (same rows twice: timing only)
            ev[0].record()
            eng.partial_fit_rows(X, r)
            ev[1].record()
            torch.cuda.synchronize()
            t[name].append(ev[0].elapsed_time(ev[1]))
    out = {k: round(statistics.median(v), 4) for k, v in t.items()}
    out["speedup_sorted"] = round(out["philox_order"] / out["sorted"], 4)
    out.update(shard_rows=args.shard_rows, batch=args.batch, d=args.d, k=args.k)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
