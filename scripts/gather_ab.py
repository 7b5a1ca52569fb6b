"""Where does the gathered assign's extra time go (cfg5 shape)?  One resident shard, one
16.8M-row batch, timed in one process, interleaved: the contiguous batch (no index list),
the same rows through an index list in order (arange: the index round trip only), and
Philox-sampled rows (index round trip + random rows)."""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from mikmeans import ops
from mikmeans.data import blobs as B
from mikmeans.ops import native


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shard-rows", type=int, default=60_000_000)
    ap.add_argument("--batch", type=int, default=1 << 24)
    ap.add_argument("--d", type=int, default=256)
    ap.add_argument("--k", type=int, default=512)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    C = native.require()
    X = B.make_blobs(a.shard_rows, a.d, a.k, seed=1, dtype=torch.bfloat16, device="cuda")
    cen = X[: a.k].float()
    pack = ops.pack_centers(cen, a.d, torch.bfloat16, "cuda")
    b = a.batch
    rnd = torch.empty(b, dtype=torch.int64, device="cuda")
    C.sample_index(a.shard_rows, b, 0, 0, 1, rnd)
    arms = {
        "contiguous": (X[:b], None, False),
        "arange_rows": (X, torch.arange(b, dtype=torch.int64, device="cuda"), False),
        "sorted_rows": (X, rnd.sort().values, False),
        "philox_rows": (X, rnd, False),
        "philox_rows_inertia": (X, rnd, True),      # the mini-batch step's call: batch inertia slots
        "contiguous_inertia": (X[:b], None, True),
    }
    slots = torch.zeros(C.NSLOT * C.SLOT_STRIDE, dtype=torch.float64, device="cuda")
    lab = torch.empty(b, dtype=torch.int32, device="cuda")
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    t = {k: [] for k in arms}
    for rd in range(a.rounds):
        order = list(arms) if rd % 2 == 0 else list(arms)[::-1]
        for name in order:
            Xa, rows, sl = arms[name]
            sarg = slots if sl else None
            pack.assign(Xa, None, lab, None, sarg, False, rows=rows)
            ev[0].record()
            for _ in range(a.reps):
                pack.assign(Xa, None, lab, None, sarg, False, rows=rows)
            ev[1].record()
            torch.cuda.synchronize()
            t[name].append(ev[0].elapsed_time(ev[1]) / a.reps)
    base = statistics.median(t["contiguous"])
    print(json.dumps({k: {"median_ms": round(statistics.median(v), 4),
                          "vs_contiguous": round(statistics.median(v) / base, 4)} for k, v in t.items()}), flush=True)


if __name__ == "__main__":
    main()
