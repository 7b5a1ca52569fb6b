#!/usr/bin/env python3
"""Where the one-ring-per-CU assign's waves spend their cycles (csrc/assign_ring.hip, with the
timeline hook armed: per-wave s_memtime counters).  Prints the mean share of each wave's life
spent spinning for a position, in prologues, in epilogues and in the touch / publish work.

usage: python scripts/ring_timeline.py --n 20000000 [--arm assign_ring=1]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from mikmeans.data.blobs import blob_centers, make_blobs  # noqa: E402
from mikmeans.models.init import init_random  # noqa: E402
from mikmeans.models.lloyd import LloydEngine  # noqa: E402
from mikmeans.ops import native  # noqa: E402
from mikmeans.parallel import Comm  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=20_000_000)
    ap.add_argument("--k", type=int, default=1024)
    ap.add_argument("--arm", default="assign_ring=1")
    a = ap.parse_args()
    dev = torch.device("cuda")
    comm = Comm.local(dev)
    X = make_blobs(a.n, 128, a.k, seed=0, dtype=torch.bfloat16, device=dev,
                   centers=blob_centers(a.k, 128, 10.0, 0, device=dev))
    eng = LloydEngine(X, a.k, comm=comm).set_centers(init_random(X, 128, a.k, a.n, 0, comm, 0))
    for _ in range(2):
        eng.step()
    for kv in filter(None, a.arm.split(",")):
        k, v = kv.split("=")
        native.set_variant(k, int(v))
    C = native.require()
    buf = torch.zeros(4096 * 8, dtype=torch.int64, device=dev)
    C.set_assign_timeline(buf)
    lab = torch.empty(a.n, dtype=torch.int32, device=dev)
    for _ in range(3):
        eng.pk.assign(eng.X, eng.xn, lab)
    torch.cuda.synchronize()
    C.set_assign_timeline(None)
    t = buf.view(-1, 8).double().cpu()
    live = t[:, 0] > 0
    t = t[live]
    tot = t[:, 0]
    names = ["total", "ready_spin", "prologue", "epilogue", "touch_publish", "blocks", "sleeping_polls", "startup"]
    out = {"waves": int(live.sum()), "fault": C.assign_ring_fault(),
           "mean_total_cycles": float(tot.mean())}
    for i, nm in enumerate(names[1:], 1):
        if nm in ("blocks", "sleeping_polls"):
            out[nm + "_mean"] = float(t[:, i].mean())
        else:
            out[nm + "_share"] = round(float((t[:, i] / tot).mean()), 4)
    out["compute_share"] = round(1.0 - sum(out[n + "_share"] for n in ("ready_spin", "prologue", "epilogue",
                                                                         "touch_publish", "startup")), 4)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
