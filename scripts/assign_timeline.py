#!/usr/bin/env python3
"""Per-workgroup timeline of one assign launch (csrc/assign16.hip AssignArgs::timeline):
entry, chunk-loop start, epilogue start and exit in real-time ticks (10 ns) plus the CU each
workgroup ran on.  Prints the phase durations (prologue = entry -> loop, loop, epilogue) and
how the workgroups' starts spread in time -- whether co-resident workgroups load their rows
together.

usage: python scripts/assign_timeline.py --n 20000000 --d 128 --k 1024"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from mikmeans.data.blobs import blob_centers, make_blobs  # noqa: E402
from mikmeans.models.init import init_random  # noqa: E402
from mikmeans.models.lloyd import LloydEngine  # noqa: E402
from mikmeans.ops import native  # noqa: E402
from mikmeans.parallel import Comm  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=20_000_000)
    ap.add_argument("--d", type=int, default=128)
    ap.add_argument("--k", type=int, default=1024)
    ap.add_argument("--arm", default="", help="kernel switches, e.g. assign_early=0")
    a = ap.parse_args()
    dev = torch.device("cuda")
    comm = Comm.local(dev)
    X = make_blobs(a.n, a.d, a.k, seed=0, dtype=torch.bfloat16, device=dev,
                   centers=blob_centers(a.k, a.d, 10.0, 0, device=dev))
    eng = LloydEngine(X, a.k, comm=comm).set_centers(init_random(X, a.d, a.k, a.n, 0, comm, 0))
    for _ in range(2):
        eng.step()
    for kv in filter(None, a.arm.split(",")):
        k, v = kv.split("=")
        native.set_variant(k, int(v))
    C = native.require()
    cap = a.n // 16 + 1
    buf = torch.zeros(cap * 8, dtype=torch.int64, device=dev)
    eng.pk.assign(eng.X, eng.xn, eng.labels, eng.mind, eng.slots, True)   # warm
    C.set_assign_timeline(buf)
    eng.pk.assign(eng.X, eng.xn, eng.labels, eng.mind, eng.slots, True)
    torch.cuda.synchronize()
    C.set_assign_timeline(None)
    t = buf.view(-1, 8).cpu().numpy()
    t = t[t[:, 0] > 0]
    t0 = t[:, 0].min()
    ent, loop, epi, ext = (t[:, i] - t0 for i in range(4))
    hw = t[:, 4]
    cu = (hw >> 8) & 0xF
    sh = (hw >> 12) & 0x1
    se = (hw >> 13) & 0x7
    xcc = t[:, 5] & 0xF
    cu_id = ((xcc * 8 + se) * 2 + sh) * 16 + cu
    us = 0.01
    pro, lp, ep = (loop - ent) * us, (epi - loop) * us, (ext - epi) * us
    land = (t[:, 6] - t0 - ent) * us       # entry -> the prologue's loads landed
    out_land = {"median": float(np.median(land)), "p90": float(np.percentile(land, 90))}
    frag = (t[:, 7] - t0 - ent) * us
    out_frag = {"median": float(np.median(frag)), "p90": float(np.percentile(frag, 90))}
    out = {"n": a.n, "d": a.d, "k": a.k, "arm": a.arm, "workgroups": int(len(t)),
           "kernel_us": float((ext.max()) * us),
           "prologue_us": {"median": float(np.median(pro)), "p90": float(np.percentile(pro, 90))},
           "loads_landed_us": out_land,
           "fragments_landed_or_issued_us": out_frag,   # (early prologue: issued)
           "loop_us": {"median": float(np.median(lp)), "p90": float(np.percentile(lp, 90))},
           "epilogue_us": {"median": float(np.median(ep)), "p90": float(np.percentile(ep, 90))},
           "distinct_cus": int(len(np.unique(cu_id)))}
    # first resident wave: the earliest-starting workgroup of each CU and the starts of the
    # others sharing that CU while it runs
    order = np.argsort(ent)
    first = order[: min(len(order), 1024)]
    out["first_wave_start_spread_us"] = float((ent[first].max() - ent[first].min()) * us)
    # the first resident wave runs with idle neighbours: its prologue is the unloaded latency
    out["first_wave_loads_landed_us"] = float(np.median(land[first]))
    out["first_wave_prologue_us"] = float(np.median(pro[first]))
    late = order[len(order) // 2:]
    out["steady_loads_landed_us"] = float(np.median(land[late]))
    # how aligned are co-resident workgroups: for each CU, the gaps between consecutive starts
    gaps = []
    for c in np.unique(cu_id):
        s = np.sort(ent[cu_id == c])
        if len(s) > 1:
            gaps.append(np.diff(s) * us)
    g = np.concatenate(gaps) if gaps else np.zeros(1)
    out["per_cu_start_gap_us"] = {"p10": float(np.percentile(g, 10)), "median": float(np.median(g)),
                                  "p90": float(np.percentile(g, 90))}
    # fraction of the kernel during which a workgroup is in its prologue, summed over workgroups
    out["prologue_share"] = float(pro.sum() / (pro + lp + ep).sum())
    print(json.dumps(out))


if __name__ == "__main__":
    main()
