"""Full-E-step Lloyd against the bounded (Hamerly) E-step, from the same start.

Per iteration: wall time of ``step()`` (CUDA events), rows the bounded E-step re-assigned,
label agreement with the full-E-step engine; at the end the centre difference and both
engines' total time.  Blob data, centres = ``K`` random rows (the bench's init).

run (GPU): python scripts/hamerly_ab.py [--n N --d D --k K --dtype bf16|f32 --iters I]
"""
import argparse
import json
import sys

import torch

sys.path.insert(0, ".")
from mikmeans.data.blobs import make_blobs  # noqa: E402
from mikmeans.models.lloyd import LloydEngine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=20_000_000)
    ap.add_argument("--d", type=int, default=128)
    ap.add_argument("--k", type=int, default=1024)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--blobs", type=int, default=0, help="blob count (default: K)")
    ap.add_argument("--init", default="random", choices=["random", "k-means||"],
                    help="random rows (the bench's start) or k-means|| seeding")
    a = ap.parse_args()
    dt = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    X = make_blobs(a.n, a.d, a.blobs or a.k, seed=7, dtype=dt, device="cuda")
    g = torch.Generator(device="cpu").manual_seed(1)
    if a.init == "random":
        C0 = X[torch.randint(0, a.n, (a.k,), generator=g).cuda()].float()
    else:
        from mikmeans.models.init import init_kmeans_parallel
        from mikmeans.parallel import Comm

        C0 = init_kmeans_parallel(X, a.d, a.k, a.n, 0, Comm.local(X.device), seed=1)
    ea = LloydEngine(X, a.k, incremental=True).set_centers(C0)
    eb = LloydEngine(X, a.k, incremental=True, bounded=True).set_centers(C0)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    rows = []
    tot = [0.0, 0.0]
    for it in range(a.iters):
        ev[0].record()
        ea.step()
        ev[1].record()
        eb.step()
        ev[2].record()
        torch.cuda.synchronize()
        ta, tb = ev[0].elapsed_time(ev[1]), ev[1].elapsed_time(ev[2])
        tot[0] += ta
        tot[1] += tb
        agree = float((ea.labels == eb.labels).float().mean())
        rows.append({"it": it, "full_ms": round(ta, 3), "bounded_ms": round(tb, 3),
                     "reassigned": eb.reassigned, "frac": round(eb.reassigned / a.n, 4),
                     "changed": ea.last_stats().n_changed, "agree": round(agree, 6)})
        print(json.dumps(rows[-1]), flush=True)
    dc = float((ea.centers - eb.centers).abs().max())
    print(json.dumps({"n": a.n, "d": a.d, "k": a.k, "dtype": a.dtype, "iters": a.iters, "init": a.init,
                      "full_total_ms": round(tot[0], 2), "bounded_total_ms": round(tot[1], 2),
                      "speedup": round(tot[0] / max(tot[1], 1e-9), 3), "max_centre_diff": dc}), flush=True)


if __name__ == "__main__":
    main()
