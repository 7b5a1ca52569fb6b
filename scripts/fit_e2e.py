"""Cost of the host convergence checks in LloydEngine.run at the BASELINE shapes.

``bench.py`` times bare engine steps; ``KMeans.fit`` drives ``LloydEngine.run``, which
reads each iteration's statistics on the host (convergence test, metrics, checkpoints).
This times ``run(iters, tol=-inf)`` on one engine -- no setup inside the clock -- with a
check every iteration against no checks, eager and graph-replayed.  Median of rounds.
(A pipelined variant -- iteration i+1 enqueued before iteration i's statistics are read,
rolled back on convergence -- measured no faster and was not kept:
profiles/r2_26_check_overhead_ab.md.)

run (GPU): python scripts/fit_e2e.py [cfg2 cfg4 cfg3]
"""
import json
import math
import statistics
import sys
import time

import torch

sys.path.insert(0, ".")
from mikmeans.data.blobs import make_blobs  # noqa: E402
from mikmeans.models.lloyd import LloydEngine  # noqa: E402

SHAPES = {
    "cfg2": (1_000_000, 128, 256, torch.float32, 100),
    "cfg4": (10_000_000, 64, 4096, torch.bfloat16, 40),
    "cfg3": (100_000_000, 128, 1024, torch.bfloat16, 10),
}


def timed_run(eng, C0, iters, check_every):
    eng.set_centers(C0)
    eng.reset_labels()
    it0 = eng.iteration
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n, _, _ = eng.run(iters, -math.inf, check_every=check_every, callback=lambda st: None)
    torch.cuda.synchronize()
    # (a run with checks stops early once no label changes: per executed iteration)
    return (time.perf_counter() - t0) * 1e3 / max(n - it0, 1)


def main():
    names = sys.argv[1:] or ["cfg2", "cfg4"]
    out = {}
    for name in names:
        n, d, k, dt, iters = SHAPES[name]
        X = make_blobs(n, d, k, seed=0, dtype=dt, device="cuda")
        C0 = X[torch.randperm(n, device="cuda")[:k]].float()
        for graph in (False, True):
            eng = LloydEngine(X, k, incremental=False).set_centers(C0)
            if graph:
                eng.capture()
            variants = {"no_checks": 0, "checks": 1}
            ts = {v: [] for v in variants}
            timed_run(eng, C0, 3, 1)                            # warm-up
            for _ in range(5):
                for v, ce in variants.items():
                    ts[v].append(timed_run(eng, C0, iters, ce))
            out[f"{name}_graph={int(graph)}"] = {v: round(statistics.median(t), 4) for v, t in ts.items()}
            print(json.dumps(out), flush=True)
            del eng
        del X
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
