#!/usr/bin/env python3
"""A/B of the previous-label hint in the 16x16 assign kernel (one process, interleaved).

    python scripts/ab_hint.py --n 20000000 --d 128 --k 1024 --rounds 7

Times the E-step on the same centres (a) without the hint, (b) hinted with the exact
current labels (steady state: no tile takes the exact path), (c) hinted with the labels
of the previous Lloyd iteration (what a fit sees), (d) hinted with random labels.
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
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=6, help="Lloyd iterations before timing")
    a = ap.parse_args()

    from mikmeans.data.blobs import make_blobs
    from mikmeans.models.lloyd import LloydEngine

    X = make_blobs(a.n, a.d, a.k, seed=0, dtype=torch.bfloat16, device="cuda")
    eng = LloydEngine(X, a.k).set_centers(X[: a.k].float())
    for _ in range(a.iters):
        eng.step()
    prev_labels = eng.labels.clone()
    eng.step()                       # centres now one step past prev_labels
    torch.cuda.synchronize()
    exact = torch.empty_like(eng.labels)
    exact.fill_(-1)
    eng.pk.assign(eng.X, eng.xn, exact)          # exact labels for the current centres
    g = torch.Generator(device="cuda").manual_seed(1)
    rnd = torch.randint(0, a.k, eng.labels.shape, device="cuda", generator=g, dtype=torch.int32)
    cases = {"nohint": (exact, False), "hint_exact": (exact, True), "hint_prev": (prev_labels, True),
             "hint_random": (rnd, True)}
    res = {c: [] for c in cases}
    lab = torch.empty_like(exact)
    ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
    for _ in range(a.rounds):
        for c, (src, hint) in cases.items():
            lab.copy_(src)
            e0, e1 = ev(), ev()
            e0.record()
            eng.pk.assign(eng.X, eng.xn, lab, None, eng.slots, True, hint=hint)
            e1.record()
            torch.cuda.synchronize()
            res[c].append(e0.elapsed_time(e1))
    ab = hasattr(eng._C, "set_assign16_cfg")
    try:   # A/B build only (MIKMEANS_AB=1): fast-path-only timing and exact-path tile counts
        eng._C.set_assign16_cfg(60)
        t = []
        for _ in range(a.rounds):
            lab.copy_(exact)
            e0, e1 = ev(), ev()
            e0.record()
            eng.pk.assign(eng.X, eng.xn, lab, None, eng.slots, True, hint=True)
            e1.record()
            torch.cuda.synchronize()
            t.append(e0.elapsed_time(e1))
        res["hint_no_epilogue"] = t
        eng._C.set_assign16_cfg(62)
        t = []
        for _ in range(a.rounds):
            lab.copy_(exact)
            e0, e1 = ev(), ev()
            e0.record()
            eng.pk.assign(eng.X, eng.xn, lab, None, eng.slots, True, hint=True)
            e1.record()
            torch.cuda.synchronize()
            t.append(e0.elapsed_time(e1))
        res["hint_no_prologue"] = t
        eng._C.set_assign16_cfg(61)
        counts = {}
        for c in ("hint_exact", "hint_prev", "hint_random"):
            lab.copy_(cases[c][0])
            eng.slots.zero_()
            eng.pk.assign(eng.X, eng.xn, lab, None, eng.slots, True, hint=True)
            torch.cuda.synchronize()
            counts[c] = float(eng.slots.view(-1)[2])
        eng.slots.zero_()
        waves = (a.n + 63) // 64
        tiles = (a.k + 15) // 16
        res_counts = {c: {"exact_path_tiles": v, "fraction_of_wave_tiles": v / (waves * tiles)}
                      for c, v in counts.items()}
    except RuntimeError as e:
        res_counts = {"skipped": str(e)[:200]}
    finally:
        if ab:
            eng._C.set_assign16_cfg(0)
    changed = int((prev_labels != exact).sum())
    flop = 2.0 * a.n * a.k * a.d
    out = {"n": a.n, "d": a.d, "k": a.k, "prev_vs_exact_changed": changed, "exact_path": res_counts}
    for c, v in res.items():
        out[c] = {"median_ms": statistics.median(v), "min_ms": min(v),
                  "tflops": flop / (statistics.median(v) * 1e-3) / 1e12}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
