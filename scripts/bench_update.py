#!/usr/bin/env python3
"""Time the M-step scatter-add kernel (csrc/update.hip) alone under several label patterns.

Patterns: ``random`` (uniform labels, the Lloyd case), ``mod`` (label = i mod K: distinct
labels within a wave), ``sorted`` (runs of N/K equal labels), ``one`` (all label 0:
same-address atomics + a flush every period).  Prints ms and effective read GB/s.
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
    ap.add_argument("--dtype", default="bfloat16")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--patterns", default="random,mod,sorted,one")
    ap.add_argument("--nts", default="0", help="threads/WG variants to A/B (0 = default)")
    a = ap.parse_args()
    from mikmeans.ops import fixed_exps, native

    C = native.require()
    dt = torch.bfloat16 if a.dtype == "bfloat16" else torch.float32
    X = torch.randn(a.n, a.d, device="cuda", dtype=dt)
    nch = C.update_n_chunks(native.dtype_code(dt), a.k, a.d, a.n)
    slab = torch.empty(nch * a.k * a.d, dtype=torch.int64, device="cuda")
    cnt = torch.empty(nch * a.k, dtype=torch.int64, device="cuda")
    col_exp, _ = fixed_exps(X)
    i = torch.arange(a.n, device="cuda")
    pats = {
        "random": lambda: torch.randint(0, a.k, (a.n,), device="cuda", dtype=torch.int32),
        "mod": lambda: (i % a.k).to(torch.int32),
        "sorted": lambda: (i * a.k // a.n).to(torch.int32),
        "one": lambda: torch.zeros(a.n, dtype=torch.int32, device="cuda"),
    }
    out = {"n": a.n, "d": a.d, "k": a.k, "dtype": a.dtype, "n_chunks": nch,
           "slice_width": C.update_slice_width(native.dtype_code(dt), a.k, a.d)}
    for p in a.patterns.split(","):
        lab = pats[p]()
        ts = {nt: [] for nt in a.nts.split(",")}
        for nt in ts:
            C.set_update_nt(int(nt))
            C.update(X, lab, a.k, slab, cnt, nch, None, col_exp, 0, False)
        for _ in range(a.reps):
            for nt in ts:
                C.set_update_nt(int(nt))
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                C.update(X, lab, a.k, slab, cnt, nch, None, col_exp, 0, False)
                e1.record()
                torch.cuda.synchronize()
                ts[nt].append(e0.elapsed_time(e1))
        C.set_update_nt(0)
        for nt, v in ts.items():
            ms = statistics.median(v)
            key = p if nt == "0" else f"{p}_nt{nt}"
            out[key] = {"ms": round(ms, 4), "read_GBps": round(X.numel() * X.element_size() / ms / 1e6, 1)}
    # reference point: a plain streaming read of X (column sums in f32)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    X.sum(0, dtype=torch.float32)
    e0.record()
    X.sum(0, dtype=torch.float32)
    e1.record()
    torch.cuda.synchronize()
    out["torch_colsum_ms"] = round(e0.elapsed_time(e1), 4)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
