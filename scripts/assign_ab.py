#!/usr/bin/env python3
"""A/B of assign-kernel variants (mikmeans.ops.native.set_variant) in one process, interleaved
rounds, on the bench's blob data a few Lloyd iterations in.

usage: assign_ab.py [--n N] [--d D] [--k K] [--dtype bf16|f32] [--rounds R] [--reps M]
                    --arms "assign_geom=0;assign_geom=1;assign_geom=2"
Prints one JSON line per shape: median / min ms per arm, TF/s, whether every arm's labels
equal the first arm's (bitwise), and -- from the GFX clock sampled during each arm's timed
launches (mikmeans/utils/telemetry.py, amdsmi) -- the mean clock and the cycles per MFMA per
SIMD (16 for a v_mfma_f32_16x16x32_bf16 issued back to back): a clock-normalised cost, so
an A/B across boxes or power states compares work per cycle, not wall time.
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from mikmeans.data.blobs import blob_centers, make_blobs  # noqa: E402
from mikmeans.models.init import init_random  # noqa: E402
from mikmeans.models.lloyd import LloydEngine  # noqa: E402
from mikmeans.ops import native  # noqa: E402
from mikmeans.parallel import Comm  # noqa: E402


def parse_arm(spec: str) -> dict:
    out = {}
    for kv in filter(None, spec.split(",")):
        if kv.strip() in ("default", "-"):
            continue
        k, v = kv.split("=")
        out[k.strip()] = int(v)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=20_000_000)
    ap.add_argument("--d", type=int, default=128)
    ap.add_argument("--k", type=int, default=1024)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--arms", default="assign_early=0;assign_early=1")
    ap.add_argument("--gather", type=int, default=0,
                    help="> 0: time the gathered assign of this many random rows (the mini-batch "
                         "resident path: X[rows] read in place, norms from the fragments)")
    a = ap.parse_args()
    dt = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    dev = torch.device("cuda")
    comm = Comm.local(dev)
    X = make_blobs(a.n, a.d, a.k, seed=0, dtype=dt, device=dev, centers=blob_centers(a.k, a.d, 10.0, 0, device=dev))
    eng = LloydEngine(X, a.k, comm=comm).set_centers(init_random(X, a.d, a.k, a.n, 0, comm, 0))
    for _ in range(3 if not a.gather else 1):
        eng.step()
    if a.gather:
        g = torch.Generator(device=dev).manual_seed(5)
        rows = torch.randint(0, a.n, (a.gather,), device=dev, generator=g)
        glab = torch.empty(a.gather, dtype=torch.int32, device=dev)

        def call():
            eng.pk.assign(eng.X, None, glab, None, eng.slots, False, rows=rows)
    else:
        def call():
            eng.pk.assign(eng.X, eng.xn, eng.labels, eng.mind, eng.slots, True)
    arms = [parse_arm(s) for s in a.arms.split(";")]
    names = [s or "default" for s in a.arms.split(";")]
    labels = {}
    times = {n: [] for n in names}
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]

    from mikmeans.utils.telemetry import ClockSampler

    clocks = {n: [] for n in names}

    def run(arm, name):
        old = {k: native.get_variant(k) for k in arm}
        for k, v in arm.items():
            native.set_variant(k, v)
        try:
            call()   # warm / attributes
            torch.cuda.synchronize()
            with ClockSampler(0, period_s=0.01) as cs:
                ev[0].record()
                for _ in range(a.reps):
                    call()
                ev[1].record()
                torch.cuda.synchronize()
            sm = cs.summary()
            if sm and sm.get("clock_mhz"):
                clocks[name].append(sm["clock_mhz"])
            return ev[0].elapsed_time(ev[1]) / a.reps, (glab if a.gather else eng.labels).clone()
        finally:
            for k, v in old.items():
                native.set_variant(k, v)

    for rd in range(a.rounds):
        order = list(zip(names, arms)) if rd % 2 == 0 else list(zip(names, arms))[::-1]
        for n, arm in order:
            t, lab = run(arm, n)
            times[n].append(t)
            labels.setdefault(n, lab)
    ref = labels[names[0]]
    res = {"n": a.n, "d": a.d, "k": a.k, "dtype": a.dtype, "rounds": a.rounds, "reps": a.reps,
           "gathered_rows": a.gather}
    m = a.gather or a.n
    kpad = eng.pk.Kpad
    # MFMA instructions per SIMD: 16-point blocks x 16-centre tiles x K-steps of 32 (bf16) / 4 x 4 (f32)
    ksteps = eng.pk.dpad // 32 if dt == torch.bfloat16 else eng.pk.dpad // 4
    mfma_per_simd = (m / 16) * (kpad / 16) * ksteps / 1024
    for n in names:
        med = statistics.median(times[n])
        res[n] = {"median_ms": round(med, 4), "min_ms": round(min(times[n]), 4),
                  "tflops": round(2.0 * m * a.k * a.d / (med * 1e-3) / 1e12, 1),
                  "labels_equal": bool(torch.equal(labels[n], ref))}
        if clocks[n]:
            clk = statistics.fmean(clocks[n])
            res[n]["clock_mhz"] = round(clk, 1)
            res[n]["cycles_per_mfma"] = round(med * 1e-3 * clk * 1e6 / mfma_per_simd, 2)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
