"""Probe: does splitting the CUs between the assign and the M-step pay at the headline?

The assign kernel is power-bound (profiles/r2_08_assign_clock_study.md) and the M-step is
HBM-bound; launched together on two unmasked streams they do not overlap
(profiles/r1_16_overlap_ab.json).  Here the segmented step (LloydEngine(segments=S):
segment s scattered on a side stream while segment s+1 is assigned) runs with the two
streams on DISJOINT CU sets (hipExtStreamCreateWithCUMask).  The side set is spread so it
takes the same number of CUs from every XCD whether the runtime numbers mask bits per XCD
or round-robin over XCDs.

run (GPU): python scripts/cumask_probe.py [--n 100000000] [--steps 5]
"""
import argparse
import ctypes
import json
import sys

import torch

sys.path.insert(0, ".")
from mikmeans.data.blobs import blob_centers, make_blobs  # noqa: E402
from mikmeans.models.init import init_random  # noqa: E402
from mikmeans.models.lloyd import LloydEngine  # noqa: E402
from mikmeans.parallel import Comm  # noqa: E402


def _hip():
    for line in open("/proc/self/maps"):
        if "libamdhip64.so" in line:
            return ctypes.CDLL(line.split()[-1])
    return ctypes.CDLL("libamdhip64.so")


def side_set(n_cu: int, per_xcd: int) -> set:
    """per_xcd CUs of each of the 8 XCDs under both plausible bit numberings."""
    per = n_cu // 8
    out = set()
    for a in range(8):
        for b in range(per_xcd):  # 4 rows of 8 per residue class, residues rotating with a
            out.add(a * per + 8 * (b % 4) + (a + b // 4) % 8)
    assert len(out) == 8 * per_xcd
    return out


def masked_stream(hip, n_cu: int, cus: set):
    words = (ctypes.c_uint32 * ((n_cu + 31) // 32))()
    for c in cus:
        words[c // 32] |= 1 << (c % 32)
    s = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), len(words), words)
    assert rc == 0, rc
    return torch.cuda.ExternalStream(s.value)


def timed(fn, stream, steps, warm=2):
    with torch.cuda.stream(stream):
        for _ in range(warm):
            fn()
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record(stream)
        for _ in range(steps):
            fn()
        b.record(stream)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100_000_000)
    ap.add_argument("--steps", type=int, default=5)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    hip = _hip()
    n_cu = torch.cuda.get_device_properties(dev).multi_processor_count
    N, D, K = args.n, 128, 1024
    cen = blob_centers(K, D, 10.0, 0, device=dev)
    X = make_blobs(N, D, K, seed=0, dtype=torch.bfloat16, device=dev, centers=cen)
    C0 = init_random(X, D, K, N, 0, Comm.local(dev), 0)
    res = {"n_cu": n_cu}
    allc = set(range(n_cu))

    base = LloydEngine(X, K).set_centers(C0)
    res["serial_default"] = timed(base.step, torch.cuda.current_stream(), args.steps)
    for px in (4, 8):
        side = side_set(n_cu, px)
        ms = masked_stream(hip, n_cu, allc - side)
        res[f"serial_main{n_cu - len(side)}"] = timed(base.step, ms, args.steps)
    # M-step alone on the side sets (its HBM rate on few CUs)
    for px in (4, 8, 16):
        side = side_set(n_cu, px)
        ss = masked_stream(hip, n_cu, side)
        C = base._C
        res[f"update_only_side{len(side)}"] = timed(
            lambda: C.update(base.X, base.labels, base.K, base.slab, base.cnt_slab, base.n_chunks,
                             None, base.col_exp, base.cnt_exp, False), ss, args.steps)
    res["assign_only_default"] = timed(
        lambda: base.pk.assign(base.X, base.xn, base.labels, base.mind, base.slots, True),
        torch.cuda.current_stream(), args.steps)
    del base
    torch.cuda.empty_cache()
    print(json.dumps(res), flush=True)
    for segs in (8, 16):
        for px in (0, 4, 8):
            eng = LloydEngine(X, K, segments=segs, overlap_sw=0 if px else 8).set_centers(C0)
            if px:
                side = side_set(n_cu, px)
                eng.side = masked_stream(hip, n_cu, side)
                main = masked_stream(hip, n_cu, allc - side)
            else:
                main = torch.cuda.current_stream()
            res[f"seg{segs}_side{8 * px}"] = timed(eng.step, main, args.steps)
            print(json.dumps(res), flush=True)
            del eng
            torch.cuda.empty_cache()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
