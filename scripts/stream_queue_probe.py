#!/usr/bin/env python3
"""Which hardware queue does each HIP stream land on, and do two streams overlap?

Creates the bench's one-rank RCCL group (as bench.py does), then side streams made three ways
-- torch.cuda.Stream(), a high-priority torch stream, and one created before the group --
and times a blob-generator launch on a side stream against an M-step-shaped launch on the
default stream: alone, and both at once.  Run under ``rocprofv3 --kernel-trace`` to read the
Queue_Id of every dispatch.

usage: stream_queue_probe.py [--n 16777216] [--d 256]"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 24)
    ap.add_argument("--d", type=int, default=256)
    ap.add_argument("--k", type=int, default=512)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    early = torch.cuda.Stream(dev)                       # before any group
    os.environ.setdefault("MIKMEANS_FORCE_PG", "1")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    for k, v in (("RANK", "0"), ("LOCAL_RANK", "0"), ("WORLD_SIZE", "1")):
        os.environ.setdefault(k, v)
    from mikmeans.data.blobs import blob_centers, make_blobs
    from mikmeans.ops import cluster_sums
    from mikmeans.parallel import Comm

    comm = Comm.from_env("cuda")
    late = torch.cuda.Stream(dev)
    high = torch.cuda.Stream(dev, priority=-1)
    C = blob_centers(a.k, a.d, 10.0, 0, device=dev)
    X = make_blobs(a.n, a.d, a.k, seed=0, dtype=torch.bfloat16, device=dev, centers=C)
    Y = torch.empty_like(X)
    lab = torch.randint(0, a.k, (a.n,), device=dev, dtype=torch.int32)
    comm.allreduce_(torch.ones(4, device=dev))        # (RCCL's own streams exist from here)

    def gen(s):
        with torch.cuda.stream(s):
            make_blobs(a.n, a.d, a.k, seed=1, dtype=torch.bfloat16, device=dev, centers=C, out=Y)

    def mstep():
        cluster_sums(X, lab, a.k)

    def timed(fn, reps=5):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / reps * 1e3

    res = {"mstep_alone_ms": timed(mstep)}
    for name, s in (("early", early), ("late", late), ("high", high)):
        res[f"gen_alone_{name}_ms"] = timed(lambda s=s: gen(s))

        def both(s=s):
            ev = torch.cuda.Event()
            ev.record()
            s.wait_event(ev)
            gen(s)
            mstep()
            torch.cuda.current_stream().wait_stream(s)
        res[f"both_{name}_ms"] = timed(both)
    print(json.dumps({k: round(v, 3) for k, v in res.items()}), flush=True)
    comm.close()


if __name__ == "__main__":
    main()
