#!/usr/bin/env python3
"""Out-of-core Lloyd throughput: X in pinned host memory, streamed through the GPU.

    python scripts/bench_streaming.py --n 20000000 --d 128 --k 1024 --chunk 4194304

Reports seconds per Lloyd iteration, the host->device bytes per second it implies, and a
plain pinned H2D copy of the same bytes as the ceiling (PCIe), plus the device-resident
step time of the same shape for comparison.
"""
import argparse
import json
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=20_000_000)
    ap.add_argument("--d", type=int, default=128)
    ap.add_argument("--k", type=int, default=1024)
    ap.add_argument("--chunk", type=int, default=1 << 22)
    ap.add_argument("--iters", type=int, default=3)
    a = ap.parse_args()

    from mikmeans.data.blobs import make_blobs
    from mikmeans.models.lloyd import LloydEngine
    from mikmeans.models.streaming import StreamingLloydEngine

    dev = torch.device("cuda")
    Xd = make_blobs(a.n, a.d, a.k, seed=0, dtype=torch.bfloat16, device=dev)
    Xh = torch.empty(Xd.shape, dtype=Xd.dtype, pin_memory=True)
    Xh.copy_(Xd)
    C0 = Xd[: a.k].float()
    nbytes = Xh.numel() * Xh.element_size()
    # ceiling: one pinned H2D copy of the whole shard
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    Xd.copy_(Xh, non_blocking=True)
    torch.cuda.synchronize()
    h2d = time.perf_counter() - t0
    res = LloydEngine(Xd, a.k).set_centers(C0)
    res.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.iters):
        res.step()
    torch.cuda.synchronize()
    t_res = (time.perf_counter() - t0) / a.iters
    del res, Xd
    st = StreamingLloydEngine(Xh, a.k, chunk_rows=a.chunk, device=dev).set_centers(C0)
    st.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.iters):
        st.step()
    torch.cuda.synchronize()
    t_st = (time.perf_counter() - t0) / a.iters
    print(json.dumps({"n": a.n, "d": a.d, "k": a.k, "chunk_rows": a.chunk, "bytes": nbytes,
                      "streaming_s_per_iter": round(t_st, 4), "streaming_h2d_GBps": round(nbytes / t_st / 1e9, 1),
                      "pinned_h2d_copy_GBps": round(nbytes / h2d / 1e9, 1),
                      "resident_s_per_iter": round(t_res, 5),
                      "overlap_efficiency": round(max(h2d, t_res) / t_st, 3)}, indent=1))


if __name__ == "__main__":
    main()
