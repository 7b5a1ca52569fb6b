"""Local multi-process launcher (one process per rank) for CPU/gloo runs and tests.

GPU jobs use ``torchrun --nproc-per-node N`` (one rank per GPU, RCCL); this helper
spawns ``world`` CPU ranks on 127.0.0.1 with the gloo backend so the exact same
distributed code paths (sharding, packed all-reduce, k-means++ owner selection,
checkpoint broadcast, room replication) run without a GPU.
"""
from __future__ import annotations

import os
import socket
import tempfile
import traceback

import torch
import torch.multiprocessing as mp


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, fn, args, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from .comm import Comm, set_comm

    comm = Comm.from_env("cpu")
    set_comm(comm)
    try:
        res = fn(comm, *args)
        torch.save({"ok": True, "res": res}, os.path.join(outdir, f"r{rank}.pt"))
    except BaseException:  # report, never hang the others silently
        torch.save({"ok": False, "err": traceback.format_exc()}, os.path.join(outdir, f"r{rank}.pt"))
        raise
    finally:
        comm.close()


def spawn_local(fn, world: int, *args, timeout: float = 300.0):
    """Run ``fn(comm, *args)`` on ``world`` gloo ranks; return the list of per-rank results."""
    port = free_port()
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, port, fn, args, d), nprocs=world, join=True)
        out = []
        for r in range(world):
            rec = torch.load(os.path.join(d, f"r{r}.pt"), weights_only=True)
            if not rec["ok"]:
                raise RuntimeError(f"rank {r} failed:\n{rec['err']}")
            out.append(rec["res"])
        return out
