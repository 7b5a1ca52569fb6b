"""Local multi-process launcher (one process per rank) for CPU/gloo runs and tests.

GPU jobs run one rank per GPU (RCCL): ``launch_self`` starts a script as an N-rank
``torch.distributed.run`` child with optional fresh-process restarts (bench.py and
``mikmeans launch`` use it); ``spawn_local`` runs a function on ``world`` CPU ranks on
127.0.0.1 with the gloo backend so the exact same distributed code paths (sharding,
packed all-reduce, k-means++ owner selection, checkpoint broadcast, room replication)
run without a GPU.
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys
import tempfile
import traceback

import torch
import torch.multiprocessing as mp


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _to_cpu(obj):
    """Results leave the rank as host tensors (the parent may not share the rank's GPU)."""
    if torch.is_tensor(obj):
        return obj.detach().cpu()
    if isinstance(obj, dict):
        return {k: _to_cpu(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_to_cpu(v) for v in obj)
    return obj


def _worker(rank, world, port, fn, args, outdir, device="cpu"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from .comm import Comm, set_comm

    comm = Comm.from_env(device, staged=device == "cuda")
    set_comm(comm)
    try:
        res = _to_cpu(fn(comm, *args))
        if device == "cuda":
            torch.cuda.synchronize()
        torch.save({"ok": True, "res": res}, os.path.join(outdir, f"r{rank}.pt"))
    except BaseException:  # report, never hang the others silently
        torch.save({"ok": False, "err": traceback.format_exc()}, os.path.join(outdir, f"r{rank}.pt"))
        raise
    finally:
        comm.close()


def torchrun_cmd(nproc: int, script_argv: list[str], port: int | None = None) -> list[str]:
    """``python -m torch.distributed.run`` for ``nproc`` local ranks on 127.0.0.1."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
            "--master-addr", "127.0.0.1", "--master-port", str(port or free_port()), *script_argv]


def launch_self(nproc: int, script_argv: list[str], max_restarts: int = 0, env: dict | None = None,
                dmabuf_ipc: bool = False) -> int:
    """Start ``script_argv`` (a script path plus its arguments) as an ``nproc``-rank job and
    return its exit code -- the MI355X analogue of the reference meshing every tab on page
    load (app.mjs:70-118, called at :583).

    The caller must not have initialised the GPU: the job runs as a CHILD process (never an
    exec of this one).  A failed job is relaunched up to ``max_restarts`` times as a fresh
    process tree; a script that checkpoints resumes from its last checkpoint then
    (``mikmeans fit --resume auto``), so a lost rank costs at most the work since it.
    """
    env = dict(os.environ if env is None else env)
    if dmabuf_ipc or os.environ.get("MIKMEANS_DMABUF_IPC", "0") not in ("", "0"):
        # Opt-in: hosts whose amdgpu driver only supports dmabuf IPC need the HSA runtime's
        # legacy IPC mode off, or RCCL's peer mappings fail with "hipIpcGetMemHandle: invalid
        # argument".  Other hosts keep whatever the caller's environment says.
        env["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    rc = 1
    for attempt in range(max_restarts + 1):
        cmd = torchrun_cmd(nproc, script_argv)
        if attempt:
            print(f"[mikmeans launch] job failed (rc={rc}); restart {attempt}/{max_restarts}", file=sys.stderr,
                  flush=True)
        rc = subprocess.call(cmd, env=env)
        if rc == 0:
            break
    return rc


def spawn_local(fn, world: int, *args, timeout: float = 300.0, device: str = "cpu"):
    """Run ``fn(comm, *args)`` on ``world`` gloo ranks; return the list of per-rank results.

    ``device="cuda"``: GPU ranks over a host-staged gloo group (:class:`~.comm.Comm`
    ``staged``), rank r on GPU ``r % device_count`` -- on a one-GPU box all ranks share it
    and run the real HIP kernels."""
    port = free_port()
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, port, fn, args, d, device), nprocs=world, join=True)
        out = []
        for r in range(world):
            rec = torch.load(os.path.join(d, f"r{r}.pt"), weights_only=True)
            if not rec["ok"]:
                raise RuntimeError(f"rank {r} failed:\n{rec['err']}")
            out.append(rec["res"])
        return out
