"""Checkpoint / resume.

Lloyd state is tiny -- centroids ``[K, D]`` f32, the iteration counter, the
config and the metric history -- so a checkpoint is one safetensors file plus a
JSON sidecar and the flat-float centroid JSON.  Only rank 0 writes; on load,
rank 0 reads and broadcasts (the analogue of the reference's full-state sync
``U:encodeStateAsUpdate``, app.mjs:96), so a job can resume with a different
world size (points are re-sharded, centroids are replicated).

Loading never executes code from the file: safetensors + JSON only.  The
reference's manual Export/Import (app.mjs:263-282) is :mod:`mikmeans.models.room`.
"""
from __future__ import annotations

import json
import os
from pathlib import Path

import torch
from safetensors.torch import load_file, save_file

from .jsjson import centroids_to_json

CKPT_TENSORS = "centroids.safetensors"
CKPT_META = "state.json"
CKPT_FLAT = "centroids.json"


def save_checkpoint(path, centers: torch.Tensor, iteration: int, config=None, *, history=None,
                    comm=None, extra: dict | None = None) -> Path:
    path = Path(path)
    rank = comm.rank if comm is not None else 0
    if rank == 0:
        path.mkdir(parents=True, exist_ok=True)
        c = centers.detach().to("cpu", torch.float32).contiguous()
        tmp = path / (CKPT_TENSORS + ".tmp")
        save_file({"centers": c}, str(tmp))
        os.replace(tmp, path / CKPT_TENSORS)
        meta = {
            "format": "mikmeans-checkpoint-v1",
            "iteration": int(iteration),
            "n_clusters": int(c.shape[0]),
            "n_features": int(c.shape[1]),
            "config": config.to_dict() if hasattr(config, "to_dict") else (config or {}),
            "history": history or [],
            "world_size": comm.world if comm is not None else 1,
        }
        if extra:
            meta.update(extra)
        tmpm = path / (CKPT_META + ".tmp")
        tmpm.write_text(json.dumps(meta, default=_jsonable))
        os.replace(tmpm, path / CKPT_META)
        (path / CKPT_FLAT).write_text(centroids_to_json(c))
    if comm is not None:
        comm.barrier()
    return path


def _jsonable(o):
    if hasattr(o, "tolist"):
        return o.tolist()
    if hasattr(o, "as_dict"):
        return o.as_dict()
    return str(o)


def load_checkpoint(path, comm=None, device=None) -> dict:
    """Read a checkpoint (rank 0) and broadcast it to every rank of ``comm``."""
    path = Path(path)
    rank = comm.rank if comm is not None else 0
    state = None
    if rank == 0:
        meta = json.loads((path / CKPT_META).read_text())
        t = load_file(str(path / CKPT_TENSORS))["centers"]
        state = {**meta, "centers": t}
    if comm is not None and comm.world > 1:
        blob = None
        if state is not None:
            hdr = {k: v for k, v in state.items() if k != "centers"}
            hdr["_shape"] = list(state["centers"].shape)
            blob = json.dumps(hdr).encode()
        meta = json.loads(comm.broadcast_bytes(blob, 0).decode())   # JSON, never unpickled
        shape = meta.pop("_shape")
        buf = (state["centers"] if state else torch.zeros(shape)).to(comm.device)
        comm.broadcast_(buf, 0)
        state = {**meta, "centers": buf.cpu()}
    if device is not None:
        state["centers"] = state["centers"].to(device)
    return state
