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
                    comm=None, extra: dict | None = None, tensors: dict | None = None) -> Path:
    """Write the checkpoint (rank 0) and barrier.  ``tensors``: further named state
    (e.g. mini-batch running counts) stored in the same safetensors file."""
    path = Path(path)
    rank = comm.rank if comm is not None else 0
    if rank == 0:
        path.mkdir(parents=True, exist_ok=True)
        c = centers.detach().to("cpu", torch.float32).contiguous()
        tmp = path / (CKPT_TENSORS + ".tmp")
        blobs = {"centers": c}
        for k, v in (tensors or {}).items():
            if k == "centers":
                raise ValueError("'centers' is reserved")
            blobs[k] = v.detach().to("cpu").contiguous()
        save_file(blobs, str(tmp))
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


def has_checkpoint(path) -> bool:
    path = Path(path)
    return (path / CKPT_META).is_file() and (path / CKPT_TENSORS).is_file()


_DTYPES = {str(d): d for d in (torch.float32, torch.float64, torch.int32, torch.int64, torch.uint8, torch.bfloat16)}


def load_checkpoint(path, comm=None, device=None) -> dict:
    """Read a checkpoint (rank 0) and broadcast it to every rank of ``comm``.

    Returns the JSON state plus ``centers`` and ``tensors`` (every other named tensor)."""
    path = Path(path)
    rank = comm.rank if comm is not None else 0
    state = None
    if rank == 0:
        meta = json.loads((path / CKPT_META).read_text())
        ts = load_file(str(path / CKPT_TENSORS))
        state = {**meta, "centers": ts.pop("centers"), "tensors": ts}
    if comm is not None and comm.world > 1:
        blob = None
        if state is not None:
            hdr = {k: v for k, v in state.items() if k not in ("centers", "tensors")}
            hdr["_tensors"] = [["centers", list(state["centers"].shape), str(state["centers"].dtype)]] + \
                [[k, list(v.shape), str(v.dtype)] for k, v in state["tensors"].items()]
            blob = json.dumps(hdr).encode()
        meta = json.loads(comm.broadcast_bytes(blob, 0).decode())   # JSON, never unpickled
        specs = meta.pop("_tensors")
        got = {}
        for name, shape, dt in specs:
            src = None if state is None else (state["centers"] if name == "centers" else state["tensors"][name])
            buf = (src if src is not None else torch.zeros(shape, dtype=_DTYPES[dt])).to(comm.device)
            comm.broadcast_(buf, 0)
            got[name] = buf.cpu()
        state = {**meta, "centers": got.pop("centers"), "tensors": got}
    if device is not None:
        state["centers"] = state["centers"].to(device)
    return state
