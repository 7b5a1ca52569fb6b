"""Dataset IO: memory-mapped, rank-sharded loading of point matrices.

``load_points(path, rank, world)`` reads ONLY the calling rank's contiguous row
range (``parallel.shard_range``) from ``.npy`` (memory-mapped, never unpickled),
``.safetensors`` (tensor ``"X"`` or the first tensor) or ``.csv`` (small files),
so a multi-GPU job never materialises the whole dataset in one process.
"""
from __future__ import annotations

from pathlib import Path

import numpy as np
import torch

from ..parallel.shard import shard_range


def num_rows(path) -> tuple[int, int]:
    p = Path(path)
    if p.suffix == ".npy":
        a = np.load(p, mmap_mode="r", allow_pickle=False)
        return int(a.shape[0]), int(a.shape[1])
    if p.suffix == ".safetensors":
        from safetensors import safe_open

        with safe_open(str(p), framework="pt") as f:
            key = "X" if "X" in f.keys() else next(iter(f.keys()))
            shape = f.get_slice(key).get_shape()
            return int(shape[0]), int(shape[1])
    a = np.loadtxt(p, delimiter=",", ndmin=2, dtype=np.float32)
    return int(a.shape[0]), int(a.shape[1])


def load_points(path, rank: int = 0, world: int = 1, dtype=torch.float32) -> tuple[torch.Tensor, int, int]:
    """Rows ``[start, end)`` of the dataset for this rank; returns ``(X_local, n_global, start)``."""
    p = Path(path)
    n, _ = num_rows(p)
    s, e = shard_range(n, rank, world)
    if p.suffix == ".npy":
        a = np.load(p, mmap_mode="r", allow_pickle=False)
        X = torch.from_numpy(np.array(a[s:e], dtype=np.float32, copy=True))
    elif p.suffix == ".safetensors":
        from safetensors import safe_open

        with safe_open(str(p), framework="pt") as f:
            key = "X" if "X" in f.keys() else next(iter(f.keys()))
            X = f.get_slice(key)[s:e].to(torch.float32)
    else:
        X = torch.from_numpy(np.loadtxt(p, delimiter=",", ndmin=2, dtype=np.float32)[s:e])
    return X.to(dtype), n, s


def save_points(path, X) -> Path:
    p = Path(path)
    arr = X.detach().cpu().float().numpy() if torch.is_tensor(X) else np.asarray(X, dtype=np.float32)
    if p.suffix == ".safetensors":
        from safetensors.numpy import save_file

        save_file({"X": np.ascontiguousarray(arr)}, str(p))
    elif p.suffix == ".csv":
        np.savetxt(p, arr, delimiter=",")
    else:
        np.save(p, arr, allow_pickle=False)
    return p
