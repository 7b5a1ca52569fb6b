"""Run configuration: one dataclass, settable by kwargs or CLI flags.

The reference has no config system; its only inputs are the URL ``room`` code
(app.mjs:15-19), the ``mode`` select (learn/playtest/custom, index.html:125-127,
stored verbatim, no behaviour) and the manual ``iteration`` field (app.mjs:288).
``mode`` is kept as free-form metadata; ``run_id`` plays the room code.
"""
from __future__ import annotations

import argparse
from dataclasses import asdict, dataclass, fields

import torch

DTYPES = {
    "float32": torch.float32,
    "fp32": torch.float32,
    "f32": torch.float32,
    "bfloat16": torch.bfloat16,
    "bf16": torch.bfloat16,
}


def resolve_dtype(dtype) -> torch.dtype:
    if isinstance(dtype, torch.dtype):
        if dtype not in (torch.float32, torch.bfloat16):
            raise ValueError(f"unsupported dtype {dtype}")
        return dtype
    try:
        return DTYPES[str(dtype).lower()]
    except KeyError:
        raise ValueError(f"unsupported dtype {dtype!r} (float32 | bfloat16)") from None


def dtype_name(dtype) -> str:
    return "bfloat16" if resolve_dtype(dtype) == torch.bfloat16 else "float32"


@dataclass
class KMeansConfig:
    n_clusters: int = 8
    init: str = "k-means++"          # random | k-means++ | greedy-k-means++ (or an array via the API)
    n_init: int = 1
    max_iter: int = 300
    tol: float = 1e-4                # relative to the mean feature variance (sklearn semantics)
    dtype: str = "float32"           # compute dtype of the points: float32 | bfloat16
    seed: int = 0
    device: str | None = None        # None -> cuda if available else cpu
    batch_size: int = 0              # > 0 selects mini-batch k-means
    empty_cluster: str = "keep"      # keep | farthest
    check_every: int = 1             # host convergence check period (0 = never; benchmark)
    checkpoint_every: int = 0
    checkpoint_dir: str | None = None
    n_local_trials: int | None = None
    mode: str = "learn"              # free-form metadata, as in the reference
    run_id: str | None = None
    verbose: int = 0
    metrics_path: str | None = None  # per-iteration JSONL (rank 0)
    graph: bool = False              # replay each Lloyd iteration as one captured hipGraph
    incremental: bool = True         # M-step re-scatters only rows whose label changed (exact)
    chunk_rows: int | None = None    # out-of-core: keep X on the host, stream it in chunks of rows
    metric: str = "euclidean"        # euclidean | cosine (spherical k-means on unit rows)
    algorithm: str = "auto"          # auto | lloyd | hamerly (bounded E-step: re-assign only unproven rows)
    init_sampling: str = "exact"     # multi-rank k-means++: exact | two-stage (one all-gather per centre)
    timeout_s: float = 60.0          # collective timeout: a lost rank fails the job after this long
    resume: str | None = None        # checkpoint dir to continue from, or "auto" (= checkpoint_dir if present)

    def to_dict(self):
        return asdict(self)

    @classmethod
    def from_dict(cls, d):
        names = {f.name for f in fields(cls)}
        return cls(**{k: v for k, v in d.items() if k in names})

    @classmethod
    def add_arguments(cls, ap: argparse.ArgumentParser):
        for f in fields(cls):
            flag = "--" + f.name.replace("_", "-")
            default = f.default
            if isinstance(default, bool):
                # --flag / --no-flag (a default-on switch must be switchable off)
                ap.add_argument(flag, action=argparse.BooleanOptionalAction, default=default)
            elif default is None:
                typ = int if f.name in ("n_local_trials", "chunk_rows") else str
                ap.add_argument(flag, type=typ, default=None)
            else:
                ap.add_argument(flag, type=type(default), default=default)
        return ap

    @classmethod
    def from_args(cls, ns: argparse.Namespace):
        return cls(**{f.name: getattr(ns, f.name) for f in fields(cls) if hasattr(ns, f.name)})
