"""Public estimator API: ``KMeans``, ``MiniBatchKMeans``, functional ``fit`` / ``predict``.

The surface follows scikit-learn's (``fit``, ``predict``, ``fit_predict``,
``transform``, ``score``, ``cluster_centers_``, ``labels_``, ``inertia_``,
``n_iter_``) on a PyTorch-ROCm engine: GPU tensors run the gfx950 kernels, CPU
tensors the PyTorch reference path, and a multi-process job (one rank per GPU,
RCCL) fits on per-rank shards with :class:`~mikmeans.parallel.Comm`.

Reference parity map: assignment of points to centroids
(R14/R25-R27 drag/drop + select, app.mjs:358-402) -> ``predict``/E-step;
centroid management (R13 addCentroid/removeCentroid, app.mjs:125-142) ->
``n_clusters``/``init``; locked centroids (app.mjs:128, :360) -> ``frozen``;
iteration counter + metric snapshots (R23/R31, app.mjs:288, :498-508) ->
``n_iter_`` / ``history_``; export/import (R21/R22) -> ``save``/``load`` and
:mod:`mikmeans.utils.io_json`.
"""
from __future__ import annotations

import math
import time

import numpy as np
import torch

from .config import KMeansConfig, resolve_dtype
from .models.init import resolve_init
from .models.lloyd import LloydEngine, tol_to_abs
from .models.minibatch import MiniBatchEngine
from .ops import pad_columns
from .parallel.comm import Comm, get_comm
from .utils import faults
from .utils import metrics as mmetrics


def _default_device(device, X=None):
    """Explicit device > the input tensor's device > cuda when available > cpu."""
    if device is not None:
        return torch.device(device)
    if X is not None and torch.is_tensor(X):
        return X.device
    return torch.device("cuda" if torch.cuda.is_available() else "cpu")


def _to_tensor(X, device, dtype):
    was_numpy = not torch.is_tensor(X)
    t = torch.as_tensor(np.asarray(X) if was_numpy else X)
    if t.dim() != 2:
        raise ValueError(f"X must be 2-D [n_samples, n_features], got shape {tuple(t.shape)}")
    t = t.to(device=device)
    if t.dtype != dtype:
        t = t.to(dtype)
    return t, was_numpy


def _unit_rows(X: torch.Tensor, block: int = 1 << 22) -> torch.Tensor:
    """Rows scaled to unit L2 norm (f32 arithmetic, result in X's dtype; zero rows stay 0)."""
    out = torch.empty_like(X)
    for i in range(0, X.shape[0], block):
        xb = X[i : i + block].to(torch.float32)
        out[i : i + block] = (xb / xb.norm(dim=1, keepdim=True).clamp_min(1e-30)).to(X.dtype)
    return out


def native_dpad(D: int, dtype) -> int:
    """The MFMA kernels' padded width for D features (0: D > 1024, PyTorch GEMM path)."""
    from .ops import native

    return native.dpad_for(pad_columns(torch.empty((0, D), dtype=dtype)).shape[1], dtype)


def native_mod():
    from .ops import native

    return native.require()


def _device_rows(X: torch.Tensor, device, dtype, gpu: bool, block_bytes: int = 1 << 26) -> torch.Tensor:
    """``X`` on ``device`` in ``dtype`` -- column-padded to 16-byte rows for the GPU kernels --
    built block by block: a host block lands on the device in its own dtype (≤ 64 MB,
    memplan.staging_items) and is converted there, so no full-size temporary in another
    dtype ever exists.  ``X`` itself when it already qualifies."""
    if not gpu:
        t = X.to(device=device)
        return t if t.dtype == dtype else t.to(dtype)
    if X.device == device and X.dtype == dtype:
        P = pad_columns(X)
        if P is X:
            return X
    n, D = X.shape
    v = 8 if dtype == torch.bfloat16 else 4
    Dp = -(-D // v) * v
    out = torch.empty((n, Dp), dtype=dtype, device=device)
    if Dp > D:
        out[:, D:].zero_()
    rows = max(1, block_bytes // max(1, D * max(X.element_size(), out.element_size())))
    for i in range(0, n, rows):
        blk = X[i : i + rows]
        if blk.device != out.device:
            blk = blk.to(out.device)          # the staging block, in the source dtype
        out[i : i + rows, :D].copy_(blk)      # cast (and pad) on the device
        del blk
    return out


def buf_empty(eng, device) -> torch.Tensor:
    """A 0-row batch for a rank with an empty shard (it still joins every step's all-reduce)."""
    return torch.zeros((0, eng.Dp), dtype=eng.dtype, device=device)


def _shard_info(n_local: int, comm: Comm, device):
    sizes = comm.all_gather(torch.tensor([n_local], dtype=torch.int64, device=device)).reshape(-1).cpu()
    start = int(sizes[: comm.rank].sum())
    return int(sizes.sum()), start


class _Params:
    """scikit-learn estimator protocol: ``get_params`` / ``set_params`` over the constructor's
    keyword arguments (so ``sklearn.base.clone``, pipelines and grid searches can rebuild an
    estimator), and a repr of the non-default ones."""

    @classmethod
    def _param_names(cls) -> list[str]:
        import inspect

        sig = inspect.signature(cls.__init__)
        return [n for n, p in sig.parameters.items() if n != "self" and p.kind == p.KEYWORD_ONLY
                or n == "n_clusters"]

    def get_params(self, deep: bool = True) -> dict:
        out = {}
        for n in self._param_names():
            if n == "random_state":
                out[n] = None          # (folded into seed by the constructor)
            else:
                out[n] = getattr(self, n, None)
        return out

    def set_params(self, **params):
        names = set(self._param_names())
        bad = [k for k in params if k not in names]
        if bad:
            raise ValueError(f"invalid parameter(s) {bad} for {type(self).__name__}")
        # validate / normalise through the constructor, then copy the parameters over
        ref = type(self)(**{**self.get_params(), **params})
        for n in names:
            if n != "random_state" and hasattr(ref, n):
                setattr(self, n, getattr(ref, n))
        return self

    def __repr__(self):
        import inspect

        sig = inspect.signature(type(self).__init__)
        cur = self.get_params()
        diff = [f"n_clusters={cur['n_clusters']}"]
        for n, p in sig.parameters.items():
            if n == "n_clusters":
                continue
            if n in cur and p.default is not inspect.Parameter.empty:
                v = cur[n]
                d = p.default
                if n == "dtype":
                    v, d = str(v).replace("torch.", ""), str(resolve_dtype(d)).replace("torch.", "")
                if isinstance(v, (int, float, str, bool, type(None))) and v != d:
                    diff.append(f"{n}={v!r}")
        return f"{type(self).__name__}({', '.join(diff)})"


class _Serving(_Params):
    """Inference surface shared by KMeans and MiniBatchKMeans (fitted ``cluster_centers_``)."""

    def _serving_pack(self, Xt):
        """The fitted centres packed for the assign kernel, built once and reused by every
        predict/score call until the centres change (serving: one kernel launch per batch)."""
        from . import ops

        c = self.cluster_centers_
        if not Xt.is_cuda or not c.is_cuda:
            return None
        D = ops.pad_columns(Xt[:1]).shape[1]
        if ops.dpad_for(D, Xt.dtype) == 0:
            return None
        key = (c._version, Xt.dtype, D, Xt.device)
        cached = getattr(self, "_pack_cache", None)
        # (the cache holds the centres tensor itself: identity + version detect any change)
        if cached is None or cached[0] is not c or cached[1] != key:
            cached = (c, key, ops.pack_centers(c, D, Xt.dtype, Xt.device))
            self._pack_cache = cached
        return cached[2]

    def _inputs(self, X):
        """X on the model's device and dtype; unit rows for the cosine metric (on the GPU by
        the same kernel the fit normalised with)."""
        Xt, was_numpy = _to_tensor(X, self.cluster_centers_.device, self.dtype)
        if getattr(self, "metric", "euclidean") == "cosine":
            if Xt.is_cuda and native_dpad(Xt.shape[1], Xt.dtype):
                P = pad_columns(Xt)
                if torch.is_tensor(X) and P.data_ptr() == X.data_ptr():
                    P = P.clone()          # never normalise the caller's rows in place
                native_mod().row_normalize(P)
                Xt = P
            else:
                Xt = _unit_rows(Xt)
        return Xt, was_numpy

    def _assign_rows(self, X, with_dist: bool, block_rows: int | None = None):
        """(labels, squared distances or None) of every row of X under the fitted centres.
        Host rows bound for a GPU model go through in blocks of ~256 MB (or ``block_rows``:
        a host-shard fit labels its rows in batch-sized blocks, the memory plan's), so a
        shard larger than HBM (a streamed fit's) is never copied to the device whole."""
        from . import ops

        dev = self.cluster_centers_.device
        host = not (torch.is_tensor(X) and X.device == dev)
        n = X.shape[0]
        if dev.type != "cuda" or not host or n == 0:
            Xt, was_numpy = self._inputs(X)
            lab, mind = ops.assign(Xt, self.cluster_centers_, with_dist=with_dist, pack=self._serving_pack(Xt))
            return lab, mind, was_numpy
        was_numpy = not torch.is_tensor(X)
        block = int(block_rows) if block_rows else max(1, (1 << 28) // max(1, X.shape[1] * 4))
        labels = torch.empty(n, dtype=torch.int32, device=dev)
        mind = torch.empty(n, dtype=torch.float32, device=dev) if with_dist else None
        for i in range(0, n, block):
            Xt, _ = self._inputs(X[i : i + block])
            lab, md = ops.assign(Xt, self.cluster_centers_, with_dist=with_dist, pack=self._serving_pack(Xt))
            labels[i : i + block] = lab
            if with_dist:
                mind[i : i + block] = md
        return labels, mind, was_numpy

    def transform(self, X):
        """Euclidean distances to every centre, ``[n, K]`` (float32; for the cosine
        metric, between unit rows and unit centres: sqrt(2 - 2 cos)).  On the GPU: the MFMA
        transform kernel on the serving pack (csrc/transform.hip)."""
        from . import ops

        self._check_fitted()
        Xt, was_numpy = self._inputs(X)
        d = ops.transform(Xt, self.cluster_centers_, pack=self._serving_pack(Xt))
        return d.cpu().numpy() if was_numpy else d

    def fit_transform(self, X, *args, **kw):
        """``fit(X)`` then the distances of ``X`` to the fitted centres."""
        return self.fit(X, *args, **kw).transform(X)

    def _check_fitted(self):
        if not hasattr(self, "cluster_centers_"):
            raise RuntimeError(f"{type(self).__name__} instance is not fitted yet; call fit() first")


class KMeans(_Serving):
    """Lloyd k-means on MI355X (full batch, data-parallel over ranks)."""

    def __init__(self, n_clusters: int = 8, *, init="k-means++", n_init: int = 1, max_iter: int = 300,
                 tol: float = 1e-4, dtype="float32", device=None, seed: int | None = 0,
                 random_state: int | None = None, comm: Comm | None = None, frozen=None,
                 empty_cluster: str = "keep", check_every: int = 1, n_local_trials=None,
                 verbose: int = 0, mode: str = "learn", run_id: str | None = None,
                 checkpoint_every: int = 0, checkpoint_dir: str | None = None, metrics_path: str | None = None,
                 graph: bool = False, incremental: bool = True, chunk_rows: int | None = None,
                 init_size: int | None = None, metric: str = "euclidean", algorithm: str = "auto",
                 init_sampling: str = "exact"):
        self.n_clusters = int(n_clusters)
        self.init = init
        self.n_init = int(n_init)
        self.max_iter = int(max_iter)
        self.tol = float(tol)
        self.dtype = resolve_dtype(dtype)
        self.device = device
        self.seed = int(random_state if random_state is not None else (seed or 0))
        self.comm = comm
        self.frozen = frozen
        self.empty_cluster = empty_cluster
        self.check_every = int(check_every)
        self.n_local_trials = n_local_trials
        self.verbose = verbose
        self.mode = mode
        self.run_id = run_id
        self.checkpoint_every = int(checkpoint_every)
        self.checkpoint_dir = checkpoint_dir
        self.metrics_path = metrics_path
        self.graph = bool(graph)
        self.incremental = bool(incremental)
        # out-of-core fits (models/streaming.py): X stays in host memory and streams through
        # the GPU in chunks of `chunk_rows`; the init (and tol scale) use `init_size` rows
        self.chunk_rows = int(chunk_rows) if chunk_rows else None
        if metric not in ("euclidean", "cosine"):
            raise ValueError(f"metric must be 'euclidean' or 'cosine', got {metric!r}")
        # cosine = spherical k-means: unit rows, centres re-normalised after every M-step
        self.metric = metric
        # 'hamerly' (sklearn's 'elkan' maps here too): the GPU E-step keeps per-row distance
        # bounds and re-assigns only the rows they cannot vouch for (models/lloyd.py) -- the
        # full E-step's labels bit for bit (tests/test_gpu_bounded.py), far fewer MFMA passes
        # once few rows move.  'auto' (default): 'hamerly' wherever the memory plan holds the
        # bounds resident (~21 B/row) and the options are the bounded path's, else 'lloyd';
        # the choice is agreed by every rank and reported as ``algorithm_``.
        algo = {"elkan": "hamerly", "full": "lloyd"}.get(algorithm, algorithm)
        if algo not in ("auto", "lloyd", "hamerly"):
            raise ValueError(f"algorithm must be 'auto', 'lloyd' or 'hamerly' ('elkan'), got {algorithm!r}")
        self.algorithm = algo
        self.algorithm_ = None
        # multi-rank k-means++: 'exact' (world-size invariant, two collectives per centre) or
        # 'two-stage' (one all-gather per centre; models/init.py)
        if init_sampling not in ("exact", "two-stage"):
            raise ValueError(f"init_sampling must be 'exact' or 'two-stage', got {init_sampling!r}")
        self.init_sampling = init_sampling
        self.init_size = init_size
        self.history_: list[dict] = []

    # ---------------------------------------------------------------- config
    @classmethod
    def from_config(cls, cfg: KMeansConfig, **kw):
        return cls(n_clusters=cfg.n_clusters, init=cfg.init, n_init=cfg.n_init, max_iter=cfg.max_iter,
                   tol=cfg.tol, dtype=cfg.dtype, device=cfg.device, seed=cfg.seed,
                   empty_cluster=cfg.empty_cluster, check_every=cfg.check_every,
                   n_local_trials=cfg.n_local_trials, verbose=cfg.verbose, mode=cfg.mode,
                   run_id=cfg.run_id, checkpoint_every=cfg.checkpoint_every,
                   checkpoint_dir=cfg.checkpoint_dir, metrics_path=cfg.metrics_path, graph=cfg.graph,
                   incremental=cfg.incremental, chunk_rows=cfg.chunk_rows, metric=cfg.metric,
                   algorithm=cfg.algorithm, init_sampling=cfg.init_sampling, **kw)

    def get_config(self) -> KMeansConfig:
        return KMeansConfig(n_clusters=self.n_clusters, init=self.init if isinstance(self.init, str) else "array",
                            n_init=self.n_init, max_iter=self.max_iter, tol=self.tol,
                            dtype="bfloat16" if self.dtype == torch.bfloat16 else "float32",
                            device=str(self.device) if self.device else None, seed=self.seed,
                            empty_cluster=self.empty_cluster, check_every=self.check_every,
                            n_local_trials=self.n_local_trials, mode=self.mode, run_id=self.run_id,
                            verbose=self.verbose, checkpoint_every=self.checkpoint_every,
                            checkpoint_dir=self.checkpoint_dir, metrics_path=self.metrics_path,
                            graph=self.graph, incremental=self.incremental, chunk_rows=self.chunk_rows,
                            metric=self.metric, algorithm=self.algorithm, init_sampling=self.init_sampling)

    # ------------------------------------------------------------------- fit
    AUTO_MIN_ROWS = 1 << 16      # per rank: below it the full E-step's pass costs less than the bounds
    AUTO_MIN_CLUSTERS = 32

    def _auto_bounded_ok(self, n_local: int, weighted: bool) -> bool:
        """This rank's vote for the bounded E-step under algorithm='auto': the option set the
        bounded path covers bit for bit (plain Euclidean, unweighted, 'keep' empty clusters, an
        in-HBM shard) and a problem big enough for the bounds to pay."""
        return (self.metric == "euclidean" and not weighted and self.empty_cluster == "keep"
                and self.chunk_rows is None and n_local >= self.AUTO_MIN_ROWS
                and self.n_clusters >= self.AUTO_MIN_CLUSTERS)

    def _memory_plan(self, X, comm, device, D, weighted):
        """Resident or streamed (parallel/memplan.py), agreed by every rank: a rank whose
        shard does not fit makes all of them stream (the init sample and its collectives
        must match).  ``chunk_rows`` forces streaming with that chunk."""
        from .parallel import memplan

        n_local = int(X.shape[0])
        self.algorithm_ = "hamerly" if self.algorithm == "hamerly" else "lloyd"
        es_src = X.element_size() if torch.is_tensor(X) else np.asarray(X).itemsize
        x_dev = torch.is_tensor(X) and X.is_cuda
        kw = dict(weighted=weighted, init=self.init, n_local_trials=self.n_local_trials,
                  empty_policy=self.empty_cluster)
        budget = memplan.hbm_budget(device)
        if self.chunk_rows is not None and not x_dev:
            plan = memplan.plan_streaming(n_local, D, self.n_clusters, self.dtype, chunk_rows=self.chunk_rows,
                                          init_rows=self.init_size, src_itemsize=es_src, **kw)
            plan.budget = budget
            # every rank learns whether any forced chunk does not fit (one collective, as below)
            flags = torch.tensor([0.0 if plan.fits else 1.0], dtype=torch.float64, device=comm.device)
            comm.allreduce_max_(flags)
            if flags[0].item() > 0:
                raise memplan.HBMCapacityError(
                    f"KMeans.fit: chunk_rows={self.chunk_rows} does not fit "
                    + (plan.summary() if not plan.fits else "another rank's HBM budget")
                    + "; use a smaller chunk_rows or more ranks")
        else:
            fit_kw = dict(budget=budget, x_on_device=x_dev, incremental=self.incremental, init_rows=self.init_size,
                          src_itemsize=es_src, copy_x=not self._x_ready(X, device), **kw)
            auto_b = self.algorithm == "auto" and self._auto_bounded_ok(n_local, weighted)
            plan = None
            if auto_b:
                try:   # the bounds must fit beside a resident shard, else the plain plan decides
                    plan = memplan.plan_fit(n_local, D, self.n_clusters, self.dtype, bounded=True, **fit_kw)
                    auto_b = plan.mode == "resident"
                except memplan.HBMCapacityError:
                    auto_b = False
                if not auto_b:
                    plan = None
            try:
                if plan is None:
                    plan = memplan.plan_fit(n_local, D, self.n_clusters, self.dtype,
                                            bounded=self.algorithm == "hamerly", **fit_kw)
                err = 0.0
            except memplan.HBMCapacityError as e:
                plan, err = e, 1.0
            no_b = 0.0 if (auto_b or self.algorithm == "hamerly") else 1.0
            flags = torch.tensor([err, 1.0 if (err == 0.0 and plan.mode == "streaming") else 0.0, no_b],
                                 dtype=torch.float64, device=comm.device)
            comm.allreduce_max_(flags)
            if self.algorithm == "auto" and flags[2].item() == 0.0:
                self.algorithm_ = "hamerly"     # every rank voted for the bounds (and holds them)
            if flags[0].item() > 0:
                raise plan if isinstance(plan, memplan.HBMCapacityError) else memplan.HBMCapacityError(
                    "KMeans.fit: another rank's shard does not fit its HBM budget")
            if flags[1].item() > 0:
                # some rank streams: all must (the init sample and its collectives must match);
                # a second agreement, so a rank that cannot follow fails every rank together
                msg = None
                if plan.mode != "streaming":
                    if x_dev:
                        msg = ("KMeans.fit: other ranks stream their shards; pass this rank's rows as a host "
                               "tensor too")
                    else:
                        try:
                            plan = self._stream_plan(n_local, D, es_src, budget, kw)
                        except memplan.HBMCapacityError as e:
                            msg = str(e)
                f2 = torch.tensor([1.0 if msg else 0.0], dtype=torch.float64, device=comm.device)
                comm.allreduce_max_(f2)
                if f2[0].item() > 0:
                    raise memplan.HBMCapacityError(msg or "KMeans.fit: another rank cannot stream its shard")
        if self.verbose and comm.rank == 0:
            print(f"[mikmeans] memory plan: {plan.summary()}", flush=True)
        return plan

    def _stream_plan(self, n_local, D, es_src, budget, kw):
        from .parallel import memplan

        R = memplan.ROW_ALIGN
        while R * 2 <= (1 << 24) and R < n_local:
            R *= 2
        while True:
            pl = memplan.plan_streaming(n_local, D, self.n_clusters, self.dtype, chunk_rows=R,
                                        init_rows=self.init_size, src_itemsize=es_src, **kw)
            pl.budget = budget
            if pl.fits:
                return pl
            if R <= memplan.ROW_ALIGN:
                # (another rank chose streaming and this one cannot stream within its budget)
                raise memplan.HBMCapacityError(f"KMeans.fit: {pl.summary()} does not fit even in "
                                               f"{memplan.ROW_ALIGN}-row chunks")
            R //= 2

    def _x_ready(self, X, device) -> bool:
        """X is already the device tensor the resident engine computes on (no copy made)."""
        if not (torch.is_tensor(X) and X.device == device and X.dtype == self.dtype) or self.metric == "cosine":
            return False
        return pad_columns(X[:0]).data_ptr() == X[:0].data_ptr() if X.shape[0] else True

    def fit(self, X, y=None, sample_weight=None, *, resume_from=None):
        """Lloyd fit.  On a GPU the memory plan (``memory_plan_``) decides whether the shard
        is copied into HBM or streamed from host memory chunk by chunk; both give the same
        model from the same start (init 'random', an array, or a resumed checkpoint;
        k-means++ seeds a streamed fit from an ``init_size``-row sample)."""
        comm = self.comm or get_comm()
        device = _default_device(self.device, X) if self.device is not None or comm.world == 1 else comm.device
        if not torch.is_tensor(X):
            X = torch.from_numpy(np.ascontiguousarray(np.asarray(X, dtype=np.float32)
                                                      if np.asarray(X).dtype not in (np.float32, np.float64)
                                                      else np.asarray(X)))
            self._numpy_io = True
        else:
            self._numpy_io = False
        if X.dim() != 2:
            raise ValueError(f"X must be 2-D [n_samples, n_features], got shape {tuple(X.shape)}")
        D = int(X.shape[1])
        w = None
        if sample_weight is not None:
            w = torch.as_tensor(np.asarray(sample_weight) if not torch.is_tensor(sample_weight)
                                else sample_weight, dtype=torch.float32)
        gpu = device.type == "cuda" and native_dpad(D, self.dtype) != 0
        self.memory_plan_ = None
        self.algorithm_ = "hamerly" if self.algorithm == "hamerly" else "lloyd"
        streaming = False
        if gpu:
            plan = self._memory_plan(X, comm, device, D, w is not None)
            self.memory_plan_ = plan.as_dict()
            streaming = plan.mode == "streaming"
        n_global, start = _shard_info(X.shape[0], comm, comm.device)
        if n_global < self.n_clusters:
            raise ValueError(f"n_samples={n_global} should be >= n_clusters={self.n_clusters}")
        spherical = self.metric == "cosine"
        if streaming:
            from .models.streaming import StreamingLloydEngine

            Xh = X if X.device.type == "cpu" else X.cpu()
            sengine = StreamingLloydEngine(Xh, self.n_clusters, chunk_rows=plan.chunk_rows, comm=comm,
                                           device=device, frozen=self.frozen, n_features=D, dtype=self.dtype,
                                           sample_weight=w, empty_policy=self.empty_cluster, spherical=spherical)
            tol_abs = tol_to_abs(self.tol, None, comm, n_global, D, stats=sengine.stats)
            Xt = None
        else:
            Xt = _device_rows(X, device, self.dtype, gpu)
            if spherical:
                if gpu:
                    if Xt is X:
                        Xt = Xt.clone()
                    from .ops import native as _nat

                    _nat.require().row_normalize(Xt)
                else:
                    Xt = _unit_rows(Xt)
            if w is not None:
                w = w.to(device)
        best = None
        t0 = time.perf_counter()
        start_iter = 0
        for trial in range(max(1, self.n_init)):
            if streaming:
                eng = sengine
                eng.reset_labels()
            else:
                eng = LloydEngine(Xt, self.n_clusters, comm=comm, sample_weight=w, frozen=self.frozen,
                                  empty_policy=self.empty_cluster, n_features=D, incremental=self.incremental,
                                  spherical=spherical, bounded=self.algorithm_ == "hamerly")
                if trial == 0:
                    stats = eng.stats if eng.gpu else None
                    tol_abs = tol_to_abs(self.tol, Xt, comm, n_global, D, stats=stats)
            if resume_from is not None and trial == 0:
                from .utils.checkpoint import load_checkpoint

                ck = load_checkpoint(resume_from, comm=comm)
                centers = ck["centers"].to(device)
                start_iter = int(ck["iteration"])
            else:
                centers = self._init_centers(eng if streaming else Xt, streaming, D, n_global, start, comm,
                                             trial)
            eng.set_centers(centers[:, :D])
            eng.iteration = start_iter
            hist = []
            mlog = mmetrics.MetricsLogger(self.metrics_path, rank=comm.rank, world=comm.world,
                                          n_points=n_global, run_id=self.run_id) if self.metrics_path else None

            def cb(st, _eng=eng, _hist=hist, _mlog=mlog):
                rec = st.as_dict()
                counts = _eng.counts.tolist() if (self.verbose > 1 or _mlog is not None) else None
                rec["counts"] = counts if self.verbose > 1 else None
                if getattr(_eng, "bounded", False):
                    rec["reassigned"] = _eng.reassigned     # rows the bounded E-step re-assigned
                _hist.append(rec)
                if _mlog is not None:
                    _mlog.log(st, counts)
                faults.maybe_fail(comm.rank, st.iteration)
                if self.verbose and comm.rank == 0:
                    what = (f"reassigned {rec['reassigned']}" if "reassigned" in rec
                            else f"inertia {st.inertia:.6g}")
                    print(f"[mikmeans] iter {st.iteration} {what} shift {st.shift:.3g} changed {st.n_changed}",
                          flush=True)
                if self.checkpoint_every and self.checkpoint_dir and st.iteration % self.checkpoint_every == 0:
                    from .utils.checkpoint import save_checkpoint

                    # Lloyd draws random numbers only while seeding (Philox / seeded NumPy keyed
                    # by config.seed and the trial); a resumed run continues from the centres
                    save_checkpoint(self.checkpoint_dir, _eng.centers, st.iteration, self.get_config(),
                                    history=_hist, comm=comm,
                                    extra={"rng": {"scheme": "seeding only, keyed by (seed, trial)",
                                                   "seed": self.seed, "trial": trial}})

            if self.graph:
                eng.capture()
            remaining = max(0, self.max_iter - start_iter)
            n_iter, converged, _ = eng.run(remaining, tol_abs, check_every=self.check_every, callback=cb)
            if mlog is not None:
                mlog.close()
            labels, mind = eng.assign(True)
            inert = torch.zeros(1, dtype=torch.float64, device=eng.device)
            if eng.n:
                if eng.weights is not None and eng.gpu:
                    C_ = native_mod()
                    C_.wdot(mind, eng.weights, inert,
                            torch.empty(C_.WDOT_SCRATCH, dtype=torch.float64, device=mind.device))
                elif eng.weights is not None:
                    inert += (mind.double() * eng.weights.double()).sum().to(inert.device)
                else:
                    inert += mind.sum(dtype=torch.float64).to(inert.device)
            del mind
            inert = inert.to(comm.device)
            comm.allreduce_(inert)
            inertia = float(inert.item())
            if best is None or inertia < best[0]:
                best = (inertia, eng, labels, n_iter, converged, hist)
                if streaming:   # the engine is reused by the next trial: keep this one's centres
                    best = best + (eng.centers.clone(),)
        inertia, eng, labels, n_iter, converged, hist = best[:6]
        self._engine = eng
        self.cluster_centers_ = best[6] if streaming else eng.centers.clone()
        self.labels_ = labels
        self.inertia_ = inertia
        self.n_iter_ = n_iter
        self.converged_ = converged
        self.history_ = hist
        self.n_features_in_ = D
        self.fit_time_s_ = time.perf_counter() - t0
        cnt = torch.bincount(labels, minlength=self.n_clusters).to(torch.float64).to(comm.device)
        comm.allreduce_(cnt)
        self.counts_ = cnt.cpu()
        return self

    def _init_centers(self, src, streaming: bool, D: int, n_global: int, start: int, comm, trial: int):
        """Initial centres.  Streamed shards: 'random' draws its rows from the whole shard
        (fetched from host memory, so the resident fit's rows), k-means++ runs on a
        device-resident ``init_size``-row sample of every rank's rows."""
        seed = self.seed + trial
        if not streaming:
            return resolve_init(self.init, src, D, self.n_clusters, n_global, start, comm, seed,
                                self.n_local_trials, sampling=self.init_sampling)
        name = self.init.lower().replace("_", "-") if isinstance(self.init, str) else None
        if name == "random":
            from .models.init import init_random

            return init_random(None, D, self.n_clusters, n_global, start, comm, seed, fetch=src.fetch_rows,
                               n_local=src.n)
        if name is None:
            return resolve_init(self.init, src.fetch_rows([]), D, self.n_clusters, n_global, start, comm,
                                seed, self.n_local_trials)
        m = self.init_size or max(20 * self.n_clusters, 1 << 16)
        Xs = src.sample_rows(m, self.seed)
        s_global, s_start = _shard_info(Xs.shape[0], comm, comm.device)
        return resolve_init(self.init, Xs, D, self.n_clusters, s_global, s_start, comm, seed,
                            self.n_local_trials, sampling=self.init_sampling)

    def fit_predict(self, X, y=None, sample_weight=None):
        return self.fit(X, sample_weight=sample_weight)._out(self.labels_)

    # --------------------------------------------------------------- predict
    def reset(self):
        """Forget the fit (the reference's hard reset, app.mjs:225-237); keeps the config."""
        for k in ("cluster_centers_", "labels_", "inertia_", "n_iter_", "converged_", "counts_",
                  "n_features_in_", "fit_time_s_", "_engine"):
            self.__dict__.pop(k, None)
        self.history_ = []
        return self

    def _out(self, t):
        if getattr(self, "_numpy_io", False):
            return t.cpu().numpy()
        return t

    def predict(self, X, *, unassign_nonfinite: bool = False):
        """Nearest-centre labels.  ``unassign_nonfinite`` gives rows with NaN/inf
        coordinates the label -1 ("unassigned", the reference's unassigned list,
        app.mjs:421-433); the M-step ignores such labels."""
        self._check_fitted()
        labels, _, was_numpy = self._assign_rows(X, False)
        if unassign_nonfinite:
            Xt = torch.as_tensor(np.asarray(X) if not torch.is_tensor(X) else X)
            bad = (~torch.isfinite(Xt).all(dim=1)).to(labels.device)
            labels = labels.masked_fill(bad, -1)
        return labels.cpu().numpy() if was_numpy else labels

    def score(self, X, sample_weight=None):
        """Negative inertia of ``X`` under the fitted centres."""
        self._check_fitted()
        _, mind, _ = self._assign_rows(X, True)
        if sample_weight is not None:
            mind = mind * torch.as_tensor(np.asarray(sample_weight), dtype=torch.float32, device=mind.device)
        return -float(mind.sum(dtype=torch.float64))

    # --------------------------------------------------------------- metrics
    def metrics(self) -> dict:
        """Dashboard metrics of the fit (reference snapshotMetrics parity, app.mjs:481-496)."""
        self._check_fitted()
        counts = [int(c) for c in self.counts_.tolist()]
        return {
            "k": self.n_clusters,
            "counts": counts,
            "balance": mmetrics.balance(counts),
            "inertia": self.inertia_,
            "n_iter": self.n_iter_,
        }

    # ------------------------------------------------------------- persist
    def save(self, path):
        from .utils.checkpoint import save_checkpoint

        self._check_fitted()
        return save_checkpoint(path, self.cluster_centers_, self.n_iter_, self.get_config(),
                               history=self.history_, comm=self.comm or get_comm())

    @classmethod
    def load(cls, path, device=None):
        from .utils.checkpoint import load_checkpoint

        ck = load_checkpoint(path)
        cfg = KMeansConfig.from_dict(ck["config"])
        km = cls.from_config(cfg)
        dev = _default_device(device)
        km.cluster_centers_ = ck["centers"].to(dev)
        km.n_iter_ = int(ck["iteration"])
        km.history_ = ck.get("history", [])
        km.n_features_in_ = km.cluster_centers_.shape[1]
        return km


def _splitmix64(x: int) -> int:
    x = (x + 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
    return x ^ (x >> 31)


def _step_generator(seed: int, rank: int, step: int) -> torch.Generator:
    """CPU generator for one mini-batch step (step -1: the init sample), keyed by
    (seed, rank, step) so a resumed fit draws the rows the uninterrupted one would."""
    key = _splitmix64(_splitmix64(_splitmix64(seed & 0xFFFFFFFFFFFFFFFF) ^ rank) ^ (step & 0xFFFFFFFFFFFFFFFF))
    return torch.Generator(device="cpu").manual_seed(key & 0x7FFFFFFFFFFFFFFF)


class MiniBatchKMeans(_Serving):
    """Mini-batch k-means (Sculley 2010) over tensors or device-generated streams."""

    def __init__(self, n_clusters: int = 8, *, batch_size: int = 1024, max_iter: int = 100,
                 max_steps: int | None = None, init="k-means++", init_size: int | None = None,
                 dtype="float32", device=None, seed: int = 0, comm: Comm | None = None, frozen=None,
                 tol: float = 0.0, verbose: int = 0, init_sampling: str = "exact"):
        self.n_clusters = int(n_clusters)
        self.batch_size = int(batch_size)
        if init_sampling not in ("exact", "two-stage"):
            raise ValueError(f"init_sampling must be 'exact' or 'two-stage', got {init_sampling!r}")
        self.init_sampling = init_sampling
        self.max_iter = int(max_iter)
        self.max_steps = max_steps
        self.init = init
        self.init_size = init_size
        self.dtype = resolve_dtype(dtype)
        self.device = device
        self.seed = int(seed)
        self.comm = comm
        self.frozen = frozen
        self.tol = float(tol)
        self.verbose = verbose
        self._eng = None

    def _engine(self, D, device):
        if self._eng is None:
            comm = self.comm or get_comm()
            self._eng = MiniBatchEngine(self.n_clusters, D, self.batch_size, dtype=self.dtype,
                                        device=device, comm=comm, frozen=self.frozen)
        return self._eng

    def _init_centers(self, sample: torch.Tensor):
        comm = self.comm or get_comm()
        D = sample.shape[1]
        n_global, start = _shard_info(sample.shape[0], comm, sample.device)
        Xs = pad_columns(sample) if sample.is_cuda else sample
        return resolve_init(self.init, Xs, D, self.n_clusters, n_global, start, comm, self.seed,
                            None, sampling=self.init_sampling)[:, :D]

    def fit(self, X, *, resume_from=None, checkpoint_every: int = 0, checkpoint_dir=None):
        """Fit on a tensor/array (random batches each step; ``max_iter`` epochs).

        Batch row j of step s on rank r is local row floor(u * n) for a Philox draw keyed by
        (seed; j, s, r) (:mod:`mikmeans.data.sampler`), so the sampler's state is the step
        counter itself: ``checkpoint_every`` saves centres, running counts, scales and the
        step, and ``resume_from`` continues such a run with the rows every later step draws
        -- bit for bit the uninterrupted fit on the same world size.

        On a GPU the memory plan (``memory_plan_``, parallel/memplan.py) keeps the shard in
        HBM when it fits and draws every batch on the device (csrc/rows.hip: one gather
        kernel, no host work per step); a shard over the budget stays in host memory and its
        batches (the same rows) are gathered on the host.  The fixed-point scales come from
        the whole shard's column maxima, so no batch can saturate them and steps never
        synchronise with the host (the ``tol`` check reads the shift every 10 steps)."""
        from .data.sampler import sample_indices
        from .ops import col_stats
        from .parallel import memplan
        from .utils import faults
        from .utils.checkpoint import load_checkpoint

        comm = self.comm or get_comm()
        device = _default_device(self.device, X) if self.device is not None or comm.world == 1 else comm.device
        if not torch.is_tensor(X):
            a = np.asarray(X)
            X = torch.from_numpy(np.ascontiguousarray(a if a.dtype in (np.float32, np.float64)
                                                      else a.astype(np.float32)))
            self._numpy_io = True
        else:
            self._numpy_io = False
        n, D = int(X.shape[0]), int(X.shape[1])
        gpu = device.type == "cuda" and native_dpad(D, self.dtype) != 0
        b = min(self.batch_size, n) if n else 0
        self.memory_plan_ = None
        resident = True
        if gpu:
            x_ready = (torch.is_tensor(X) and X.device == device and X.dtype == self.dtype
                       and (not n or pad_columns(X[:0]).data_ptr() == X[:0].data_ptr()))
            src_es = X.element_size() if torch.is_tensor(X) else 4
            plan = memplan.plan_minibatch(n, D, self.n_clusters, self.dtype, batch_rows=self.batch_size,
                                          resident=True, init_rows=self.init_size, copy_x=not x_ready,
                                          src_itemsize=src_es if not X.is_cuda else memplan.esize_of(self.dtype))
            plan.budget = memplan.hbm_budget(device)
            if not plan.fits and not X.is_cuda:
                plan = memplan.plan_minibatch(n, D, self.n_clusters, self.dtype, batch_rows=self.batch_size,
                                              resident=False, init_rows=self.init_size, src_itemsize=src_es)
                plan.budget = memplan.hbm_budget(device)
                resident = False
            if not plan.fits:
                raise memplan.HBMCapacityError(f"MiniBatchKMeans.fit: {plan.summary()} does not fit; "
                                               "use a smaller batch_size or more ranks")
            self.memory_plan_ = plan.as_dict()
        # (sizes only: the fit's device copies are freed when it returns; a refit allocates
        # its own before anything of this one could still be referenced)
        self._fit_buffer_bytes = {}
        if not gpu or resident:
            Xt = _device_rows(X, device, self.dtype, gpu)
            Xh = None
        else:
            Xt, Xh = None, (X if X.device.type == "cpu" else X.cpu())
        eng = self._engine(D, device)
        if eng.gpu:
            # per-column bound of the whole shard (in the compute dtype): fixed scales, never exceeded
            if Xt is not None:
                bound = col_stats(Xt, stats=False).absmax
            else:
                bound = torch.zeros(D, dtype=torch.float64)
                for i in range(0, n, 1 << 20):
                    xb = Xh[i : i + (1 << 20)].to(self.dtype).float().abs()
                    bound = torch.maximum(bound, xb.amax(0).double())
            eng.set_bound(bound)
        # the fit's own device buffers, allocated before the seeding so the plan's phases
        # (persistent + the largest transient) bound the real peak
        from .parallel.memplan import _r

        buf = rows = None
        fb = self._fit_buffer_bytes
        if eng.gpu and Xt is not None and Xt.data_ptr() != getattr(X, "data_ptr", lambda: None)():
            fb["X"] = _r(Xt.numel() * Xt.element_size())     # the fit's device copy of the shard
        if eng.gpu and b:
            if Xt is not None:    # device shard: the step reads X[rows] in place, nothing gathered
                rows = torch.empty(b, dtype=torch.int64, device=device)
                fb["rows"] = _r(rows.numel() * rows.element_size())
            else:                 # host shard: the batch's rows are gathered on the host
                buf = torch.zeros((b, eng.Dp), dtype=self.dtype, device=device)
                fb["batch"] = _r(buf.numel() * buf.element_size())
        if resume_from is not None:
            ck = load_checkpoint(resume_from, comm=comm)
            if ck.get("kind") != "minibatch" or int(ck["n_features"]) != D:
                raise ValueError(f"{resume_from} is not a mini-batch checkpoint for {D} features")
            shard_bound = eng.bound.clone() if (eng.gpu and eng.bound is not None) else None
            eng.load_state(ck["centers"], ck["tensors"], ck["iteration"], ck.get("rescales", 0))
            if shard_bound is not None and eng.bound is not None:
                # the restored scales must still cover this shard (the fit's M-step runs
                # unclamped): a checkpoint written with a smaller bound (fit_stream's, or an
                # earlier fit's first-batch bound) is widened to the shard's (all-reduced MAX)
                eng.set_bound(torch.maximum(eng.bound.to(shard_bound.device), shard_bound))
        else:
            g = _step_generator(self.seed, comm.rank, -1)
            init_n = min(n, self.init_size or max(3 * self.batch_size, 3 * self.n_clusters))
            sample_idx = torch.randperm(n, generator=g)[:init_n]
            sample = (Xt[sample_idx.to(Xt.device)] if Xt is not None
                      else _device_rows(Xh[sample_idx], device, self.dtype, True))
            eng.set_centers(self._init_centers(sample))
            del sample                         # (the plan's "init" phase: freed before the steps)
            eng.steps = 0
        # the step count must be the same on every rank (each step is a collective): derive
        # it from the global row count, never from this rank's shard size
        n_global, _ = _shard_info(n, comm, comm.device)
        steps = self.max_steps or max(1, math.ceil(self.max_iter * n_global / (self.batch_size * comm.world)))
        C = native_mod() if eng.gpu else None
        while eng.steps < steps:
            s = eng.steps
            if not n:
                eng.partial_fit(X[:0].to(device) if not eng.gpu else buf_empty(eng, device))
            elif rows is not None:
                C.sample_index(n, b, self.seed, comm.rank, s, rows)           # Philox draws on device
                eng.partial_fit_rows(Xt, rows)
            else:
                idx = torch.from_numpy(sample_indices(n, b, self.seed, comm.rank, s))
                if eng.gpu:
                    buf[:, :D].copy_(Xh[idx].to(device, non_blocking=False))
                    eng.partial_fit(buf)
                else:
                    eng.partial_fit(Xt[idx])
            faults.maybe_fail(comm.rank, eng.steps)
            if checkpoint_every and checkpoint_dir and eng.steps % checkpoint_every == 0:
                self._finish(eng)
                self._save(checkpoint_dir, comm)
            if self.tol > 0 and (s + 1) % 10 == 0:
                if float(eng.shift.sum()) <= self.tol:
                    break
        self._finish(eng)
        if Xt is not None:
            self.labels_ = self.predict(Xt)
        else:   # host shard: label it in batch-sized blocks (memplan.plan_minibatch "predict")
            self.labels_ = self._assign_rows(Xh, False, block_rows=max(1, b))[0]
        if self._numpy_io and torch.is_tensor(self.labels_):
            self.labels_ = self.labels_.cpu().numpy()
        return self

    def fit_stream(self, stream, steps: int, init_batch: torch.Tensor | None = None, *, resume_from=None,
                   checkpoint_every: int = 0, checkpoint_dir=None):
        """Fit on an iterator of per-rank batches (e.g. :class:`~mikmeans.data.blobs.BlobStream`).

        ``steps`` counts the whole run; with ``checkpoint_every`` the state (centres, running
        counts, fixed-point scales, step and the stream's global row position) is saved
        every that many steps, and ``resume_from`` continues such a run -- also on another
        world size: a stream with the same global batch (``batch * world``) then replays the
        same rows per step and the exact integer M-step gives the same centres (the
        reference's export/import of the whole board, app.mjs:263-282).  Across world sizes
        that holds up to near-ties of the bf16 assign: its key offset is shared by a
        workgroup of rows, and which rows share one changes with the per-rank batch
        (f32 data, and a resume on the same world size, are bitwise).  A generic iterator
        must itself be positioned at the checkpoint's ``stream_pos`` (BlobStream is seeked)."""
        from .utils import faults
        from .utils.checkpoint import load_checkpoint

        comm = self.comm or get_comm()
        if resume_from is not None:
            ck = load_checkpoint(resume_from, comm=comm)
            if ck.get("kind") != "minibatch":
                raise ValueError(f"{resume_from} is not a mini-batch checkpoint")
            device = torch.device(getattr(stream, "device", None) or self.device or comm.device)
            eng = self._engine(int(ck["n_features"]), device)
            eng.load_state(ck["centers"], ck["tensors"], ck["iteration"], ck.get("rescales", 0))
            if hasattr(stream, "seek"):
                stream.seek(int(ck["stream_pos"]))
        else:
            first = init_batch if init_batch is not None else next(iter(stream))
            eng = self._engine(first.shape[1], first.device)
            eng.set_centers(self._init_centers(first.to(self.dtype)))
        vb = getattr(stream, "value_bound", None)
        if vb is not None and eng.gpu and (eng.col_exp is None or bool((eng.bound >= float(vb)).all())):
            # bounded stream: no per-step clamp check (also after a resume, whose restored
            # scales came from the same bound)
            eng.value_bound = float(vb)
            eng.bounded = True
        while eng.steps < steps:
            Xb = next(stream)
            eng.partial_fit(Xb, getattr(stream, "last_norms", None))
            faults.maybe_fail(comm.rank, eng.steps)
            if checkpoint_every and checkpoint_dir and eng.steps % checkpoint_every == 0:
                self._finish(eng)
                self._save(checkpoint_dir, comm, stream_pos=stream.position() if hasattr(stream, "position")
                           else None)
        self._finish(eng)
        return self

    # ------------------------------------------------------------- persist
    def _save(self, path, comm, stream_pos=None):
        from .utils.checkpoint import save_checkpoint

        eng = self._eng
        cfg = {"n_clusters": self.n_clusters, "batch_size": self.batch_size, "max_iter": self.max_iter,
               "init": self.init if isinstance(self.init, str) else "array", "dtype": str(self.dtype),
               "seed": self.seed, "tol": self.tol}
        extra = {"kind": "minibatch", "rescales": getattr(eng, "rescales", 0),
                 # the samplers are counter-based: (seed, rank, step) is the whole RNG state
                 "rng": {"scheme": "fit: Philox4x32-10 row draws keyed by (seed; row, step, rank), "
                                   "data/sampler.py; streams: Philox4x32-10 by global row (BlobStream)",
                         "seed": self.seed, "step": int(eng.steps)}}
        if stream_pos is not None:
            extra["stream_pos"] = int(stream_pos)
        return save_checkpoint(path, eng.centers, eng.steps, cfg, comm=comm, extra=extra,
                               tensors=eng.state_tensors())

    def save(self, path):
        """Checkpoint the fitted state (centres, running counts, scales, step count)."""
        self._check_fitted()
        return self._save(path, self.comm or get_comm())

    @classmethod
    def load(cls, path, device=None, comm=None):
        """A MiniBatchKMeans that continues from ``path`` (``partial_fit`` / ``predict``)."""
        from .config import resolve_dtype
        from .utils.checkpoint import load_checkpoint

        ck = load_checkpoint(path, comm=comm)
        if ck.get("kind") != "minibatch":
            raise ValueError(f"{path} is not a mini-batch checkpoint")
        c = ck["config"]
        dt = "bfloat16" if "bfloat16" in c.get("dtype", "") else "float32"
        km = cls(c["n_clusters"], batch_size=c["batch_size"], max_iter=c.get("max_iter", 100),
                 init=c.get("init", "k-means++"), dtype=resolve_dtype(dt), device=device,
                 seed=c.get("seed", 0), comm=comm, tol=c.get("tol", 0.0))
        dev = _default_device(device)
        eng = km._engine(int(ck["n_features"]), dev)
        eng.load_state(ck["centers"], ck["tensors"], ck["iteration"], ck.get("rescales", 0))
        km._finish(eng)
        return km

    def partial_fit(self, Xb):
        comm = self.comm or get_comm()
        device = _default_device(self.device, Xb) if self.device is not None or comm.world == 1 else comm.device
        Xt, _ = _to_tensor(Xb, device, self.dtype)
        eng = self._engine(Xt.shape[1], device)
        if not hasattr(self, "cluster_centers_"):
            eng.set_centers(self._init_centers(Xt))
        eng.partial_fit(Xt)
        self._finish(eng)
        return self

    def device_buffers(self) -> dict:
        """Allocator bytes of the last ``fit``'s persistent device buffers (engine + the fit's
        shard copy / row list / batch buffer), named as ``memplan.plan_minibatch`` plans them."""
        out = dict(self._eng.device_buffers()) if self._eng is not None else {}
        out.update(getattr(self, "_fit_buffer_bytes", {}))
        return out

    def _finish(self, eng):
        self.cluster_centers_ = eng.centers.clone()
        self.n_steps_ = eng.steps
        self.counts_ = eng.vcount.clone()

    def predict(self, X):
        self._check_fitted()
        labels, _, was_numpy = self._assign_rows(X, False)
        return labels.cpu().numpy() if was_numpy else labels

    def fit_predict(self, X):
        return self.fit(X).predict(X)

    def score(self, X):
        self._check_fitted()
        _, mind, _ = self._assign_rows(X, True)
        return -float(mind.sum(dtype=torch.float64))


# ------------------------------------------------------------------ functional
def fit(X, k: int, **kw):
    """``fit(X, k) -> (centers, labels)`` — the north-star functional surface."""
    km = KMeans(n_clusters=k, **kw).fit(X)
    return km._out(km.cluster_centers_), km._out(km.labels_)


def predict(X, centers, dtype="float32"):
    """Nearest-centre labels of ``X`` for given ``centers``."""
    from . import ops

    was_numpy = not torch.is_tensor(X)
    c = torch.as_tensor(np.asarray(centers) if not torch.is_tensor(centers) else centers, dtype=torch.float32)
    dev = c.device if torch.is_tensor(centers) else _default_device(None)
    Xt, _ = _to_tensor(X, dev, resolve_dtype(dtype))
    labels, _ = ops.assign(Xt, c.to(dev), with_dist=False)
    return labels.cpu().numpy() if was_numpy else labels


def fit_predict(X, k: int, **kw):
    return fit(X, k, **kw)[1]


def kmeans_plusplus(X, n_clusters: int, *, seed: int = 0, n_local_trials=None, comm: Comm | None = None,
                    dtype="float32", device=None, sampling: str = "exact"):
    """k-means++ seeding only; returns the ``[K, D]`` initial centres."""
    comm = comm or get_comm()
    dev = _default_device(device, X)
    Xt, was_numpy = _to_tensor(X, dev, resolve_dtype(dtype))
    D = Xt.shape[1]
    Xp = pad_columns(Xt) if Xt.is_cuda else Xt
    n_global, start = _shard_info(Xt.shape[0], comm, dev)
    name = "greedy-k-means++" if (n_local_trials or 1) > 1 else "k-means++"
    c = resolve_init(name, Xp, D, n_clusters, n_global, start, comm, seed, n_local_trials, sampling=sampling)
    return c.cpu().numpy() if was_numpy else c
