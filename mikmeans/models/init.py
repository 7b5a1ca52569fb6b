"""Centroid initialisation: uniform random rows, k-means++ (D^2 sampling), or user array.

All schemes are defined on the *global* dataset and give the same centres for any
world size given the same seed:

* ``random``: K distinct global row indices by Floyd's algorithm (O(K), no
  permutation of N), each owner rank contributes its rows to a SUM all-reduce.
* ``k-means++``: Arthur & Vassilvitskii (2007).  The first centre is a uniform
  global row; each next centre is drawn with probability proportional to
  D^2(x) = min_j |x - c_j|^2.  On GPU the D^2 update (K5) and the sampling (K6)
  are HIP kernels and the K-1 steps run without any host synchronisation; the
  per-rank potential totals are all-gathered (C3) and the owner of the drawn row
  contributes it to an all-reduce (C4).
* ``greedy k-means++`` (``n_local_trials > 1``, sklearn's default 2+log K): each
  step draws several candidates and keeps the one with the lowest potential.
* ``k-means||`` (Bahmani et al. 2012, "scalable k-means++"): a few oversampling rounds
  each keep every row with probability ``min(1, l D^2(x) / psi)`` (``l = 2K``), so the
  whole seeding is ~2 collectives per round instead of per centre; the candidates,
  weighted by the rows they attract, are then reclustered by weighted k-means++ on every
  rank alike.  Rows are drawn with a philox uniform keyed by the global row.

Reference parity: the reference seeds one fixed card (``JESSICA``,
app.mjs:188-196) and leaves centroid placement to humans (addCentroid,
app.mjs:126-129); here seeding is algorithmic and reproducible by seed.
"""
from __future__ import annotations

import math
import os

import numpy as np
import torch

from ..ops import native
from ..parallel.comm import Comm


def floyd_sample(n: int, k: int, rng: np.random.Generator) -> np.ndarray:
    """k distinct integers from [0, n) in draw order (Floyd's algorithm)."""
    if k > n:
        raise ValueError(f"cannot draw {k} distinct rows from {n}")
    chosen: dict[int, None] = {}
    for j in range(n - k, n):
        t = int(rng.integers(0, j + 1))
        chosen[t if t not in chosen else j] = None
    out = np.fromiter(chosen.keys(), dtype=np.int64, count=k)
    rng.shuffle(out)
    return out


def gather_rows(X: torch.Tensor | None, D: int, global_idx: np.ndarray, start: int, comm: Comm, *,
                fetch=None, n_local: int | None = None) -> torch.Tensor:
    """Rows ``global_idx`` of the sharded dataset, replicated on every rank (f32 [k, D]).
    ``fetch(local_idx) -> [m, >=D]`` supplies local rows from elsewhere (a streamed shard's
    host memory) when ``X`` is None; the sum all-reduce runs on the communicator's device."""
    k = len(global_idx)
    dev = comm.device if X is None else X.device
    out = torch.zeros((k, D), dtype=torch.float64, device=dev)
    n = X.shape[0] if X is not None else int(n_local)
    loc = global_idx - start
    mine = np.nonzero((loc >= 0) & (loc < n))[0]
    if len(mine):
        if X is not None:
            li = torch.as_tensor(loc[mine], device=X.device)
            rows = X[li][:, :D]
        else:
            rows = fetch(loc[mine])[:, :D]
        out[torch.as_tensor(mine, device=dev)] = rows.to(device=dev, dtype=torch.float64)
    comm.allreduce_(out)
    return out.to(torch.float32)


def init_random(X, D, K, n_global, start, comm: Comm, seed: int, *, fetch=None,
                n_local: int | None = None) -> torch.Tensor:
    rng = np.random.default_rng(seed)
    idx = floyd_sample(n_global, K, rng)
    return gather_rows(X, D, idx, start, comm, fetch=fetch, n_local=n_local)


def init_kmeanspp(X: torch.Tensor, D: int, K: int, n_global: int, start: int, comm: Comm, seed: int,
                  n_local_trials: int = 1, xn: torch.Tensor | None = None,
                  prune: bool | None = None, owner_path: bool | None = None,
                  sampling: str = "exact") -> torch.Tensor:
    """k-means++ seeding; returns replicated f32 centres [K, D].

    ``X`` may be column-padded (only the first ``D`` columns are real).  ``prune``
    (GPU; default on, ``MIKMEANS_KPP_PRUNE=0`` turns it off) skips the rows the
    triangle inequality rules out of each D^2 pass; the centres are bit-identical.
    ``owner_path`` (GPU): draw through the multi-rank owner selection (all-gather of the
    potentials, owner kernel, all-reduce of the row) -- default only when world > 1; a
    one-rank RCCL group can force it to rehearse the collectives.

    ``sampling``: ``"exact"`` draws each centre at ``u * (global potential)`` through the
    rank that owns that point -- two dependent collectives per seeding step (the potentials'
    all-gather, then the drawn row's all-reduce), world-size invariant.  ``"two-stage"``
    draws a row inside every rank first (at ``u * local potential``) and ships it with the
    potential in ONE all-gather; a second number ``v`` then picks the rank with probability
    potential_r / total.  Same D^2 distribution (P(rank) P(row | rank) = d2_i / total), one
    round trip per step -- what a W = 8 seeding of K = 4096 centres is bound by -- but the
    centres drawn depend on how the rows are sharded.  W = 1 gives the exact centres.
    """
    if sampling not in ("exact", "two-stage"):
        raise ValueError(f"k-means++ sampling must be 'exact' or 'two-stage', got {sampling!r}")
    if prune is None:
        prune = os.environ.get("MIKMEANS_KPP_PRUNE", "1") not in ("0", "")
    rng = np.random.default_rng(seed)
    first = int(rng.integers(0, n_global))
    centers = torch.zeros((K, X.shape[1]), dtype=torch.float32, device=X.device)
    centers[0, :D] = gather_rows(X, D, np.array([first]), start, comm)[0]
    if K == 1:
        return centers[:, :D].contiguous()
    L = max(1, int(n_local_trials))
    # every random number up front: the GPU loop then never waits for the host
    u = torch.as_tensor(rng.random((K - 1) * L), dtype=torch.float64)
    # (the rank-choice numbers come after u: the exact path's stream is unchanged)
    v = torch.as_tensor(rng.random((K - 1) * L), dtype=torch.float64) if sampling == "two-stage" else None
    if X.is_cuda:
        multi = comm.world > 1 if owner_path is None else bool(owner_path)
        if v is not None and multi:
            _kpp_gpu_two_stage(X, centers, K, comm, u.to(X.device), v.to(X.device), L, prune)
        else:
            _kpp_gpu(X, centers, K, comm, u.to(X.device), L, prune, multi)
    else:
        _kpp_cpu(X, centers, K, comm, u, L, v)
    return centers[:, :D].contiguous()


def pick_rank(totals: torch.Tensor, v: torch.Tensor) -> torch.Tensor:
    """Index r with probability totals[r] / sum (inverse CDF at ``v * sum``), on the tensors'
    device without a host read; past-the-end (rounding) goes to the last non-empty rank."""
    cum = torch.cumsum(totals, 0)
    r = torch.searchsorted(cum, (v * cum[-1]).reshape(1), right=True)[0]
    nz = (totals > 0).to(torch.int64)
    last = (nz * torch.arange(totals.numel(), device=totals.device)).max()
    return torch.minimum(r, last)


def _local_target(totals_all: torch.Tensor, u: torch.Tensor, rank: int) -> tuple[torch.Tensor, torch.Tensor]:
    """Given per-rank potentials [W] and u in [0,1): (rank-local target or -1, global total)."""
    total = totals_all.sum()
    target = u * total
    cum = torch.cumsum(totals_all, 0)
    before = cum[rank] - totals_all[rank]
    local = target - before
    owner = (local >= 0) & (local < totals_all[rank])
    # fp edge: a target past the last rank's cumulative sum belongs to the last non-empty rank
    nz = torch.nonzero(totals_all > 0).flatten()
    last = nz[-1] if nz.numel() else torch.tensor(totals_all.numel() - 1, device=totals_all.device)
    edge = (target >= cum[-1]) & (last == rank)
    owner = owner | edge
    local = torch.where(edge, totals_all[rank] * (1 - 1e-12), local)
    return torch.where(owner, local, torch.full_like(local, -1.0)), total


def _kpp_gpu(X, centers, K, comm: Comm, u, L, prune: bool = True, multi: bool = False):
    C = native.require()
    n = X.shape[0]
    dev = X.device
    D = X.shape[1]
    rpb = max(256, -(-n // 2048)) if n else 256
    nb = max(1, -(-n // rpb))
    d2 = torch.empty(max(n, 1), dtype=torch.float32, device=dev)
    bs = torch.zeros(nb, dtype=torch.float64, device=dev)
    d2c = torch.empty_like(d2) if L > 1 else None
    bsc = torch.zeros_like(bs) if L > 1 else None
    cand = torch.empty((L, D), dtype=torch.float32, device=dev)
    # Triangle-inequality pruning of the D^2 passes (csrc/kpp.hip, KPP_PRUNE): owner[i] is
    # the centre d2[i] belongs to, cc the new centre's squared distances to the previous
    # ones.  Same d2 bits and block sums as the unpruned pass, far fewer rows read.
    owner = torch.zeros(max(n, 1), dtype=torch.int32, device=dev) if prune else None
    cc = torch.empty(K, dtype=torch.float32, device=dev) if prune else None

    def d2_pass(c, k, d2_, bs_, record):
        if owner is None:
            C.kpp_d2(X, c, False, d2_, bs_, rpb)
        else:
            C.kpp_cc(centers, k, c, cc)
            C.kpp_d2(X, c, False, d2_, bs_, rpb, owner, cc, k, k if record else -1)

    if n:
        C.kpp_d2(X, centers[0], True, d2, bs, rpb)
    # Per seeding step: L == 1 -- [all-gather of the W potentials] + sample + [all-reduce of
    # the drawn row, straight into centers[k]]; greedy (L > 1) -- ONE all-gather (the L
    # trials draw from the same D^2), L samples into cand, ONE all-reduce of cand [L, D],
    # L potential passes, ONE all-reduce of the L potentials.  No host synchronisation.
    for k in range(1, K):
        allt = None
        if multi:
            tot = bs.sum().reshape(1) if n else torch.zeros(1, dtype=torch.float64, device=dev)
            allt = comm.all_gather(tot).reshape(-1)
        for t in range(L):
            uk = u[(k - 1) * L + t: (k - 1) * L + t + 1]
            row = centers[k] if L == 1 else cand[t]
            if not multi:
                C.kpp_sample(bs, d2, rpb, uk, X, row, None, 1, None, 0)  # target = u * total, on device
            elif n:
                C.kpp_sample(bs, d2, rpb, uk, X, row, None, 2, allt, comm.rank)  # owner's row, else zeros
            else:
                row.zero_()
        if multi:
            comm.allreduce_(centers[k] if L == 1 else cand)
        if L == 1:
            if n:
                d2_pass(centers[k], k, d2, bs, True)
            continue
        # greedy: potential of each candidate, keep the best (ties -> first)
        pots = torch.zeros(L, dtype=torch.float64, device=dev)
        for t in range(L):
            if n:
                d2c.copy_(d2)
                d2_pass(cand[t], k, d2c, bsc, False)
                pots[t] = bsc.sum()
        comm.allreduce_(pots)
        best = torch.argmin(pots)
        centers[k] = cand[best]
        if n:
            d2_pass(centers[k], k, d2, bs, True)


def _kpp_gpu_two_stage(X, centers, K, comm: Comm, u, v, L, prune: bool = True):
    """Multi-rank k-means++ with one all-gather per seeding step (``sampling='two-stage'``):
    every rank draws its L candidates from its own D^2 (csrc/kpp.hip sample, target
    ``u * local potential``), the message [potential, L rows] is all-gathered, and every
    rank picks the same source rank per trial with ``v`` (:func:`pick_rank`).  Greedy
    trials add the one all-reduce of their L potentials, as in the exact path."""
    C = native.require()
    n, dev, D = X.shape[0], X.device, X.shape[1]
    rpb = max(256, -(-n // 2048)) if n else 256
    nb = max(1, -(-n // rpb))
    d2 = torch.empty(max(n, 1), dtype=torch.float32, device=dev)
    bs = torch.zeros(nb, dtype=torch.float64, device=dev)
    d2c = torch.empty_like(d2) if L > 1 else None
    bsc = torch.zeros_like(bs) if L > 1 else None
    rows = torch.zeros((L, D), dtype=torch.float32, device=dev)
    msg = torch.zeros(1 + L * D, dtype=torch.float64, device=dev)
    owner = torch.zeros(max(n, 1), dtype=torch.int32, device=dev) if prune else None
    cc = torch.empty(K, dtype=torch.float32, device=dev) if prune else None

    def d2_pass(c, k, d2_, bs_, record):
        if owner is None:
            C.kpp_d2(X, c, False, d2_, bs_, rpb)
        else:
            C.kpp_cc(centers, k, c, cc)
            C.kpp_d2(X, c, False, d2_, bs_, rpb, owner, cc, k, k if record else -1)

    if n:
        C.kpp_d2(X, centers[0], True, d2, bs, rpb)
    for k in range(1, K):
        if n:
            msg[0] = bs.sum()
            for t in range(L):
                C.kpp_sample(bs, d2, rpb, u[(k - 1) * L + t: (k - 1) * L + t + 1], X, rows[t], None, 1, None, 0)
            msg[1:] = rows.reshape(-1)
        else:
            msg.zero_()
        allm = comm.all_gather(msg).reshape(comm.world, 1 + L * D)
        tots = allm[:, 0]
        cand = torch.stack([allm.index_select(0, pick_rank(tots, v[(k - 1) * L + t]).reshape(1))[0,
                                                1 + t * D: 1 + (t + 1) * D] for t in range(L)]).float()
        if L == 1:
            centers[k] = cand[0]
        else:
            pots = torch.zeros(L, dtype=torch.float64, device=dev)
            for t in range(L):
                if n:
                    d2c.copy_(d2)
                    d2_pass(cand[t], k, d2c, bsc, False)
                    pots[t] = bsc.sum()
            comm.allreduce_(pots)
            centers[k] = cand[torch.argmin(pots)]
        if n:
            d2_pass(centers[k], k, d2, bs, True)


def _kpp_cpu(X, centers, K, comm: Comm, u, L, v=None):
    n = X.shape[0]
    Xf = X.to(torch.float32)
    D = X.shape[1]

    def dist_to(c):
        return ((Xf - c[None, :]) ** 2).sum(1)

    d2 = dist_to(centers[0]) if n else torch.zeros(0)
    for k in range(1, K):
        # one all-gather of the rank potentials and one all-reduce of the L drawn rows per
        # step (the trials draw from the same D^2), as on the GPU
        cs = torch.cumsum(d2.double(), 0) if n else None
        if v is not None and comm.world > 1:
            # two-stage: a row per trial drawn inside this rank, one all-gather, rank by v
            msg = torch.zeros(1 + L * D, dtype=torch.float64)
            if n:
                msg[0] = cs[-1]
                for t in range(L):
                    msg[1 + t * D: 1 + (t + 1) * D] = Xf[_draw(cs, d2, float(u[(k - 1) * L + t]) * float(cs[-1]))]
            allm = comm.all_gather(msg).reshape(comm.world, 1 + L * D)
            cand = torch.stack([allm[int(pick_rank(allm[:, 0], v[(k - 1) * L + t])), 1 + t * D: 1 + (t + 1) * D]
                                for t in range(L)]).float()
            _finish_step(comm, centers, k, cand, d2, dist_to, L)
            if n:
                d2 = torch.minimum(d2, dist_to(centers[k]))
            continue
        allt = comm.all_gather(d2.double().sum().reshape(1)).reshape(-1)
        cand = torch.zeros((L, D), dtype=torch.float32)
        for t in range(L):
            target, _ = _local_target(allt, u[(k - 1) * L + t], comm.rank)
            tv = float(target.item())
            if tv >= 0 and n:
                cand[t] = Xf[_draw(cs, d2, tv)]
        comm.allreduce_(cand)
        _finish_step(comm, centers, k, cand, d2, dist_to, L)
        if n:
            d2 = torch.minimum(d2, dist_to(centers[k]))


def _draw(cs: torch.Tensor, d2: torch.Tensor, tv: float) -> int:
    """Row at cumulative potential ``tv`` (host path); rounding past the end -> last row with d2 > 0."""
    n = d2.numel()
    i = int(torch.searchsorted(cs, torch.tensor([tv], dtype=torch.float64), right=True).item())
    if i >= n or d2[min(i, n - 1)] <= 0:
        pos = torch.nonzero(d2 > 0).flatten()
        i = int(pos[-1].item()) if pos.numel() else 0
    return i


def _finish_step(comm, centers, k, cand, d2, dist_to, L):
    if L == 1:
        centers[k] = cand[0]
        return
    n = d2.numel()
    pots = torch.tensor([float(torch.minimum(d2, dist_to(cand[t])).double().sum()) if n else 0.0
                         for t in range(L)], dtype=torch.float64)
    comm.allreduce_(pots)
    centers[k] = cand[int(torch.argmin(pots))]


def default_local_trials(K: int) -> int:
    return 2 + int(math.log(K)) if K > 1 else 1


def resolve_init(init, X, D, K, n_global, start, comm: Comm, seed: int, n_local_trials=None,
                 sampling: str = "exact"):
    if isinstance(init, str):
        name = init.lower().replace("_", "-")
        if name == "random":
            return init_random(X, D, K, n_global, start, comm, seed)
        if name in ("k-means++", "kmeans++", "kpp"):
            return init_kmeanspp(X, D, K, n_global, start, comm, seed, n_local_trials or 1, sampling=sampling)
        if name in ("greedy-k-means++", "greedy-kmeans++"):
            return init_kmeanspp(X, D, K, n_global, start, comm, seed,
                                 n_local_trials or default_local_trials(K), sampling=sampling)
        if name in ("k-means||", "kmeans||", "scalable-k-means++"):
            return init_kmeans_parallel(X, D, K, n_global, start, comm, seed, n_local_trials=n_local_trials,
                                        sampling=sampling)
        raise ValueError(f"unknown init {init!r}")
    c = torch.as_tensor(np.asarray(init) if not torch.is_tensor(init) else init, dtype=torch.float32)
    if c.shape != (K, D):
        raise ValueError(f"init array must be [{K}, {D}], got {tuple(c.shape)}")
    return c.to(X.device)


# ----------------------------------------------------------------------------- k-means||
KPAR_BLOCK = 8192          # centres per assign launch (the kernel keeps |c|^2 of all in LDS)


def _nearest(X, xn, Cb: torch.Tensor, want_labels: bool):
    """(squared distance to, index of) the nearest row of ``Cb`` [m, D] for every local row:
    the MFMA assign on the GPU (centre blocks of KPAR_BLOCK), f32 matmul distances on the
    CPU.  Ties across blocks keep the earlier block."""
    from .. import ops

    n = X.shape[0]
    best = torch.full((n,), float("inf"), dtype=torch.float32, device=X.device)
    lab = torch.zeros(n, dtype=torch.int64, device=X.device) if want_labels else None
    for b0 in range(0, Cb.shape[0], KPAR_BLOCK):
        cb = Cb[b0:b0 + KPAR_BLOCK]
        if X.is_cuda:
            pk = ops.pack_centers(cb, X.shape[1], X.dtype, X.device)
            lb = torch.empty(n, dtype=torch.int32, device=X.device)
            md = torch.empty(n, dtype=torch.float32, device=X.device)
            pk.assign(X, xn, lb, md)
        else:
            Xf = X[:, : cb.shape[1]].to(torch.float32)
            md = torch.empty(n, dtype=torch.float32)
            lb = torch.empty(n, dtype=torch.int64)
            for r0 in range(0, n, 65536):
                xs = Xf[r0:r0 + 65536]
                d = (xs * xs).sum(1, keepdim=True) - 2.0 * xs @ cb.T + (cb * cb).sum(1)[None, :]
                v, i = d.clamp_min(0).min(1)
                md[r0:r0 + 65536], lb[r0:r0 + 65536] = v, i
        if want_labels:
            upd = md < best
            lab = torch.where(upd, lb.to(torch.int64) + b0, lab)
        best = torch.minimum(best, md)
    return best, lab


def _gather_varlen(rows: torch.Tensor, comm: Comm) -> torch.Tensor:
    """Every rank's ``[m_r, D]`` rows, concatenated in rank order (one all-gather of the
    counts, one of the rows padded to the largest m_r)."""
    m = torch.tensor([rows.shape[0]], dtype=torch.int64, device=comm.device)
    counts = comm.all_gather(m).reshape(-1).tolist()
    mx = max(counts)
    if mx == 0:
        return rows[:0]
    pad = torch.zeros((mx, rows.shape[1]), dtype=torch.float32, device=comm.device)
    pad[: rows.shape[0]] = rows.to(device=comm.device, dtype=torch.float32)
    allr = comm.all_gather(pad)
    return torch.cat([allr[r, : counts[r]] for r in range(comm.world)]).to(rows.device)


def weighted_kmeanspp(C: torch.Tensor, w: torch.Tensor, K: int, u: torch.Tensor, *, graph_steps: int = 64,
                      native_kernels: bool | None = None) -> torch.Tensor:
    """k-means++ over the rows of ``C`` [M, D] weighted by ``w`` (D^2 x weight sampling),
    ``u`` [K] uniforms (``u[0]`` draws the first centre by weight); identical inputs give
    identical centres on every rank.

    On a GPU the draws run on the framework's kernels (csrc/kpp.hip ``wkpp``): per draw one
    pass lowers the candidates' f64 d2 against the previous pick and scans w * d2 per block,
    one workgroup turns u * total into the pick -- two launches, no host read, fixed summation
    orders.  Elsewhere (and with ``native_kernels=False``, the test oracle) the same draws as
    PyTorch ops (cumsum / searchsorted, replayed as hipGraphs of ``graph_steps`` steps on a
    GPU).  The two agree draw for draw unless a target falls within f64 rounding of a
    cumulative-weight boundary (their prefix sums associate differently)."""
    if native_kernels is None:
        native_kernels = C.is_cuda
    if native_kernels:
        return _weighted_kmeanspp_native(C, w, K, u)
    return _weighted_kmeanspp_torch(C, w, K, u, graph_steps=graph_steps)


def _weighted_kmeanspp_native(C: torch.Tensor, w: torch.Tensor, K: int, u: torch.Tensor) -> torch.Tensor:
    Cn = native.require()
    M, D = C.shape
    dev = C.device
    Ct = C.to(torch.float32).t().contiguous()            # [D, M]: a wave's candidate loads coalesce
    d2 = torch.full((M,), float("inf"), dtype=torch.float64, device=dev)  # (step 0 draws by weight alone)
    cum = torch.empty(M, dtype=torch.float64, device=dev)
    part = torch.empty(-(-M // 256), dtype=torch.float64, device=dev)
    state = torch.tensor([-1, 0], dtype=torch.int64, device=dev)
    out = torch.empty((K, D), dtype=torch.float32, device=dev)
    Cn.wkpp(Ct, w.to(device=dev, dtype=torch.float64).contiguous(), d2, cum, part,
            u.to(device=dev, dtype=torch.float64).contiguous(), state, out, K)
    return out


def _weighted_kmeanspp_torch(C: torch.Tensor, w: torch.Tensor, K: int, u: torch.Tensor, *,
                             graph_steps: int = 64) -> torch.Tensor:
    M = C.shape[0]
    Cd = C.double()
    wd = w.double()
    out = torch.empty((K, C.shape[1]), dtype=torch.float32, device=C.device)
    cum = torch.cumsum(wd, 0)
    i = torch.clamp(torch.searchsorted(cum, (u[0] * cum[-1]).reshape(1), right=True), max=M - 1)
    c = Cd.index_select(0, i)
    out[0:1] = c.float()
    d2 = ((Cd - c) ** 2).sum(1)
    kdev = torch.ones(1, dtype=torch.int64, device=C.device)

    def step():
        cum_ = torch.cumsum(wd * d2, 0)
        j = torch.searchsorted(cum_, u.index_select(0, kdev) * cum_[-1:], right=True).clamp_(max=M - 1)
        cj = Cd.index_select(0, j)
        out.index_copy_(0, kdev, cj.float())
        torch.minimum(d2, ((Cd - cj) ** 2).sum(1), out=d2)
        kdev.add_(1)

    done = 1
    G = int(graph_steps)
    if C.is_cuda and G > 0 and K - 1 >= 3 + 2 * G:
        side = torch.cuda.Stream(device=C.device)
        side.wait_stream(torch.cuda.current_stream(C.device))
        with torch.cuda.stream(side):       # warm-up: real steps 1..3
            for _ in range(3):
                step()
        torch.cuda.current_stream(C.device).wait_stream(side)
        done += 3
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):           # recorded, not run
            for _ in range(G):
                step()
        for _ in range((K - done) // G):
            g.replay()
            done += G
    for _ in range(K - done):
        step()
    return out


def init_kmeans_parallel(X: torch.Tensor, D: int, K: int, n_global: int, start: int, comm: Comm, seed: int,
                         *, rounds: int = 5, oversampling: float = 2.0, xn: torch.Tensor | None = None,
                         n_local_trials: int | None = None, sampling: str = "exact") -> torch.Tensor:
    """k-means|| seeding (Bahmani et al. 2012); returns replicated f32 centres [K, D].

    Per round: psi = the global potential (one all-reduce), every row g kept with probability
    ``min(1, l d2_g / psi)`` by the uniform keyed by g (csrc/rows.hip ``kpar_select``, NumPy
    mirror on the CPU), the kept rows compacted on the device and all-gathered in global row
    order, and d2 lowered against them on the MFMA assign.  Then every candidate's weight
    (rows nearest to it, one all-reduce) and a weighted k-means++ recluster run alike on
    every rank.  About 2 collectives per round plus 3 -- against 2 per centre for exact
    k-means++ -- and the candidates do not depend on the sharding (up to the f64 association
    of psi).  Data with fewer than K distinct candidates (tiny or duplicated rows) falls back
    to k-means++ with the caller's ``n_local_trials`` and ``sampling``."""
    rng = np.random.default_rng(seed)
    first = int(rng.integers(0, n_global))
    C = gather_rows(X, D, np.array([first]), start, comm)
    n = X.shape[0]
    dev = X.device
    if X.is_cuda and xn is None:
        from .. import ops

        xn = ops.row_sqnorm(X)
    ell = float(oversampling) * K
    d2 = _nearest(X, xn, C, False)[0] if n else torch.zeros(0, device=dev)
    if X.is_cuda:
        Cn = native.require()
        cand = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)
        rows = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
        cnt = torch.zeros(1, dtype=torch.int64, device=dev)
        scratch = torch.empty(max(1, Cn.compact_blocks(n)), dtype=torch.int64, device=dev)
    for rnd in range(int(rounds)):
        psi = (d2.sum(dtype=torch.float64) if n else torch.zeros((), dtype=torch.float64, device=dev)).reshape(1)
        psi = psi.to(comm.device)
        comm.allreduce_(psi)
        if float(psi.item()) <= 0.0:
            break                       # every row sits on a candidate
        if n and X.is_cuda:
            Cn.kpar_select(d2, start, psi.to(dev), ell, seed, rnd, cand)
            Cn.compact(cand[:n], rows, cnt, scratch)
            sel = rows[: int(cnt.item())]
        elif n:
            from ..data.sampler import kpar_uniform

            u = torch.from_numpy(kpar_uniform(start, n, seed, rnd))
            sel = torch.nonzero(u < ell * d2.double() / float(psi.item())).flatten()
        else:
            sel = torch.zeros(0, dtype=torch.int64, device=dev)
        new = _gather_varlen(X[sel][:, :D].to(torch.float32) if n else torch.zeros((0, D), device=dev), comm)
        if new.shape[0] == 0:
            continue
        C = torch.cat([C, new.to(C.device)])
        if n:
            d2 = torch.minimum(d2, _nearest(X, xn, new.to(dev), False)[0])
    M = C.shape[0]
    if M <= K:
        # (tiny data: every candidate is a centre; the rest by exact k-means++)
        if M < K:
            return init_kmeanspp(X, D, K, n_global, start, comm, seed, n_local_trials or 1, sampling=sampling)
        return C
    # candidate weights: rows nearest to each candidate (integer counts, exact in f64)
    if n:
        _, lab = _nearest(X, xn, C.to(dev), True)
        w = torch.bincount(lab, minlength=M).to(torch.float64)
    else:
        w = torch.zeros(M, dtype=torch.float64, device=dev)
    w = w.to(comm.device)
    comm.allreduce_(w)
    u = torch.as_tensor(rng.random(K), dtype=torch.float64, device=C.device)
    return weighted_kmeanspp(C, w.to(C.device), K, u)
