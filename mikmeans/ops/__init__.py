"""Op layer: natural-layout entry points over the gfx950 kernels.

GPU tensors run the hand-written HIP kernels of ``mikmeans._C`` (fail loudly if
the extension is missing); CPU tensors run :mod:`mikmeans.ops.cpu`, the plain
PyTorch reference of the same op (the test oracle and the demo-parity path,
BASELINE config 1).  There is no third backend.

* :func:`row_sqnorm`   K1  |x_i|^2
* :func:`assign`       K2  nearest centroid + squared distance (MFMA GEMM + argmin)
* :func:`cluster_sums` K3  per-cluster sums / counts (LDS scatter-add + f64 slab reduce)
* :class:`CentroidPack` K4 fragment-packed centroids for the assign kernel
"""
from __future__ import annotations

import torch

from . import cpu
from .native import available, dpad_for, dtype_code, require, vec_elems

__all__ = [
    "available",
    "require",
    "dpad_for",
    "vec_elems",
    "pad_columns",
    "pack_centers",
    "row_sqnorm",
    "assign",
    "cluster_sums",
    "CentroidPack",
]


def pad_columns(X: torch.Tensor, dtype: torch.dtype | None = None) -> torch.Tensor:
    """Return ``X`` in ``dtype`` with columns zero-padded to a 16-byte multiple.

    Zero columns change neither distances nor cluster sums; the GPU kernels need
    16-byte rows.  No copy when ``X`` already qualifies.
    """
    dtype = dtype or X.dtype
    v = vec_elems(dtype)
    n, d = X.shape
    dp = (d + v - 1) // v * v
    ok = X.dtype == dtype and d == dp and X.stride(1) == 1 and (n <= 1 or X.stride(0) % v == 0)
    if ok and X.data_ptr() % 16 == 0:
        return X
    out = torch.zeros((n, dp), dtype=dtype, device=X.device)
    out[:, :d] = X.to(dtype)
    return out


def row_sqnorm(X: torch.Tensor) -> torch.Tensor:
    if not X.is_cuda:
        return cpu.row_sqnorm(X)
    C = require()
    Xp = pad_columns(X)
    out = torch.empty(X.shape[0], dtype=torch.float32, device=X.device)
    C.row_sqnorm(Xp, out)
    return out


SPLIT_MAX_ROWS = 1 << 18   # assign16 splits the centre range only below ~1024 point blocks


class CentroidPack:
    """Centroids in the assign kernel's fragment-packed layout (see csrc/kernels.h).

    ``pack`` holds ``-2*c`` (bf16 or f32, as the points) and ``cn`` holds
    ``|c_q|^2`` of the quantised centroids, padded with a huge score for the
    rows between K and Kpad.
    """

    def __init__(self, K: int, D: int, dtype: torch.dtype, device):
        C = require()
        self._C = C
        self.K, self.D, self.dtype = K, D, dtype
        self.dpad = dpad_for(D, dtype)
        if self.dpad == 0:
            raise NotImplementedError(f"mikmeans: GPU assign supports D <= 1024 (got {D})")
        self.dt = dtype_code(dtype)
        self.Kpad = C.assign_kpad(self.dt, self.dpad, K)
        self._keys = None
        self.pack = torch.zeros(self.Kpad * self.dpad, dtype=dtype, device=device)
        self.cn = torch.zeros(C.assign_cn_len(self.Kpad), dtype=torch.float32, device=device)

    def load(self, centers: torch.Tensor) -> "CentroidPack":
        c = centers.to(device=self.pack.device, dtype=torch.float32).contiguous()
        assert c.shape == (self.K, self.D), (c.shape, self.K, self.D)
        self.finalize(0, None, c)
        return self

    def finalize(self, mode: int, packed, Cold, Cnew=None, frozen=None, mb_counts=None, shift=None,
                 counts=None, qshift=None):
        """K4: new centres from the all-reduced message (mode 1 Lloyd, 2 mini-batch) or
        pack-only (mode 0); always re-packs ``-2c`` / ``|c|^2`` for the next assign.
        ``qshift``: the squared move of the quantised centres the assign ranks."""
        self._C.finalize(mode, packed, Cold, Cnew, frozen, mb_counts, self.pack, self.cn, shift, counts,
                         self.dpad, self.Kpad, qshift)

    def assign(self, X, xn, labels, mind=None, slots=None, track_changed: bool = False, rows=None,
               ub=None, lb=None, scatter: bool = False, count=None, oseed=None):
        """K2 on these centres (``X`` column-padded, 16-B rows).  ``rows`` (int64, device):
        assign the gathered batch X[rows] without materialising it (labels etc. logical, or
        at the rows themselves with ``scatter``).  ``ub`` / ``lb``: also write every point's
        distance to its nearest and second-nearest centre (the bounded E-step's bounds).
        ``count`` (int64 [1], device): assign only ``rows[:count]`` (a compacted batch).
        ``oseed`` (bf16, f32 [X rows]): every row's seed offset, from :func:`seed_offsets` --
        a gathered row then gets bitwise the scores (and label) of the full pass over ``X``."""
        if rows is not None:
            self._C.assign(X, self.pack, self.cn, xn, labels, mind, slots, self.Kpad, self.dpad,
                           track_changed, None, rows, ub, lb, scatter, count, oseed)
            return
        keys = None
        if 0 < X.shape[0] <= SPLIT_MAX_ROWS and ub is None:
            # small batches split the centre range across workgroups (assign16 grid.y);
            # the kernels leave the scratch all-ones again, so it is filled only once
            if self._keys is None or self._keys.numel() < X.shape[0]:
                self._keys = torch.full((X.shape[0],), -1, dtype=torch.int64, device=X.device)
            keys = self._keys
            if xn is not None and mind is None:   # the splits park each point's seed offset there
                mind = torch.empty(X.shape[0], dtype=torch.float32, device=X.device)
        self._C.assign(X, self.pack, self.cn, xn, labels, mind, slots, self.Kpad, self.dpad,
                       track_changed, keys, None, ub, lb, False, None, oseed)

    def seed_offsets(self, xn: torch.Tensor) -> "torch.Tensor | None":
        """Per-row seed offsets the full assign over rows with norms ``xn`` gives its bf16
        keys (its workgroup's, or the row's own; csrc/rows.hip seed_offsets); None for f32,
        whose scores carry no offset."""
        if self.dtype != torch.bfloat16:
            return None
        out = torch.empty(xn.numel(), dtype=torch.float32, device=xn.device)
        self._C.seed_offsets(xn, out, self._C.assign_block_rows(self.dt, self.dpad, self.Kpad))
        return out


def pack_centers(centers: torch.Tensor, D: int, dtype: torch.dtype, device):
    """A CentroidPack of ``centers`` for points with ``D`` (column-padded) features."""
    cen = torch.zeros((centers.shape[0], D), dtype=torch.float32, device=device)
    cen[:, : centers.shape[1]] = centers.to(device=device, dtype=torch.float32)
    return CentroidPack(cen.shape[0], D, dtype, device).load(cen)


def assign(X: torch.Tensor, centers: torch.Tensor, *, with_dist: bool = True,
           pack: "CentroidPack | None" = None):
    """Nearest centroid of every row: returns ``(labels int32, sqdist float32 or None)``.

    bf16 points are compared against bf16-quantised centroids (scores
    accumulated in fp32 on the matrix cores); f32 points use the exact-f32 MFMA.
    ``pack``: a CentroidPack of ``centers`` made earlier by :func:`pack_centers` for the
    same (padded) width, dtype and device (serving: pack once, assign many batches).
    """
    if not X.is_cuda or dpad_for(pad_columns(X[:1]).shape[1], X.dtype) == 0:
        return cpu.assign(X, centers.to(X.device), with_dist=with_dist)  # CPU, or D > 1024 on the GPU
    C = require()
    Xp = pad_columns(X)
    D = Xp.shape[1]
    if pack is not None and (pack.D, pack.dtype, pack.pack.device) == (D, Xp.dtype, Xp.device):
        pk = pack
    else:
        pk = pack_centers(centers, D, Xp.dtype, X.device)
    n = Xp.shape[0]
    labels = torch.empty(n, dtype=torch.int32, device=X.device)
    xn = mind = None
    if with_dist:
        xn = torch.empty(n, dtype=torch.float32, device=X.device)
        C.row_sqnorm(Xp, xn)
        mind = torch.empty(n, dtype=torch.float32, device=X.device)
    pk.assign(Xp, xn, labels, mind)
    return labels, mind


def transform(X: torch.Tensor, centers: torch.Tensor, *, squared: bool = False,
              pack: "CentroidPack | None" = None) -> torch.Tensor:
    """Distance of every row to every centre, ``[n, K]`` float32 (squared with ``squared``):
    on the GPU the MFMA transform kernel (csrc/transform.hip) on the assign kernel's packed
    centres -- the distances its argmin ranks; elsewhere the PyTorch reference."""
    if not X.is_cuda or dpad_for(pad_columns(X[:1]).shape[1], X.dtype) == 0:
        c = cpu.quantize_centers(centers.to(X.device), X.dtype)
        d = torch.cdist(X.to(torch.float32), c)
        return d * d if squared else d
    C = require()
    Xp = pad_columns(X)
    D = Xp.shape[1]
    if pack is not None and (pack.D, pack.dtype, pack.pack.device) == (D, Xp.dtype, Xp.device):
        pk = pack
    else:
        pk = pack_centers(centers, D, Xp.dtype, X.device)
    n = Xp.shape[0]
    xn = torch.empty(n, dtype=torch.float32, device=X.device)
    out = torch.empty((n, pk.K), dtype=torch.float32, device=X.device)
    if n:
        C.row_sqnorm(Xp, xn)
        C.transform(Xp, pk.pack, pk.cn, pk.K, pk.Kpad, pk.dpad, xn, out, squared)
    return out


def max_abs(X: torch.Tensor) -> float:
    """max |x| without materialising |X| (one host read)."""
    if X.numel() == 0:
        return 0.0
    mn, mx = torch.aminmax(X)
    return max(abs(float(mn)), abs(float(mx)))


def _native_colstats_ok(X: torch.Tensor) -> bool:
    v = 16 // X.element_size()
    return (X.is_cuda and X.dtype in (torch.float32, torch.bfloat16) and X.dim() == 2 and X.stride(1) == 1
            and X.shape[1] % v == 0 and (X.shape[0] <= 1 or X.stride(0) % v == 0)
            and X.data_ptr() % 16 == 0)


def col_max_abs(X: torch.Tensor) -> torch.Tensor:
    """Per-column max |x| as float64 ``[D]`` (no |X| temporary)."""
    return col_stats(X, stats=False).absmax


class ColStats:
    """Per-column statistics of one streaming pass (csrc/finalize.hip col_absmax):
    ``absmax`` (f64 [D]); with ``stats``: ``sumabs``, ``sum``, ``sumsq`` (f64), ``nnz``
    (int64, nonzero values) and ``lowbit`` (int32: every value is an integer multiple of
    2^lowbit; LOWBIT_NONE for an all-zero column).  Statistics of row blocks merge with
    :meth:`merge` (streamed shards)."""

    LOWBIT_NONE = 2**31 - 1

    def __init__(self, absmax, sumabs=None, nnz=None, lowbit=None, sum=None, sumsq=None):
        self.absmax, self.sumabs, self.nnz, self.lowbit = absmax, sumabs, nnz, lowbit
        self.sum, self.sumsq = sum, sumsq

    @property
    def full(self) -> bool:
        return self.sumabs is not None

    def merge(self, other: "ColStats") -> "ColStats":
        if not (self.full and other.full):
            return ColStats(torch.maximum(self.absmax, other.absmax))
        return ColStats(torch.maximum(self.absmax, other.absmax), self.sumabs + other.sumabs,
                        self.nnz + other.nnz, torch.minimum(self.lowbit, other.lowbit),
                        self.sum + other.sum, self.sumsq + other.sumsq)

    @staticmethod
    def empty(D: int, device, full: bool = True) -> "ColStats":
        z = torch.zeros(D, dtype=torch.float64, device=device)
        if not full:
            return ColStats(z)
        return ColStats(z, z.clone(), torch.zeros(D, dtype=torch.int64, device=device),
                        torch.full((D,), ColStats.LOWBIT_NONE, dtype=torch.int32, device=device),
                        z.clone(), z.clone())


def _lowbit_torch(Xb: torch.Tensor) -> torch.Tensor:
    """Exponent of the lowest set bit of each nonzero finite value (f32 semantics)."""
    b = Xb.to(torch.float32).contiguous().view(torch.int32).long() & 0x7FFFFFFF
    e = b >> 23
    m = b & 0x7FFFFF
    sig = torch.where(e == 0, m, m | 0x800000)
    tz = ((sig & -sig).clamp_min(1).double().log2()).long()
    lb = torch.where(e == 0, -149 + tz, e - 150 + tz)
    return torch.where((b == 0) | (e == 255), torch.full_like(lb, ColStats.LOWBIT_NONE), lb)


def fused_norms_ok(X: torch.Tensor) -> bool:
    """Whether :func:`col_stats` can also write the row norms (a row of <= 64 16-B pieces)."""
    return _native_colstats_ok(X) and X.shape[1] <= 64 * (16 // X.element_size())


def col_stats(X: torch.Tensor, stats: bool = True, xn: torch.Tensor | None = None) -> ColStats:
    """One pass over ``X``: per-column max |x| and, with ``stats``, sum |x|, sum x, sum x^2,
    the nonzero count and the lowest-bit exponent (native kernel on the GPU, whose f64 sums
    are per-block partials summed in a fixed order: bitwise the same on every launch; torch
    elsewhere).  ``xn`` (GPU, :func:`fused_norms_ok`): also every row's |x|^2 into it, bitwise
    :func:`row_sqnorm`'s -- the fit's setup then reads X once."""
    D = X.shape[1]
    if X.shape[0] == 0:
        return ColStats.empty(D, X.device, stats)
    if xn is not None and not fused_norms_ok(X):
        raise ValueError("col_stats: fused row norms need a native-layout GPU X of <= 64 pieces per row")
    if _native_colstats_ok(X):
        out = torch.zeros(D, dtype=torch.int32, device=X.device)
        if not stats:
            require().col_absmax(X, out, None, None, None, xn)
            return ColStats(out.view(torch.float32).double())
        fs = torch.zeros((3, D), dtype=torch.float64, device=X.device)
        nz = torch.zeros(D, dtype=torch.int64, device=X.device)
        lb = torch.full((D,), ColStats.LOWBIT_NONE, dtype=torch.int32, device=X.device)
        require().col_absmax(X, out, fs, nz, lb, xn)
        return ColStats(out.view(torch.float32).double(), fs[0], nz, lb, fs[1], fs[2])
    mn, mx = torch.aminmax(X, dim=0)
    m = torch.maximum(mn.double().abs(), mx.double().abs())
    if not stats:
        return ColStats(m)
    st = ColStats.empty(D, X.device)
    st.absmax = m
    lb = st.lowbit.long()
    for i in range(0, X.shape[0], 1 << 16):
        xb = X[i : i + (1 << 16)].to(torch.float64)
        st.sumabs += xb.abs().sum(0)
        st.sum += xb.sum(0)
        st.sumsq += (xb * xb).sum(0)
        st.nnz += (xb != 0).sum(0)
        lb = torch.minimum(lb, _lowbit_torch(X[i : i + (1 << 16)]).amin(0))
    st.lowbit = lb.to(torch.int32)
    return st


# A column whose values do not all sit on the hi pass's grid (2^-col_exp) and whose max |x|
# exceeds WIDE_RATIO x the mean of its NONZERO |x| gets the residual (lo) M-step pass: its
# contributions are then exact to 2^-41 (not 2^-21) of the column maximum, so one outlier no
# longer coarsens every other point's contribution (csrc/update.hip UPD_RESID).  Columns the
# hi grid represents exactly (one-hot, small integers) and sparse columns never need it.
WIDE_RATIO = 256.0


def fixed_exps(X: torch.Tensor, weights: torch.Tensor | None = None, comm=None, bound=None):
    """Fixed-point exponents of the M-step accumulators (csrc/update.hip).

    Returns ``(col_exp, cnt_exp)``: an int32 device tensor ``[D]`` such that every
    contribution ``|x[:, d] * w| * 2^col_exp[d] <= 2^20``, and the exponent of the
    weighted counts.  ``bound`` (per-column float64 ``[D]``) overrides the data's
    column maxima; with ``comm`` the maxima are all-reduced so every rank uses the
    same scale (exact, world-size independent sums)."""
    sc = mstep_scales(X, weights, comm=comm, bound=bound, wide_ratio=0)
    return sc.col_exp, sc.cnt_exp


class MStepScales:
    """Fixed-point scales of one fit's M-step plus its wide-range columns.

    ``col_exp``/``cnt_exp`` as in :func:`fixed_exps`; ``wide_cols`` (int32 ``[nw]``) are
    the columns with max |x| > ``wide_ratio`` x mean |x|, ``wide_exps`` their lo-pass
    exponents (``col_exp + 20``) and ``col_exp2`` the kernel's per-column form (-1000
    = no lo pass)."""

    def __init__(self, col_exp, cnt_exp, wide_cols, device):
        self.col_exp, self.cnt_exp = col_exp, cnt_exp
        wc = sorted(int(c) for c in wide_cols)
        ce = col_exp.cpu()
        self.wide_cols = torch.tensor(wc, dtype=torch.int32, device=device)
        self.wide_exps = torch.tensor([int(ce[c]) + 20 for c in wc], dtype=torch.int32, device=device)
        e2 = torch.full_like(ce, -1000)
        for c in wc:
            e2[c] = int(ce[c]) + 20
        self.col_exp2 = e2.to(device)
        self.nw = len(wc)


def mstep_scales(X: torch.Tensor, weights: torch.Tensor | None = None, comm=None, bound=None,
                 n_global: int | None = None, wide_ratio: float | None = None,
                 stats: ColStats | None = None) -> MStepScales:
    """Scales of the fixed-point M-step (global over ranks) and the wide-range columns.
    ``stats``: this rank's column statistics when already computed (streamed shards)."""
    C = require()
    ratio = WIDE_RATIO if wide_ratio is None else float(wide_ratio)
    want = bound is None and ratio > 0
    st = None
    if bound is None:
        st = stats if stats is not None else col_stats(X, stats=want)
        m = st.absmax.to(device=X.device, dtype=torch.float64).clone()
    else:
        m = bound.to(device=X.device, dtype=torch.float64)
    wm = torch.zeros(1, dtype=torch.float64, device=X.device)
    if weights is not None and weights.numel():
        wm[0] = max_abs(weights)
    want = want and st is not None and st.sumabs is not None
    if want:
        sa = st.sumabs.to(device=X.device, dtype=torch.float64).clone()
        nz = st.nnz.to(device=X.device, dtype=torch.float64)
        lb = st.lowbit.to(device=X.device, dtype=torch.float64)
    if comm is not None:
        comm.allreduce_max_(m)
        comm.allreduce_max_(wm)
        if want:
            comm.allreduce_(sa)
            comm.allreduce_(nz)
            lb = -lb
            comm.allreduce_max_(lb)        # global min of the lowest-bit exponents
            lb = -lb
    w = float(wm.item()) if weights is not None else 1.0
    mh = m.cpu()
    exps = [C.fixed_exp(v * w) for v in mh.tolist()]
    col_exp = torch.tensor(exps, dtype=torch.int32, device=X.device)
    wide = []
    if want:
        mean_nz = (sa / nz.clamp_min(1)).cpu()
        lbh = lb.cpu()
        for d in range(len(exps)):
            # weighted contributions x*w are never assumed to sit on the grid
            exact = weights is None and lbh[d] + exps[d] >= 0
            if (mh[d] > 0 and not exact and mh[d] > ratio * mean_nz[d]
                    and exps[d] + 20 <= 126):  # the lo scale must stay a normal float
                wide.append(d)
    return MStepScales(col_exp, C.fixed_exp(w) if weights is not None else 0, wide, X.device)


def add_wide_lo(packed: torch.Tensor, K: int, D: int, sc: MStepScales) -> None:
    """After the all-reduce: add the wide columns' lo sums (message tail) onto their hi
    sums -- one f64 rounding of two exact integer-valued totals, so world-size invariant."""
    if not sc.nw:
        return
    KD = K * D
    lo = packed[KD + K + 2 : KD + K + 2 + K * sc.nw].view(K, sc.nw)
    pv = packed[:KD].view(K, D)
    idx = sc.wide_cols.long()
    pv.index_copy_(1, idx, pv.index_select(1, idx) + lo)


def cluster_sums(X: torch.Tensor, labels: torch.Tensor, K: int, weights: torch.Tensor | None = None):
    """Per-cluster f64 sums ``[K, D]`` and counts ``[K]`` (weighted when ``weights``)."""
    if not X.is_cuda:
        return cpu.cluster_sums(X, labels, K, weights)
    C = require()
    Xp = pad_columns(X)
    n, D = Xp.shape
    dt = dtype_code(Xp.dtype)
    nch = C.update_n_chunks(dt, K, D, n, weights is not None)
    slab = torch.empty(nch * K * D, dtype=torch.int64, device=X.device)
    cnt = torch.empty(nch * K, dtype=torch.int64, device=X.device)
    lab = labels.to(torch.int32).contiguous()
    w = weights.to(torch.float32).contiguous() if weights is not None else None
    sc = mstep_scales(Xp, w, n_global=n)
    if sc.nw and C.update_slice_width(dt, K, D, w is not None) == 0:
        sc = MStepScales(sc.col_exp, sc.cnt_exp, [], X.device)  # global-atomic fallback: no lo pass
    packed = torch.zeros(K * D + K + 2 + K * sc.nw, dtype=torch.float64, device=X.device)
    C.update(Xp, lab, K, slab, cnt, nch, w, sc.col_exp, sc.cnt_exp, False)
    C.reduce(slab, cnt, nch, K, D, None, packed, sc.col_exp, sc.cnt_exp)
    if sc.nw:
        C.update(Xp, lab, K, slab, cnt, nch, w, sc.col_exp, sc.cnt_exp, False, col_exp2=sc.col_exp2)
        C.reduce_cols(slab, nch, K, D, sc.wide_cols, sc.wide_exps, packed[K * D + K + 2 :])
        add_wide_lo(packed, K, D, sc)
    sums = packed[: K * D].view(K, D)[:, : X.shape[1]]
    return sums, packed[K * D : K * D + K]
