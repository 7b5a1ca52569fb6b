"""HBM-aware memory planning for MI355X (288 GB HBM3E per GPU) from the engines' real
allocations.

Every device buffer the fit engines allocate is listed here by name with its exact size
(rounded to the caching allocator's 512-byte granule), computed from the same launch
geometry the kernels use (a Python mirror of ``csrc/plan.h``, pinned against the native
functions by ``tests/test_memplan.py``).  :func:`plan_fit` turns (rows per rank, D, K,
dtype, options) and a byte budget into one of

* ``resident``  -- the rank's shard lives in HBM (:class:`~mikmeans.models.lloyd.LloydEngine`);
* ``streaming`` -- the shard stays in host memory and streams through two device chunk
  buffers every iteration (:class:`~mikmeans.models.streaming.StreamingLloydEngine`), with
  the largest chunk that fits;

or raises :class:`HBMCapacityError` when even the per-row state of a streamed fit (labels,
row norms: 8 B per row) does not fit -- a clear error instead of an allocator OOM half-way
through a fit, as the reference refuses its one capacity limit up front ("at most 3
centroids", app.mjs:127).  :func:`plan_minibatch` sizes a mini-batch fit (device-resident
shard + sampled batch, or a host shard gathered batch by batch).

The budget is ``MIKMEANS_HBM_BYTES`` when set (bytes this fit may allocate), else the
device's free memory plus what the caching allocator holds unused, minus headroom for the
runtime and RCCL (:func:`hbm_budget`).
"""
from __future__ import annotations

import math
import os
from dataclasses import asdict, dataclass, field

HBM_BYTES = 288 * 10**9          # MI355X HBM3E per GPU (spec)
GRANULE = 512                    # torch caching allocator rounding of every block
ROW_ALIGN = 1536                 # parallel/shard.py: shard / chunk row grid
SPLIT_MAX_ROWS = 1 << 18         # ops.SPLIT_MAX_ROWS: small batches keep u64 split keys
NSLOT, SLOT_STRIDE = 256, 8      # csrc/kernels.h
WDOT_SCRATCH = 1024              # csrc/rows.hip WDOT_BLOCKS (weighted-inertia partials)
COMPACT_ROWS = 4096              # csrc/rows.hip CMP_ROWS (candidate compaction block)
STAGING_BYTES = 1 << 26          # api._device_rows: host rows cross in blocks of this size
UPD_LDS_MAX = 160 * 1024         # csrc/plan.h
KS_NT = 1024
KS_LIST_BYTES = 2 * (KS_NT // 64) * 64 * 4


class HBMCapacityError(MemoryError):
    """The requested fit cannot be placed in the GPU's HBM budget in any supported mode."""


def _r(nbytes: int) -> int:
    """Bytes one allocation of ``nbytes`` takes from the caching allocator."""
    nbytes = int(nbytes)
    return 0 if nbytes <= 0 else -(-nbytes // GRANULE) * GRANULE


def _cdiv(a: int, b: int) -> int:
    return -(-a // b)


# ----------------------------------------------------------------- csrc/plan.h mirror
def esize_of(dtype) -> int:
    s = str(dtype)
    return 2 if "bfloat16" in s or s in ("bf16", "2") else 4


def vec_elems(esize: int) -> int:
    return 16 // esize


def padded_cols(D: int, esize: int) -> int:
    """ops.pad_columns: columns rounded up to a 16-byte multiple."""
    v = vec_elems(esize)
    return _cdiv(D, v) * v


def dpad_for(D: int, esize: int) -> int:
    """csrc/plan.h assign_dpad: powers of two up to 256, then 384 / 512 / 768 / 1024."""
    d = 4 * vec_elems(esize)
    while d < D and d < 256:
        d *= 2
    if D <= d:
        return d
    return next((w for w in (384, 512, 768, 1024) if D <= w), 0)


def upd_lds_bytes(K: int, ldc: int, weighted: bool) -> int:
    b = (K + 1) * ldc * 8 + (K + 1) * 4 + 8
    b = (b + 7) & ~7
    b += (K + 1) * 8 if weighted else 0
    return b + ((K + 1) * 2 + 7) // 8 * 8


def choose_sw(esize: int, K: int, D: int, weighted: bool, max_sw: int = 0) -> tuple[int, int]:
    """(slice width, LDS cell stride) of the column-slice M-step; (0, 0) = global fallback."""
    if K < 1 or D < 1 or (D * esize) % 4 or D % 2:
        return 0, 0
    dp = 2
    while dp < D:
        dp *= 2
    for sw in (64, 32, 16, 8, 4, 2):
        if sw > dp or (max_sw and sw > max_sw):
            continue
        if upd_lds_bytes(K, sw // 2 + 1, weighted) <= UPD_LDS_MAX:
            return sw, sw // 2 + 1
        if upd_lds_bytes(K, sw // 2, weighted) <= UPD_LDS_MAX:
            return sw, sw // 2
    return 0, 0


def n_chunks_slice(sw: int, D: int, N: int) -> int:
    if sw == 0:
        return 1
    n_slices = _cdiv(D, sw)
    nc = _cdiv(256, n_slices)
    nc = _cdiv(nc, 8) * 8
    if _cdiv(N, nc) < 256:
        nc = max(8, _cdiv(_cdiv(N, 256), 8) * 8)
    return nc


def choose_ks(esize: int, K: int, D: int):
    """K-split M-step plan (ks, kq, lpr, ldc) or None (plan::choose_ks)."""
    if K < 2 or D < 2 or D % 2 or (D * esize) % 4:
        return None
    v = 16 // esize
    lpr = 1
    while lpr * v < D:
        lpr *= 2
    if lpr > 64 or lpr < 8:
        return None
    ldc = lpr * v // 2 + 1
    ks = lpr // 4 if lpr // 4 > 1 else 1
    while ks > K:
        ks //= 2
    while True:
        kq = _cdiv(K, ks)
        if kq * ldc * 8 + kq * 4 + 16 + KS_LIST_BYTES <= UPD_LDS_MAX:
            return None if ks < 2 else (ks, kq, lpr, ldc)
        if ks >= 64:
            return None
        ks *= 2


def update_n_chunks(esize: int, K: int, D: int, N: int, weighted: bool) -> int:
    """update.hip update_n_chunks: M-step row chunks (slab depth) for an N-row pass."""
    sw = choose_sw(esize, K, D, weighted)[0]
    nc = n_chunks_slice(sw, D, N)
    if not weighted:
        ssw = choose_sw(esize, K, D, False)[0]
        ks = choose_ks(esize, K, D) if (0 < ssw < D and ssw * esize < 128) else None
        if ks is not None:
            nc = max(_cdiv(_cdiv(256, ks[0]), 8) * 8, nc)
    return nc


def assign_kpad(esize: int, dpad: int, K: int) -> int:
    ok = dpad >= 4 * vec_elems(esize) and dpad_for(dpad, esize) == dpad
    if not ok or K < 1 or K > (1 << 24):
        return 0
    ct = 1 if 16 * dpad * esize >= 16384 else 16384 // (16 * dpad * esize)
    m = 16 * ct
    return _cdiv(K, m) * m


def assign_cn_len(kpad: int) -> int:
    return _cdiv(kpad, 256) * 256


def staging_items(n: int, D: int, src_es: int, es: int, prefix: str) -> dict:
    """api._device_rows moving host rows to the device: one block at a time lands in its
    source dtype (and, when the destination rows are padded, converted to a contiguous
    block before the strided copy)."""
    if n <= 0:
        return {}
    rows = min(n, max(1, STAGING_BYTES // max(1, D * max(src_es, es))))
    it = {f"{prefix}_staging": _r(rows * D * src_es)}
    if padded_cols(D, es) != D and src_es != es:
        it[f"{prefix}_staging_cast"] = _r(rows * D * es)
    return it


# ------------------------------------------------------------------ inventories
def _centroid_items(K: int, Dp: int, esize: int, with_vcount: bool = False) -> dict:
    dpad = dpad_for(Dp, esize)
    kpad = assign_kpad(esize, dpad, K)
    it = {
        "C": _r(K * Dp * 4), "Cnew": _r(K * Dp * 4), "shift": _r(K * 4), "counts": _r(K * 4),
        "pack": _r(kpad * dpad * esize), "cn": _r(assign_cn_len(kpad) * 4),
        "slots": _r(NSLOT * SLOT_STRIDE * 8),
    }
    if with_vcount:
        it["vcount"] = _r(K * 8)
    return it


def kpp_workspace(n: int, Dp: int, K: int, trials: int = 1, prune: bool = True) -> dict:
    """models/init.py _kpp_gpu + init_kmeanspp device buffers (freed after seeding)."""
    rpb = max(256, _cdiv(n, 2048)) if n else 256
    nb = max(1, _cdiv(n, rpb))
    it = {"kpp_centers": _r(K * Dp * 4), "kpp_u": _r(max(0, K - 1) * trials * 8),
          "kpp_d2": _r(max(n, 1) * 4), "kpp_block_sums": _r(nb * 8), "kpp_cand": _r(trials * Dp * 4)}
    if prune:
        it["kpp_owner"] = _r(max(n, 1) * 4)
        it["kpp_cc"] = _r(K * 4)
    if trials > 1:
        it["kpp_d2c"] = _r(max(n, 1) * 4)
        it["kpp_bsc"] = _r(nb * 8)
        it["kpp_pots"] = _r(trials * 8)
    return it


def _init_items(init, n: int, Dp: int, D: int, K: int, trials: int) -> dict:
    name = init.lower().replace("_", "-") if isinstance(init, str) else "array"
    if name in ("k-means++", "kmeans++", "kpp", "greedy-k-means++", "greedy-kmeans++"):
        t = trials if trials else (2 + int(math.log(K)) if name.startswith("greedy") and K > 1 else 1)
        return kpp_workspace(n, Dp, K, max(1, t))
    if name in ("k-means||", "kmeans||", "scalable-k-means++"):
        # models/init.py init_kmeans_parallel: d2, flags, compacted rows, row norms, and the
        # nearest-candidate pass (best distance, int64 labels, one launch's labels / distances)
        m = 5 * 2 * K + 1
        return {"kpar_d2": _r(n * 4), "kpar_cand": _r(n), "kpar_rows": _r(n * 8), "kpar_xn": _r(n * 4),
                "kpar_best": _r(n * 4), "kpar_labels": _r(n * 8), "kpar_launch": 2 * _r(n * 4),
                "kpar_candidates": _r(m * D * 8), "kpar_scratch": _r(max(1, -(-n // COMPACT_ROWS)) * 8)}
    return {"init_rows": _r(K * D * 8)}


@dataclass
class MemoryPlan:
    mode: str                   # resident | streaming | minibatch-resident | minibatch-host
    n: int                      # rows of this rank
    D: int
    Dp: int                     # stored (16-byte padded) columns
    K: int
    dtype: str
    persistent: dict = field(default_factory=dict)   # live for the whole fit
    transient: dict = field(default_factory=dict)    # phases: the largest one counts
    budget: int | None = None
    chunk_rows: int = 0
    batch_rows: int = 0

    @property
    def persistent_bytes(self) -> int:
        return sum(self.persistent.values())

    @property
    def transient_bytes(self) -> int:
        return max((sum(v.values()) for v in self.transient.values()), default=0)

    @property
    def peak(self) -> int:
        return self.persistent_bytes + self.transient_bytes

    @property
    def fits(self) -> bool:
        return self.budget is None or self.peak <= self.budget

    def as_dict(self) -> dict:
        d = asdict(self)
        d.update(peak=self.peak, persistent_bytes=self.persistent_bytes,
                 transient_bytes=self.transient_bytes, fits=self.fits)
        return d

    def summary(self) -> str:
        gb = 1e9
        s = (f"{self.mode}: n={self.n} D={self.D} K={self.K} {self.dtype} peak {self.peak / gb:.3f} GB"
             + (f" of {self.budget / gb:.3f} GB budget" if self.budget is not None else ""))
        if self.chunk_rows:
            s += f", chunks of {self.chunk_rows} rows"
        if self.batch_rows:
            s += f", batches of {self.batch_rows} rows"
        return s


COLSTAT_BLOCKS = 8192     # csrc/finalize.hip


def colstat_cap(Dp: int) -> int:
    """csrc/finalize.hip ``colstat_cap``: blocks keeping the f64 partials within 32 MiB, 2048..8192."""
    return max(2048, min(COLSTAT_BLOCKS, (32 << 20) // (24 * max(Dp, 1))))


def colstat_rows(es: int, n: int, Dp: int) -> int:
    """Rows of the column-statistics partials one setup pass over ``n`` rows writes
    (csrc/finalize.hip ``colstat_rows``): its widest launch's block count."""
    V = 16 // es
    npt, rows = Dp // V, 0
    for p0 in range(0, npt, 64):
        L = 1
        while L < min(64, npt - p0):
            L *= 2
        rows = max(rows, min(colstat_cap(Dp), -(-n // (256 // L))))
    return rows


def _setup_items(n: int, Dp: int, es: int) -> dict:
    """The setup pass's transient (LloydEngine / StreamingLloydEngine ``col_stats``): the
    per-block f64 partials of the column statistics, zeroed and reduced in a fixed order."""
    return {"colstat_part": _r(colstat_rows(es, n, Dp) * 3 * Dp * 8)} if n else {}


def plan_resident(n: int, D: int, K: int, dtype="bfloat16", *, weighted: bool = False,
                  incremental: bool = True, init="k-means++", n_local_trials: int | None = None,
                  copy_x: bool = True, empty_policy: str = "keep", bounded: bool = False,
                  src_itemsize: int | None = None) -> MemoryPlan:
    """Device-resident Lloyd fit of an ``n``-row shard (``KMeans.fit``): the engine's buffers
    (models/lloyd.py ``LloydEngine._init_gpu``), the seeding workspace and the final E-step.
    ``bounded``: the Hamerly E-step's per-row bounds, flags and compacted rows (17 B/row; bf16
    adds the rows' seed offsets, 4 B/row)."""
    es = esize_of(dtype)
    Dp = padded_cols(D, es)
    wted = weighted
    p: dict = {}
    if copy_x:
        p["X"] = _r(n * Dp * es)
    if weighted:
        p["weights"] = _r(n * 4)
    p["labels"] = _r(n * 4)
    p["xn"] = _r(n * 4)
    if weighted or empty_policy == "farthest":
        p["mind"] = _r(n * 4)          # written by every step's assign (relocation reads it)
    if weighted:
        p["wdot_scratch"] = _r(WDOT_SCRATCH * 8)
    nch = update_n_chunks(es, K, Dp, max(n, 1), wted or incremental)
    p["slab"] = _r(nch * K * Dp * 8)
    p["cnt_slab"] = _r(nch * K * 8)
    p["packed"] = _r((K * Dp + K + 2) * 8)
    p.update(_centroid_items(K, Dp, es))
    final = {"labels_out": _r(n * 4), "mind_out": _r(n * 4)}
    if 0 < n <= SPLIT_MAX_ROWS:
        if bounded:
            final["split_keys"] = _r(n * 8)   # (the bounded E-step's gathered passes take no keys)
        else:
            p["split_keys"] = _r(n * 8)
    if incremental and n and n < 2**31 and choose_sw(es, K, Dp, True)[0] > 0:
        cap = max(1, min(n, int(n * 0.125)))
        p.update(delta_prev=_r(n * 4), delta_list=_r(cap * 8), delta_count=_r(4),
                 delta_tot=_r((K * Dp + K) * 8))
    if bounded:
        p.update(bound_ub=_r(n * 4), bound_lb=_r(n * 4), bound_cand=_r(n), bound_rows=_r(n * 8),
                 bound_count=_r(8), bound_scratch=_r(max(1, -(-n // COMPACT_ROWS)) * 8), bound_work=_r(16),
                 bound_qshift=_r(K * 4))
        if es == 2 and n:
            p["bound_oseed"] = _r(n * 4)   # every row's full-pass seed offset (bf16 keys)
    tr = {"init": _init_items(init, n, Dp, D, K, n_local_trials or 0), "final_assign": final,
          "setup": _setup_items(n, Dp, es)}
    if copy_x and (src_itemsize or es) != es:
        tr["load"] = staging_items(n, D, src_itemsize or es, es, "x")
    return MemoryPlan("resident", n, D, Dp, K, "bfloat16" if es == 2 else "float32", p, tr)


def plan_streaming(n: int, D: int, K: int, dtype="bfloat16", *, chunk_rows: int, weighted: bool = False,
                   init="k-means++", n_local_trials: int | None = None, init_rows: int | None = None,
                   src_itemsize: int | None = None, empty_policy: str = "keep") -> MemoryPlan:
    """Out-of-core Lloyd (models/streaming.py): per-row labels / norms on the device, two
    chunk buffers (+ a staging buffer when the host rows need a dtype / padding change),
    the M-step slab of one chunk, the init sample and its seeding workspace."""
    es = esize_of(dtype)
    Dp = padded_cols(D, es)
    R = stream_chunk_rows(chunk_rows, n)
    p = {"labels": _r(n * 4), "xn": _r(n * 4)}
    if weighted:
        p["weights"] = _r(n * 4)
        p["wdot_scratch"] = _r(WDOT_SCRATCH * 8)
    if weighted or empty_policy == "farthest":
        p["mind"] = _r(n * 4)
    p["chunk_bufs"] = 2 * _r(R * Dp * es)
    sis = src_itemsize or es
    if sis != es or Dp != D:
        p["staging"] = 2 * _r(R * D * sis)
    nch = update_n_chunks(es, K, Dp, R, weighted)
    p["slab"] = _r(nch * K * Dp * 8)
    p["cnt_slab"] = _r(nch * K * 8)
    p["packed"] = 2 * _r((K * Dp + K + 2) * 8)
    p.update(_centroid_items(K, Dp, es))
    if 0 < R <= SPLIT_MAX_ROWS:
        p["split_keys"] = _r(R * 8)
    name = init.lower().replace("_", "-") if isinstance(init, str) else "array"
    if name in ("random", "array"):
        # (api.KMeans._init_centers: rows fetched from the host shard, no device sample)
        init_tr = _init_items(init, n, Dp, D, K, 0)
    else:   # k-means++ seeds on a device-resident init_size-row sample
        m = min(n, init_rows or max(20 * K, 1 << 16))
        init_tr = {"sample": _r(m * Dp * es), **_init_items(init, m, Dp, D, K, n_local_trials or 0)}
    tr = {"init": init_tr, "final_assign": {"labels_out": _r(n * 4), "mind_out": _r(n * 4)},
          "setup": _setup_items(min(R, n), Dp, es)}      # (the statistics pass, one chunk at a time)
    pl = MemoryPlan("streaming", n, D, Dp, K, "bfloat16" if es == 2 else "float32", p, tr)
    pl.chunk_rows = R
    return pl


def stream_chunk_rows(chunk_rows: int, n: int) -> int:
    """StreamingLloydEngine's chunk: ``chunk_rows`` rounded up to the 1536-row grid, at most n."""
    return max(1, min(_cdiv(int(chunk_rows), ROW_ALIGN) * ROW_ALIGN, max(n, 1)))


def plan_minibatch(n: int, D: int, K: int, dtype="bfloat16", *, batch_rows: int, resident: bool = True,
                   init="k-means++", init_rows: int | None = None, copy_x: bool = True,
                   src_itemsize: int = 4) -> MemoryPlan:
    """Mini-batch fit (api.MiniBatchKMeans.fit, models/minibatch.py): the engine's buffers
    (``MiniBatchEngine.device_buffers``) plus the fit's own -- the shard itself when it is
    device-resident (each step then reads ``X[rows]`` in place through an int64 index list
    drawn on the device), or one gathered batch buffer for a host shard."""
    es = esize_of(dtype)
    Dp = padded_cols(D, es)
    b = int(batch_rows)
    p = {}
    if resident:
        if copy_x:
            p["X"] = _r(n * Dp * es)
        p["rows"] = _r(b * 8)
    else:
        p["batch"] = _r(b * Dp * es)
    p["batch_labels"] = _r(b * 4)
    p["clampc"] = _r(4)
    nch = update_n_chunks(es, K, Dp, b, False)
    p["slab"] = _r(nch * K * Dp * 8)
    p["cnt_slab"] = _r(nch * K * 8)
    p["packed"] = _r((K * Dp + K + 3) * 8)
    p.update(_centroid_items(K, Dp, es, with_vcount=True))
    if not resident and 0 < b <= SPLIT_MAX_ROWS:
        p["split_keys"] = _r(b * 8)     # (gathered batches take the one-pass grid: no keys)
    m = min(n, init_rows or max(3 * b, 3 * K))
    pred = {"labels_out": _r(n * 4)}
    if not resident and n:
        # api.MiniBatchKMeans.fit labels a host shard in batch-sized blocks
        # (_Serving._assign_rows): the block as copied (source dtype), its cast to the compute
        # dtype and padding, its labels
        B = min(n, max(1, b))
        pred["block_src"] = _r(B * D * src_itemsize)
        if src_itemsize != es:
            pred["block_cast"] = _r(B * D * es)
        if Dp != D:
            pred["block_padded"] = _r(B * Dp * es)
        pred["block_labels"] = _r(B * 4)
    init_tr = {"sample": _r(m * Dp * es), **_init_items(init, m, Dp, D, K, 0)}
    tr = {"init": init_tr, "predict": pred}
    if resident and copy_x and src_itemsize != es:
        tr["load"] = staging_items(n, D, src_itemsize, es, "x")
    if not resident:
        # the init sample crosses from the host through api._device_rows' staging block, and
        # every step's gathered host batch lands in its source dtype before the cast into
        # the batch buffer
        init_tr.update(staging_items(m, D, src_itemsize, es, "sample"))
        tr["step"] = {"batch_src": _r(b * D * src_itemsize)}
    pl = MemoryPlan("minibatch-resident" if resident else "minibatch-host", n, D, Dp, K,
                    "bfloat16" if es == 2 else "float32", p, tr)
    pl.batch_rows = b
    return pl


# ------------------------------------------------------------------------ budget
def hbm_budget(device=None) -> int:
    """Bytes a fit on ``device`` may allocate: ``MIKMEANS_HBM_BYTES`` when set, else the free
    device memory plus the caching allocator's unused reserve, minus headroom (2 % of HBM,
    at least 1 GiB) for the HIP runtime, RCCL buffers and the allocator's own rounding."""
    env = os.environ.get("MIKMEANS_HBM_BYTES")
    if env:
        return int(float(env))
    import torch

    free, total = torch.cuda.mem_get_info(device)
    unused = torch.cuda.memory_reserved(device) - torch.cuda.memory_allocated(device)
    return int(free + unused - max(0.02 * total, 1 << 30))


def plan_fit(n: int, D: int, K: int, dtype="bfloat16", *, budget: int, x_on_device: bool,
             weighted: bool = False, incremental: bool = True, init="k-means++",
             n_local_trials: int | None = None, init_rows: int | None = None,
             src_itemsize: int | None = None, empty_policy: str = "keep", copy_x: bool = True,
             max_chunk_rows: int = 1 << 24, bounded: bool = False) -> MemoryPlan:
    """Choose how a Lloyd fit of an ``n``-row shard runs within ``budget`` bytes of HBM:
    resident when it fits (or when X already lives on the device), else streamed in the
    largest power-of-two multiple of 1536 rows that fits; :class:`HBMCapacityError` when
    neither does."""
    res = plan_resident(n, D, K, dtype, weighted=weighted, incremental=incremental, init=init,
                        n_local_trials=n_local_trials, copy_x=copy_x, empty_policy=empty_policy,
                        bounded=bounded, src_itemsize=src_itemsize)
    res.budget = budget
    if res.fits:
        return res
    if x_on_device:
        raise HBMCapacityError(
            f"KMeans.fit: the device-resident shard needs {res.peak / 1e9:.2f} GB of HBM "
            f"({res.summary()}) but only {budget / 1e9:.2f} GB are available; pass the rows as a "
            "host (CPU) tensor to stream them, or use more ranks")
    R = ROW_ALIGN
    while R * 2 <= max_chunk_rows and R < n:
        R *= 2
    while True:
        st = plan_streaming(n, D, K, dtype, chunk_rows=R, weighted=weighted, init=init,
                            n_local_trials=n_local_trials, init_rows=init_rows, src_itemsize=src_itemsize,
                            empty_policy=empty_policy)
        st.budget = budget
        if st.fits:
            return st
        if R <= ROW_ALIGN:
            break
        R //= 2
    raise HBMCapacityError(
        f"KMeans.fit: {n} rows x {D} features need {res.peak / 1e9:.2f} GB resident and "
        f"{st.peak / 1e9:.2f} GB even when streamed in {st.chunk_rows}-row chunks "
        f"(per-row labels and norms stay on the device), but only {budget / 1e9:.2f} GB of HBM "
        "are available; use more ranks (the per-row state divides by the world size)")
