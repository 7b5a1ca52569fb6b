"""Out-of-core Lloyd: the points stay in host memory and stream through the GPU.

For shards larger than the GPU's HBM budget (N=1e9 x D=256 bf16 is
512 GB against 288 GB per MI355X; parallel/memplan.py decides) every Lloyd iteration
streams the rank's rows through two device chunk buffers.  The host tensor is page-locked
in place (hipHostRegister: no pinned copy of the shard), the host->device copy of chunk
c+1 runs on a copy stream while the compute stream assigns chunk c on the matrix cores
and scatters it into the fixed-point M-step slab, and chunk c's integer partial sums are
folded into one f64 message (exact: integer multiples of 2^-e below 2^53), so the
iteration still ends with ONE all-reduce and the same finalize as the device-resident
engine.  Per-row state stays on the device for all rows: labels and squared row norms
(8 B/row), plus distances and weights for weighted fits or the 'farthest' empty-cluster
policy.

Same options as the resident engine, with the same numerics (bitwise the resident fit
from the same start -- up to a column whose statistics sit within f64 rounding of the
wide-column threshold or the tol scale: those are f64 sums, merged chunk by chunk here and
in one pass there (each bitwise reproducible: fixed-order per-block partials,
csrc/finalize.hip), so for inexact values their last bits can differ between the two;
tests/test_gpu_mstep.py pins a column exactly at the threshold): sample weights, the cosine metric (each chunk is normalised on the
device by the same kernel as the resident rows), empty_policy 'farthest' (the farthest
rows are fetched from host memory), wide-range columns (residual lo pass per chunk, from
column statistics merged over chunks).  Host rows of another dtype or an unpadded width
are converted on the device from a staging buffer, so the host shard is never copied.

The reference has no numerics at all; its closest analog is the
export/import of the whole board (app.mjs:263-282): state that lives outside the
running replica and is brought back in.
"""
from __future__ import annotations

import torch

from ..ops import native
from ..parallel.comm import Comm
from .lloyd import LloydEngine


class StreamingLloydEngine(LloydEngine):
    """LloydEngine over a host-resident shard ``X_host`` ([n, D], CPU, any float dtype),
    computed in ``dtype`` and streamed in ``chunk_rows`` pieces.  Same public surface as
    :class:`LloydEngine` (``step``, ``run``, ``last_stats``, ``assign``, ``centers``,
    ``counts``, ``stats``); GPU only, full M-step every iteration."""

    def __init__(self, X_host: torch.Tensor, n_clusters: int, *, chunk_rows: int = 1 << 22,
                 comm: Comm | None = None, device=None, frozen=None, n_features: int | None = None,
                 dtype: torch.dtype | None = None, sample_weight: torch.Tensor | None = None,
                 empty_policy: str = "keep", spherical: bool = False):
        from ..ops import CentroidPack, ColStats, col_stats, fused_norms_ok, mstep_scales, MStepScales
        from ..parallel.memplan import padded_cols, stream_chunk_rows

        if X_host.device.type != "cpu":
            raise ValueError("StreamingLloydEngine streams a host (CPU) tensor")
        self.comm = comm or Comm.local(device or "cuda")
        dev = torch.device(device) if device is not None else self.comm.device
        if dev.type != "cuda":
            raise ValueError("StreamingLloydEngine needs a GPU device")
        C = native.require()
        self._C = C
        self.incremental = False
        self.spherical = bool(spherical)
        self.delta = None
        self.bounded = False      # (every chunk is assigned in full each pass)
        self.segments = 1
        self.empty_policy = empty_policy
        self.K = int(n_clusters)
        self.device = dev
        self.gpu = True
        self.Xh = X_host if X_host.is_contiguous() else X_host.contiguous()
        self.n, self.Dsrc = int(self.Xh.shape[0]), int(self.Xh.shape[1])
        self.D = int(n_features or self.Dsrc)
        self.dtype = dtype or self.Xh.dtype
        self.dt = native.dtype_code(self.dtype)
        self.Dp = padded_cols(self.Dsrc, 2 if self.dtype == torch.bfloat16 else 4)
        if native.dpad_for(self.Dp, self.dtype) == 0:
            raise NotImplementedError("streaming Lloyd supports D <= 1024 (the MFMA kernels' widest rows)")
        # async H2D straight from the caller's rows: page-lock them in place (no pinned copy)
        self._registered = False
        if self.n and not self.Xh.is_pinned():
            self._registered = bool(C.host_register(self.Xh))
        self.frozen = None
        if frozen is not None:
            self.frozen = torch.as_tensor(frozen, dtype=torch.uint8).reshape(-1).to(dev)
        self.weights = None
        if sample_weight is not None:
            self.weights = sample_weight.to(device=dev, dtype=torch.float32).contiguous()
            self._wscratch = torch.empty(C.WDOT_SCRATCH, dtype=torch.float64, device=dev)
        # chunks start on the 1536-row grid of the resident fit (csrc/assign16.hip seed offset)
        self.R = stream_chunk_rows(chunk_rows, self.n)
        self.ranges = [(r, min(r + self.R, self.n)) for r in range(0, self.n, self.R)]
        self.iteration = 0
        self.labels = torch.full((self.n,), -1, dtype=torch.int32, device=dev)
        self.C = torch.zeros((self.K, self.Dp), dtype=torch.float32, device=dev)
        self.Cnew = torch.zeros_like(self.C)
        self.shift = torch.zeros(self.K, dtype=torch.float32, device=dev)
        self.counts = torch.zeros(self.K, dtype=torch.float32, device=dev)
        self.mind = None
        if self.weights is not None or empty_policy == "farthest":
            self.mind = torch.empty(self.n, dtype=torch.float32, device=dev)
        self.pk = CentroidPack(self.K, self.Dp, self.dtype, dev)
        self.slots = torch.zeros(C.NSLOT * C.SLOT_STRIDE, dtype=torch.float64, device=dev)
        self.n_chunks = C.update_n_chunks(self.dt, self.K, self.Dp, self.R, self.weights is not None)
        KD = self.K * self.Dp
        self.slab = torch.empty(self.n_chunks * KD, dtype=torch.int64, device=dev)
        self.cnt_slab = torch.empty(self.n_chunks * self.K, dtype=torch.int64, device=dev)
        # compute buffers (zero padding columns stay zero) + staging for converted rows
        self.bufs = [torch.zeros((self.R, self.Dp), dtype=self.dtype, device=dev) for _ in range(2)]
        self.direct = self.Xh.dtype == self.dtype and self.Dsrc == self.Dp
        self.stage = None if self.direct else [torch.empty((self.R, self.Dsrc), dtype=self.Xh.dtype, device=dev)
                                               for _ in range(2)]
        self.copy_stream = torch.cuda.Stream(device=dev)
        self.ready = [torch.cuda.Event() for _ in range(2)]
        self.free = [torch.cuda.Event() for _ in range(2)]
        # one streaming pass: squared row norms (kept on the device; of the unit rows for the
        # cosine metric) and column statistics merged over chunks -> the fixed-point scales,
        # wide-range columns and the tol scale, all-reduced like the resident engine's
        self.xn = torch.empty(self.n, dtype=torch.float32, device=dev)
        st = ColStats.empty(self.Dp, dev)
        for Xc, r0, r1 in self._chunks():
            if r1 > r0:
                if fused_norms_ok(Xc):       # (one pass over the chunk: statistics + row norms)
                    st = st.merge(col_stats(Xc, xn=self.xn[r0:r1]))
                else:
                    C.row_sqnorm(Xc, self.xn[r0:r1])
                    st = st.merge(col_stats(Xc))
        self.stats = st
        self.scales = mstep_scales(self.bufs[0][:0], self.weights, comm=self.comm, stats=st)
        if self.scales.nw and C.update_slice_width(self.dt, self.K, self.Dp, self.weights is not None) == 0:
            self.scales = MStepScales(self.scales.col_exp, self.scales.cnt_exp, [], dev)
        self.col_exp, self.cnt_exp = self.scales.col_exp, self.scales.cnt_exp
        tail = self.K * self.scales.nw
        self.packed = torch.zeros(KD + self.K + 2 + tail, dtype=torch.float64, device=dev)
        self.part = torch.zeros_like(self.packed)        # one chunk's message

    def close(self):
        """Unpin the host rows (also on garbage collection)."""
        if getattr(self, "_registered", False):
            self._registered = False
            try:
                self._C.host_unregister(self.Xh)
            except Exception:  # noqa: BLE001 -- interpreter shutdown
                pass

    def __del__(self):
        self.close()

    # ------------------------------------------------------------ streaming
    def _upload(self, dst: torch.Tensor, src_rows: torch.Tensor, stage: torch.Tensor | None):
        """Host rows -> device compute rows (current stream): direct copy, or copy into the
        staging buffer and convert / pad on the device."""
        if stage is None:
            dst.copy_(src_rows, non_blocking=True)
        else:
            st = stage[: src_rows.shape[0]]
            st.copy_(src_rows, non_blocking=True)
            dst[:, : self.Dsrc].copy_(st)

    def _chunks(self):
        """Yield (device chunk, r0, r1) in order; chunk c+1's copy overlaps chunk c's use.
        The caller must finish enqueueing its work on chunk c before asking for c+1."""
        main = torch.cuda.current_stream(self.device)
        cp = self.copy_stream

        def issue(c):
            r0, r1 = self.ranges[c]
            s = c % 2
            cp.wait_event(self.free[s])                  # no kernel still reads this buffer
            with torch.cuda.stream(cp):
                Xc = self.bufs[s][: r1 - r0]
                self._upload(Xc, self.Xh[r0:r1], self.stage[s] if self.stage else None)
                if self.spherical:          # the resident fit's unit rows, same kernel
                    self._C.row_normalize(Xc)
            self.ready[s].record(cp)

        if not self.ranges:
            return
        # the copy stream starts behind everything the caller's stream has queued: the chunk
        # buffers' zero fill at construction (a copy racing ahead of it was overwritten by
        # zeros: wrong row norms / column statistics for chunk 0, a load-dependent race) and
        # whatever last touched them
        cp.wait_stream(main)
        issue(0)
        for c, (r0, r1) in enumerate(self.ranges):
            if c + 1 < len(self.ranges):
                issue(c + 1)
            s = c % 2
            main.wait_event(self.ready[s])
            yield self.bufs[s][: r1 - r0], r0, r1
            self.free[s].record(main)

    def _pre_collective(self):
        """The chunk loop: assign + M-step + reduce of every chunk into one message (the
        collective, wide-column lo sums, relocation and finalize are the resident engine's)."""
        C = self._C
        KD = self.K * self.Dp
        sc = self.scales
        self.packed.zero_()
        for Xc, r0, r1 in self._chunks():
            lab = self.labels[r0:r1]
            mind = self.mind[r0:r1] if self.mind is not None else None
            w = self.weights[r0:r1] if self.weights is not None else None
            self.pk.assign(Xc, self.xn[r0:r1], lab, mind, self.slots, True)
            C.update(Xc, lab, self.K, self.slab, self.cnt_slab, self.n_chunks, w, self.col_exp,
                     self.cnt_exp, False)
            C.reduce(self.slab, self.cnt_slab, self.n_chunks, self.K, self.Dp, self.slots, self.part,
                     self.col_exp, self.cnt_exp)
            if sc.nw:   # residual (lo) pass of the wide-range columns into the message tail
                C.update(Xc, lab, self.K, self.slab, self.cnt_slab, self.n_chunks, w, self.col_exp,
                         self.cnt_exp, False, col_exp2=sc.col_exp2)
                C.reduce_cols(self.slab, self.n_chunks, self.K, self.Dp, sc.wide_cols, sc.wide_exps,
                              self.part[KD + self.K + 2:])
            self.packed += self.part
        if self.weights is not None and self.n:
            self._weighted_inertia()

    def capture(self):
        self.capture_error = "streamed fit: a host-driven chunk loop (not captured)"
        return self

    def _assign_into(self, mind):
        for Xc, r0, r1 in self._chunks():
            lab = torch.empty(r1 - r0, dtype=torch.int32, device=self.device)
            self.pk.assign(Xc, self.xn[r0:r1], lab, mind[r0:r1])

    def assign(self, with_dist: bool = True):
        """Labels (and squared distances) of every row under the current centres."""
        labels = torch.empty_like(self.labels)
        mind = torch.empty(self.n, dtype=torch.float32, device=self.device) if with_dist else None
        for Xc, r0, r1 in self._chunks():
            self.pk.assign(Xc, self.xn[r0:r1], labels[r0:r1], mind[r0:r1] if with_dist else None)
        return labels, mind

    # -------------------------------------------------------------- host rows
    def fetch_rows(self, idx) -> torch.Tensor:
        """Local rows ``idx`` as the device sees them (compute dtype, padded, unit rows for
        the cosine metric): ``[m, Dp]`` on the device."""
        idx = torch.as_tensor(idx, dtype=torch.int64).cpu()
        rows = torch.zeros((idx.numel(), self.Dp), dtype=self.dtype, device=self.device)
        if idx.numel():
            rows[:, : self.Dsrc].copy_(self.Xh[idx].to(self.device))
            if self.spherical:
                self._C.row_normalize(rows)
        return rows

    def _rows(self, idx: torch.Tensor) -> torch.Tensor:
        return self.fetch_rows(idx).double()

    def sample_rows(self, m: int, seed: int) -> torch.Tensor:
        """``m`` distinct local rows (seeded, in row order) as a device tensor."""
        g = torch.Generator().manual_seed(int(seed))
        idx = torch.randperm(self.n, generator=g)[: min(m, self.n)].sort().values
        return self.fetch_rows(idx)
