"""Out-of-core Lloyd: the points stay in pinned host memory and stream through the GPU.

For shards larger than one GPU's HBM (N=1e9 x D=256 bf16 is 512 GB
against 288 GB per MI355X) every Lloyd iteration streams the rank's rows through two
device chunk buffers.  The host->device copy of chunk c+1 runs on a copy stream while
the compute stream assigns chunk c on the matrix cores and scatters it into the
fixed-point M-step slab; chunk c's integer partial sums are folded into one f64 message
(exact: integer multiples of 2^-e below 2^53), so the iteration still ends with ONE
all-reduce and the same finalize as the device-resident engine.  Labels (4 B/row) and
squared row norms (4 B/row) stay on the device for all rows.

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
    """LloydEngine over a host-resident shard ``X_host`` ([n, D], CPU), streamed in
    ``chunk_rows`` pieces.  Same public surface as :class:`LloydEngine` (``step``, ``run``,
    ``last_stats``, ``assign``, ``centers``, ``counts``); GPU only, unweighted, empty
    policy 'keep', full M-step every iteration."""

    def __init__(self, X_host: torch.Tensor, n_clusters: int, *, chunk_rows: int = 1 << 22,
                 comm: Comm | None = None, device=None, frozen=None, n_features: int | None = None):
        from ..ops import CentroidPack, fixed_exps, pad_columns

        if X_host.device.type != "cpu":
            raise ValueError("StreamingLloydEngine streams a host (CPU) tensor")
        self.comm = comm or Comm.local(device or "cuda")
        dev = torch.device(device) if device is not None else self.comm.device
        if dev.type != "cuda":
            raise ValueError("StreamingLloydEngine needs a GPU device")
        C = native.require()
        self._C = C
        self.incremental = False
        self.spherical = False
        self.delta = None
        self.segments = 1
        self.hint = False
        self.weights = None
        self.mind = None
        self.empty_policy = "keep"
        self.K = int(n_clusters)
        self.D = int(n_features or X_host.shape[1])
        self.device = dev
        self.gpu = True
        Xh = pad_columns(X_host.contiguous())            # 16-byte rows, as on the device
        if not Xh.is_pinned():
            Xh = Xh.pin_memory()                         # async H2D needs page-locked rows
        self.Xh = Xh
        self.n = int(Xh.shape[0])
        self.Dp = int(Xh.shape[1])
        self.dtype = Xh.dtype
        self.dt = native.dtype_code(self.dtype)
        if native.dpad_for(self.Dp, self.dtype) == 0:
            raise NotImplementedError("streaming Lloyd supports D <= 256")
        self.frozen = None
        if frozen is not None:
            self.frozen = torch.as_tensor(frozen, dtype=torch.uint8).reshape(-1).to(dev)
        # chunks start on the 256-row grid of the resident fit (csrc/assign16.hip seed offset)
        from ..parallel.shard import ROW_ALIGN

        self.R = max(1, min(-(-int(chunk_rows) // ROW_ALIGN) * ROW_ALIGN, max(self.n, 1)))
        self.ranges = [(r, min(r + self.R, self.n)) for r in range(0, self.n, self.R)]
        self.iteration = 0
        self.labels = torch.full((self.n,), -1, dtype=torch.int32, device=dev)
        self.C = torch.zeros((self.K, self.Dp), dtype=torch.float32, device=dev)
        self.Cnew = torch.zeros_like(self.C)
        self.shift = torch.zeros(self.K, dtype=torch.float32, device=dev)
        self.counts = torch.zeros(self.K, dtype=torch.float32, device=dev)
        KD = self.K * self.Dp
        self.packed = torch.zeros(KD + self.K + 2, dtype=torch.float64, device=dev)
        self.part = torch.zeros_like(self.packed)        # one chunk's message
        self.pk = CentroidPack(self.K, self.Dp, self.dtype, dev)
        self.slots = torch.zeros(C.NSLOT * C.SLOT_STRIDE, dtype=torch.float64, device=dev)
        self.n_chunks = C.update_n_chunks(self.dt, self.K, self.Dp, self.R, False)
        self.slab = torch.empty(self.n_chunks * KD, dtype=torch.int64, device=dev)
        self.cnt_slab = torch.empty(self.n_chunks * self.K, dtype=torch.int64, device=dev)
        self.bufs = [torch.empty((self.R, self.Dp), dtype=self.dtype, device=dev) for _ in range(2)]
        self.copy_stream = torch.cuda.Stream(device=dev)
        self.ready = [torch.cuda.Event() for _ in range(2)]
        self.free = [torch.cuda.Event() for _ in range(2)]
        # one streaming pass: squared row norms (kept on the device) + column maxima for
        # the fixed-point scales (all-reduced: every rank accumulates on the same grid)
        self.xn = torch.empty(self.n, dtype=torch.float32, device=dev)
        cmax = torch.zeros(self.Dp, dtype=torch.float64, device=dev)
        for Xc, r0, r1 in self._chunks():
            if r1 > r0:
                C.row_sqnorm(Xc, self.xn[r0:r1])
                cmax = torch.maximum(cmax, Xc.abs().amax(0).to(torch.float64))
        self.col_exp, self.cnt_exp = fixed_exps(self.bufs[0][:1], None, comm=self.comm, bound=cmax)

    # ------------------------------------------------------------ streaming
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
                self.bufs[s][: r1 - r0].copy_(self.Xh[r0:r1], non_blocking=True)
            self.ready[s].record(cp)

        if not self.ranges:
            return
        issue(0)
        for c, (r0, r1) in enumerate(self.ranges):
            if c + 1 < len(self.ranges):
                issue(c + 1)
            s = c % 2
            main.wait_event(self.ready[s])
            yield self.bufs[s][: r1 - r0], r0, r1
            self.free[s].record(main)

    def _step_gpu(self):
        C = self._C
        self.packed.zero_()
        for Xc, r0, r1 in self._chunks():
            lab = self.labels[r0:r1]
            self.pk.assign(Xc, self.xn[r0:r1], lab, None, self.slots, True)
            C.update(Xc, lab, self.K, self.slab, self.cnt_slab, self.n_chunks, None, self.col_exp,
                     self.cnt_exp, False)
            C.reduce(self.slab, self.cnt_slab, self.n_chunks, self.K, self.Dp, self.slots, self.part,
                     self.col_exp, self.cnt_exp)
            self.packed += self.part
        self.comm.allreduce_(self.packed)
        self.pk.finalize(1, self.packed, self.C, self.Cnew, self.frozen, None, self.shift, self.counts)

    def capture(self):
        return self  # a host-driven chunk loop: nothing to capture as one graph

    def assign(self, with_dist: bool = True):
        """Labels (and squared distances) of every row under the current centres."""
        labels = torch.empty_like(self.labels)
        mind = torch.empty(self.n, dtype=torch.float32, device=self.device) if with_dist else None
        for Xc, r0, r1 in self._chunks():
            self.pk.assign(Xc, self.xn[r0:r1], labels[r0:r1], mind[r0:r1] if with_dist else None)
        return labels, mind

    def sample_rows(self, m: int, seed: int) -> torch.Tensor:
        """``m`` distinct local rows (host gather, then one copy) as a device tensor."""
        g = torch.Generator().manual_seed(int(seed))
        idx = torch.randperm(self.n, generator=g)[: min(m, self.n)].sort().values
        return self.Xh[idx].to(self.device)
