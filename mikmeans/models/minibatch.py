"""Mini-batch k-means (Sculley 2010) for datasets that do not fit in HBM.

BASELINE config 5 (N=1e9, D=256, K=512) is 512 GB of bf16: more than one
MI355X's 288 GB.  Each step takes a batch (a tensor slice, a random sample, or a
device-generated :class:`~mikmeans.data.blobs.BlobStream` batch), runs the same
K2 assign and K3 update kernels as Lloyd, all-reduces the per-batch sums/counts
(C5), and applies the per-centre running-mean update in the K4 finalize kernel:

    v_k <- v_k + b_k ;  c_k <- c_k + (s_k - b_k c_k) / v_k

where b_k / s_k are the batch count / sum of centre k and v_k the running count.
"""
from __future__ import annotations

import torch

from ..ops import cpu as cpu_ops
from ..ops import native, pad_columns
from ..parallel.comm import Comm


class MiniBatchEngine:
    def __init__(self, n_clusters: int, D: int, batch_size: int, *, dtype=torch.float32,
                 device="cpu", comm: Comm | None = None, frozen=None,
                 value_bound: float | None = None):
        self.comm = comm or Comm.local(device)
        self.K, self.D = int(n_clusters), int(D)
        self.device = torch.device(device)
        self.gpu = self.device.type == "cuda"
        self.dtype = dtype
        v = native.vec_elems(dtype)
        self.Dp = (self.D + v - 1) // v * v if self.gpu else self.D
        self.batch = int(batch_size)
        self.C = torch.zeros((self.K, self.Dp), dtype=torch.float32, device=self.device)
        self.Cnew = torch.zeros_like(self.C)
        self.vcount = torch.zeros(self.K, dtype=torch.float64, device=self.device)
        self.shift = torch.zeros(self.K, dtype=torch.float32, device=self.device)
        self.counts = torch.zeros(self.K, dtype=torch.float32, device=self.device)
        # [K*D sums | K counts | inertia | changed | clamped-workgroup count]
        self.packed = torch.zeros(self.K * self.Dp + self.K + 3, dtype=torch.float64, device=self.device)
        self.frozen = None
        if frozen is not None:
            self.frozen = torch.as_tensor(frozen, dtype=torch.uint8).reshape(-1).to(self.device)
        self.steps = 0
        self.batch_inertia = 0.0
        # optional host callback between a step's assign and its M-step (enqueue time), e.g.
        # a prefetching BlobStream's kick(): the next batch's generator then overlaps the
        # memory-bound M-step rather than the matrix-core assign
        self.after_assign = None
        if self.gpu and native.dpad_for(self.Dp, dtype) == 0:
            native.warn_once(f"D={self.D} > 1024: mini-batch steps use the PyTorch GEMM path")
            self.gpu = False
        if self.gpu:
            C = native.require()
            self._C = C
            self.dt = native.dtype_code(dtype)
            from ..ops import CentroidPack

            dev = self.device
            self.pk = CentroidPack(self.K, self.Dp, dtype, dev)
            self.slots = torch.zeros(C.NSLOT * C.SLOT_STRIDE, dtype=torch.float64, device=dev)
            self.n_chunks = C.update_n_chunks(self.dt, self.K, self.Dp, self.batch)
            self.slab = torch.empty(self.n_chunks * self.K * self.Dp, dtype=torch.int64, device=dev)
            self.cnt_slab = torch.empty(self.n_chunks * self.K, dtype=torch.int64, device=dev)
            # fixed-point scales: from the first batch (x8 headroom) or the given value bound; a
            # later batch beyond them is detected on device (clamp count) and redone with scales
            # grown from its own column maxima -- never saturated silently
            self.col_exp = None
            self.bound = None    # per-column |x| bound [D] f64 the scales were made for
            self.rescales = 0    # batches redone with a wider scale
            self.value_bound = value_bound
            self.bounded = value_bound is not None   # scales cover every value: no clamp, no sync
            self.clampc = torch.zeros(1, dtype=torch.int32, device=dev)
            self.labels = torch.empty(self.batch, dtype=torch.int32, device=dev)

    def set_centers(self, centers: torch.Tensor, counts=None):
        self.C.zero_()
        self.C[:, : self.D] = centers.to(device=self.device, dtype=torch.float32)
        self.vcount.zero_()
        if counts is not None:
            self.vcount.copy_(torch.as_tensor(counts, dtype=torch.float64))
        if self.gpu:
            self.pk.finalize(0, None, self.C)

    @property
    def centers(self):
        return self.C[:, : self.D]

    def device_buffers(self) -> dict:
        """Allocator bytes of every device buffer the engine holds, under the names
        parallel/memplan.py ``plan_minibatch`` plans them by (tests/test_gpu_memplan.py)."""
        from ..parallel.memplan import _r

        if not self.gpu:
            return {}
        t = {"C": self.C, "Cnew": self.Cnew, "vcount": self.vcount, "shift": self.shift, "counts": self.counts,
             "packed": self.packed, "pack": self.pk.pack, "cn": self.pk.cn, "slots": self.slots,
             "slab": self.slab, "cnt_slab": self.cnt_slab, "batch_labels": self.labels, "clampc": self.clampc}
        if self.pk._keys is not None:
            t["split_keys"] = self.pk._keys
        return {k: _r(v.numel() * v.element_size()) for k, v in t.items()}

    def partial_fit(self, Xb: torch.Tensor, norms: torch.Tensor | None = None):
        """One mini-batch step on this rank's batch ``Xb`` (may be empty).  ``norms``
        (optional, f32 [rows], e.g. a BlobStream's fused norms): the GPU assign then takes the
        rows' |x|^2 from them (key offsets, batch inertia) and can start its matrix-core work
        while the row fragments are still in flight (the early prologue); without them it
        computes |x|^2 from the fragments -- as :meth:`partial_fit_rows` does, bit for bit."""
        if self.gpu:
            self._step_gpu(Xb, norms)
        else:
            self._step_cpu(Xb)
        self.C, self.Cnew = self.Cnew, self.C
        self.steps += 1

    # ------------------------------------------------------------ persistence
    def state_tensors(self) -> dict:
        """Everything beyond the centres a resumed stream needs to continue bit for bit."""
        t = {"vcount": self.vcount.double().cpu()}
        if self.gpu and self.bound is not None:
            t["col_bound"] = self.bound.double().cpu()
        return t

    def load_state(self, centers: torch.Tensor, tensors: dict, steps: int, rescales: int = 0):
        self.set_centers(centers)
        self.vcount.copy_(tensors["vcount"].to(device=self.device, dtype=torch.float64))
        self.steps = int(steps)
        if self.gpu:
            self.rescales = int(rescales)
            if "col_bound" in tensors and self.value_bound is None:
                from ..ops import fixed_exps

                self.bound = tensors["col_bound"].to(device=self.device, dtype=torch.float64)
                self.col_exp, _ = fixed_exps(torch.empty((0, self.Dp), dtype=self.dtype, device=self.device),
                                             None, comm=self.comm, bound=self.bound)
        return self

    def set_bound(self, bound: torch.Tensor):
        """Fix the fixed-point scales from a per-column bound on |x| over the WHOLE dataset
        (f64 ``[D]`` or ``[Dp]``; all-reduced MAX over ranks): no batch can exceed it, so
        the M-step runs unclamped and no step reads anything back to the host."""
        from ..ops import fixed_exps

        if not self.gpu:
            return self
        b = torch.zeros(self.Dp, dtype=torch.float64, device=self.device)
        bd = bound.to(device=self.device, dtype=torch.float64).reshape(-1)
        b[: bd.numel()] = bd[: self.Dp]
        self.col_exp, _ = fixed_exps(torch.empty((0, self.Dp), dtype=self.dtype, device=self.device), None,
                                     comm=self.comm, bound=b)
        self.bound = b
        self.bounded = True
        return self

    def _set_bound(self, Xb, grow: bool = False):
        from ..ops import col_max_abs, fixed_exps

        if self.value_bound is not None:
            bound = torch.full((self.Dp,), float(self.value_bound), dtype=torch.float64, device=self.device)
        else:
            # all-zero columns get the finest scale; a later nonzero value there is a clamp -> regrow
            bound = 8.0 * col_max_abs(Xb).clamp_min(1e-30)
            if grow and self.bound is not None:
                bound = torch.maximum(bound, self.bound)
        self.col_exp, _ = fixed_exps(Xb, None, comm=self.comm, bound=bound)   # bound all-reduced (MAX)
        self.bound = bound

    def _mstep(self, Xb, lab, rows=None):
        C = self._C
        KD = self.K * self.Dp
        if (rows.numel() if rows is not None else Xb.shape[0]):
            # a given value bound cannot be exceeded: no clamp, no count (the plain kernel)
            bounded = self.bounded
            C.update(Xb, lab, self.K, self.slab, self.cnt_slab, self.n_chunks, None, self.col_exp, 0,
                     not bounded, clamp_count=None if bounded else self.clampc, rows=rows)
            C.reduce(self.slab, self.cnt_slab, self.n_chunks, self.K, self.Dp, self.slots, self.packed,
                     self.col_exp, 0)
            self.packed[KD + self.K + 2] = self.clampc[0].double()
            self.clampc.zero_()
        else:
            self.packed.zero_()
        self.comm.allreduce_(self.packed)

    def partial_fit_rows(self, X: torch.Tensor, rows: torch.Tensor):
        """One step on the batch ``X[rows]`` without materialising it: the assign and the
        M-step read the sampled rows of the (device-resident, column-padded) shard through
        the index list (csrc/assign16.hip, csrc/update.hip ``rows``).  Needs fixed scales
        (:meth:`set_bound`); the same centres as :meth:`partial_fit` on the gathered batch."""
        if not self.gpu:
            self.partial_fit(X[rows.to(X.device)] if rows.numel() else X[:0])
            return
        if not self.bounded:
            raise RuntimeError("partial_fit_rows needs fixed scales: call set_bound() first")
        b = rows.numel()
        if b > self.batch:
            raise ValueError(f"batch of {b} rows exceeds the engine's batch_size {self.batch}")
        Xp = pad_columns(X, self.dtype)
        lab = self.labels[:b]
        if b:
            self.pk.assign(Xp, None, lab, None, self.slots, False, rows=rows)
        if self.after_assign is not None:
            self.after_assign()
        self._mstep(Xp, lab, rows)
        self.pk.finalize(2, self.packed, self.C, self.Cnew, self.frozen, self.vcount, self.shift, self.counts)
        self.C, self.Cnew = self.Cnew, self.C
        self.steps += 1

    def _step_gpu(self, Xb, norms=None):
        C = self._C
        Xb = pad_columns(Xb.to(self.device), self.dtype)
        b = Xb.shape[0]
        if b > self.batch:
            raise ValueError(f"batch of {b} rows exceeds the engine's batch_size {self.batch}")
        if self.col_exp is None:
            self._set_bound(Xb)
        lab = self.labels[:b]
        if b:
            # key offsets and the inertia from the caller's norms when given, else from the row
            # fragments (as the gathered-row path, partial_fit_rows, computes them)
            xn = None
            if norms is not None and norms.is_cuda and norms.numel() >= b and norms.dtype == torch.float32:
                xn = norms[:b]
            self.pk.assign(Xb, xn, lab, None, self.slots, False)
        if self.after_assign is not None:
            self.after_assign()
        self._mstep(Xb, lab)
        if not self.bounded:
            # one host read per step: the all-reduced clamp count is the same on every rank,
            # so all ranks agree to redo this batch with scales grown from its maxima
            KD = self.K * self.Dp
            if float(self.packed[KD + self.K + 2].item()) > 0:
                inertia = self.packed[KD + self.K].clone()
                self.rescales += 1
                self._set_bound(Xb, grow=True)
                self._mstep(Xb, lab)
                self.packed[KD + self.K] = inertia   # the assign's slots were consumed by the first reduce
                if float(self.packed[KD + self.K + 2].item()) > 0:
                    raise RuntimeError("mini-batch M-step still saturates after rescaling (non-finite data?)")
        self.pk.finalize(2, self.packed, self.C, self.Cnew, self.frozen, self.vcount, self.shift,
                         self.counts)

    def _step_cpu(self, Xb):
        K, Dp = self.K, self.Dp
        KD = K * Dp
        Xb = Xb.to(self.device)
        if Xb.shape[0]:
            lab, mind = cpu_ops.assign(Xb, self.C)
            sums, counts = cpu_ops.cluster_sums(Xb, lab, K)
            self.packed[:KD] = sums.reshape(-1)
            self.packed[KD : KD + K] = counts
            self.packed[KD + K] = mind.double().sum()
            self.packed[KD + K + 1] = 0
        else:
            self.packed.zero_()
        self.comm.allreduce_(self.packed)
        s = self.packed[:KD].view(K, Dp)
        b = self.packed[KD : KD + K]
        upd = b > 0
        if self.frozen is not None:
            upd &= self.frozen == 0
        vnew = self.vcount + b
        new = torch.where(upd[:, None],
                          ((self.vcount / vnew.clamp_min(1e-300))[:, None] * self.C.double()
                           + s / vnew.clamp_min(1e-300)[:, None]).to(torch.float32), self.C)
        self.vcount = torch.where(upd, vnew, self.vcount)
        self.Cnew.copy_(new)
        self.shift.copy_(((new - self.C) ** 2).sum(1))
        self.counts.copy_(b.to(torch.float32))

    def last_batch_inertia(self) -> float:
        return float(self.packed[self.K * self.Dp + self.K].item())
