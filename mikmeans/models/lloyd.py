"""Lloyd's algorithm engine: one bulk-synchronous iteration = 4 kernels + 1 collective.

Per iteration on every rank:

  K2 assign    labels, inertia/changed partials   (MFMA GEMM + online argmin)
  K3 update    per-chunk slab of sums / counts    (LDS-privatised scatter-add)
     reduce    slabs -> packed f64 message [K*D sums | K counts | inertia | changed]
  C1 all-reduce(packed)                           (RCCL over xGMI, ~516 KiB at K=1024, D=128)
  K4 finalize  C_new, per-centre shift, re-pack   (frozen / empty-cluster policy)

Everything is stream-ordered with no host synchronisation; the host reads the
tiny stats only when a convergence check is due (``check_every``).

The CPU backend runs the same stages with the PyTorch reference ops (gloo for
multi-process), so the distributed logic is identical and testable without a GPU.

Reference parity: the reference's "iteration" is a manual counter whose change
snapshots the dashboard metrics (app.mjs:288, :498-508); here the iteration
counter advances per Lloyd step and every step yields the same metric record
(counts, balance) plus inertia / shift / changed labels.
"""
from __future__ import annotations

import contextlib
import math
import os
from dataclasses import dataclass, field

import torch

from ..ops import cpu as cpu_ops
from ..ops import native
from ..parallel.comm import Comm
from ..utils import profiling

# roctx ranges around each phase (rocprofv3 --marker-trace); off by default: a range
# push/pop is a host call per phase per iteration.
_TRACE = os.environ.get("MIKMEANS_ROCTX", "0") not in ("", "0")


def _phase(name: str):
    return profiling.range(name) if _TRACE else contextlib.nullcontext()


@dataclass
class IterStats:
    iteration: int
    inertia: float          # of the assignment made with the centres *before* this update
    n_changed: int
    shift: float            # sum_k |c_k' - c_k|^2
    max_shift: float
    counts: list = field(default_factory=list)

    def as_dict(self):
        return {
            "iter": self.iteration,
            "inertia": self.inertia,
            "n_changed": self.n_changed,
            "shift": self.shift,
            "max_shift": self.max_shift,
        }


class LloydEngine:
    """Device-resident Lloyd state for one rank's shard of points.

    ``X`` is this rank's shard (``[n, D]``, float32 or bfloat16, any device);
    centroids are replicated and kept in float32.  After ``set_centers`` the
    engine is driven by :meth:`step` / :meth:`run`.
    """

    def __init__(self, X: torch.Tensor, n_clusters: int, *, comm: Comm | None = None,
                 sample_weight: torch.Tensor | None = None, frozen=None,
                 empty_policy: str = "keep", n_features: int | None = None, segments: int = 1,
                 overlap_sw: int = 8, incremental: bool = False, delta_cap: float = 0.125,
                 spherical: bool = False, bounded: bool = False, tighten: bool = False):
        from ..ops import pad_columns

        # Bounded E-step (Hamerly 2010): per-point bounds on the distance to the assigned
        # centre (ub) and to the second nearest (lb), moved by each M-step's centre shifts;
        # only points whose bounds no longer prove their label are re-assigned (a gathered
        # assign over them).  Bitwise the full E-step's iterates: a re-assigned row is seeded
        # with the offset the full pass gives it (``oseed``) and ranked by the same epilogue,
        # and a row is skipped only where the full pass's keys provably keep its label
        # (csrc/rows.hip keys_keep_label).  The step's inertia comes from the M-step's sums.
        self.bounded = bool(bounded)
        # Hamerly's tightening (exact distance to the label's centre before the full assign):
        # off by default -- here the candidates come from the falling lower bounds, so it
        # cleared few rows per step and deferred others until their stale lower bounds fell
        # (N=2e7 K=1024: 0.90 vs 0.66 ms per settled step, profiles/r4_10_hamerly_tighten_ab.md)
        self.tighten = bool(tighten)
        # Incremental M-step: keep per-rank integer running totals of the cluster sums and
        # re-scatter only the rows whose label changed (+ to the new label, - from the old).
        # Bitwise identical to the full M-step (integer fixed point); the full pass runs
        # automatically while more than ``delta_cap * n`` rows change.
        self.incremental = bool(incremental)
        self.delta_cap = float(delta_cap)
        # spherical k-means (cosine metric on unit-norm rows): every M-step's centres are
        # projected back onto the unit sphere and re-packed for the next E-step
        self.spherical = bool(spherical)
        self.segments = max(1, int(segments))
        self.overlap_sw = overlap_sw
        self.comm = comm or Comm.local(X.device)
        self.K = int(n_clusters)
        self.D = int(n_features or X.shape[1])   # real features (X may be column-padded)
        self.device = X.device
        self.gpu = X.device.type == "cuda"
        self.X = pad_columns(X) if self.gpu else X
        self.Dp = int(self.X.shape[1])
        if self.gpu and native.dpad_for(self.Dp, self.X.dtype) == 0:
            # D > 1024: wider than the MFMA kernels' register-resident rows (csrc/assign16.hip
            # covers up to 1024 features); the PyTorch path runs on the device instead
            native.warn_once(f"D={self.D} > 1024: Lloyd steps use the PyTorch GEMM path on {X.device}")
            self.gpu = False
        self.n = int(self.X.shape[0])
        self.dtype = self.X.dtype
        self.empty_policy = empty_policy
        self.weights = None
        if sample_weight is not None:
            self.weights = sample_weight.to(device=self.device, dtype=torch.float32).contiguous()
        self.frozen = None
        if frozen is not None:
            fz = torch.as_tensor(frozen, dtype=torch.uint8).reshape(-1)
            if fz.numel() != self.K:
                raise ValueError("frozen mask must have n_clusters entries")
            self.frozen = fz.to(self.device)
        self.iteration = 0
        self.labels = torch.full((self.n,), -1, dtype=torch.int32, device=self.device)
        self.C = torch.zeros((self.K, self.Dp), dtype=torch.float32, device=self.device)
        self.Cnew = torch.zeros_like(self.C)
        self.shift = torch.zeros(self.K, dtype=torch.float32, device=self.device)
        self.counts = torch.zeros(self.K, dtype=torch.float32, device=self.device)
        self.packed = torch.zeros(self.K * self.Dp + self.K + 2, dtype=torch.float64, device=self.device)
        self.mind = None
        if self.gpu:
            self._init_gpu()
        else:
            self.xn = cpu_ops.row_sqnorm(self.X)
            self.bounded = False          # (the CPU path assigns every row each step)

    # ------------------------------------------------------------------ setup
    def _init_gpu(self):
        from ..ops import CentroidPack

        C = native.require()
        self._C = C
        self.dt = native.dtype_code(self.dtype)
        dev = self.device
        self.pk = CentroidPack(self.K, self.Dp, self.dtype, dev)
        self.slots = torch.zeros(C.NSLOT * C.SLOT_STRIDE, dtype=torch.float64, device=dev)
        from ..parallel.shard import shard_range

        # Overlapped M-step: segment s is scattered on a side stream while the matrix
        # cores assign segment s+1.  Narrow slices keep the update's LDS small enough to
        # share a CU with assign workgroups.  Segments fall on the 1536-row grid, so a
        # small shard leaves some empty: they are dropped (the reduce would otherwise sum
        # their never-written slab chunks).
        segs = [sr for sr in (shard_range(self.n, s, self.segments) for s in range(self.segments))
                if sr[1] > sr[0]] if self.segments > 1 else []
        if len(segs) > 1:
            self.seg_ranges = segs
            self.segments = len(segs)
            C.set_update_max_sw(self.overlap_sw)
            seg_rows = max(e - s for s, e in self.seg_ranges)
            self.seg_chunks = C.update_n_chunks(self.dt, self.K, self.Dp, seg_rows, self.weights is not None)
            C.set_update_max_sw(0)
            self.n_chunks = self.seg_chunks * self.segments
            self.side = torch.cuda.Stream(device=dev)
            self.seg_events = [torch.cuda.Event() for _ in range(self.segments)]
            self.side_done = torch.cuda.Event()
        else:
            self.segments = 1
            self.n_chunks = C.update_n_chunks(self.dt, self.K, self.Dp, max(self.n, 1),
                                              self.weights is not None or self.incremental)
        self.slab = torch.empty(self.n_chunks * self.K * self.Dp, dtype=torch.int64, device=dev)
        self.cnt_slab = torch.empty(self.n_chunks * self.K, dtype=torch.int64, device=dev)
        self.xn = torch.empty(self.n, dtype=torch.float32, device=dev)
        # fixed-point scale of the M-step accumulators (X is static for the fit)
        from ..ops import MStepScales, col_stats, fused_norms_ok, mstep_scales

        # (global column statistics: every rank uses the same scale -> exact, world-size independent
        # sums; columns with inexact values far above their nonzero mean also get a residual lo pass)
        # One pass over X: the statistics and, rows of <= 64 pieces, the row norms with them
        fused = bool(self.n) and fused_norms_ok(self.X)
        if self.n and not fused:
            C.row_sqnorm(self.X, self.xn)
        self.stats = col_stats(self.X, xn=self.xn if fused else None)   # (also the tol scale's sums: api.fit)
        self.scales = mstep_scales(self.X, self.weights, comm=self.comm, stats=self.stats)
        if self.scales.nw and C.update_slice_width(self.dt, self.K, self.Dp, self.weights is not None) == 0:
            self.scales = MStepScales(self.scales.col_exp, self.scales.cnt_exp, [], dev)
        self.col_exp, self.cnt_exp = self.scales.col_exp, self.scales.cnt_exp
        if self.scales.nw:
            # message tail: the wide columns' lo sums [K, nw], added onto the hi sums after the all-reduce
            self.packed = torch.zeros(self.K * self.Dp + self.K + 2 + self.K * self.scales.nw,
                                      dtype=torch.float64, device=dev)
        if self.weights is not None or self.empty_policy == "farthest":
            # per-row distances written by every step's assign: the weighted inertia and the
            # 'farthest' relocation read them (no second assign pass for either)
            self.mind = torch.empty(self.n, dtype=torch.float32, device=dev)
        if self.weights is not None:
            self._wscratch = torch.empty(C.WDOT_SCRATCH, dtype=torch.float64, device=dev)
        if self.bounded and self.segments > 1:
            native.warn_once("bounded E-step: not with segment overlap; full E-steps")
            self.bounded = False
        if self.bounded:
            # per-row bounds (f32), the rows to re-assign (flags, then their compacted indices
            # and count -- on the device, so the step stays sync-free and capturable)
            self.ub = torch.empty(self.n, dtype=torch.float32, device=dev)
            self.lb = torch.empty(self.n, dtype=torch.float32, device=dev)
            self.cand = torch.empty(self.n, dtype=torch.uint8, device=dev)
            self._brows = torch.empty(self.n, dtype=torch.int64, device=dev)
            self._bcount = torch.zeros(1, dtype=torch.int64, device=dev)
            self._bscratch = torch.empty(max(1, C.compact_blocks(self.n)), dtype=torch.int64, device=dev)
            self._bwork = torch.empty(4, dtype=torch.float32, device=dev)
            # the bounds are distances to the centres the assign ranks (bf16-rounded for bf16
            # points), moved by those centres' own shifts: finalize writes them beside the f32 ones
            self.qshift = torch.zeros(self.K, dtype=torch.float32, device=dev)
            # X is static for the fit: every row's full-pass seed offset, once (bf16 keys)
            self.oseed = self.pk.seed_offsets(self.xn) if self.n else None
            # sum_i w_i |x_i|^2 over all ranks (f64): with the M-step's sums S_k and counts n_k the
            # step's inertia is sxx + sum_k (n_k |c_k|^2 - 2 c_k . S_k), no per-row distances
            sxx = torch.zeros(1, dtype=torch.float64, device=dev)
            if self.n and self.weights is None:
                sxx += self.stats.sumsq[: self.Dp].to(device=dev, dtype=torch.float64).sum()
            elif self.n:
                C.wdot(self.xn, self.weights, sxx, self._wscratch)
            self.comm.allreduce_(sxx)
            self._sxx = sxx
            self._invalidate_bounds()
        self.delta = None
        if self.incremental:
            if self.scales.nw:
                native.warn_once(f"{self.scales.nw} wide-range column(s): residual M-step pass, full passes "
                                 "instead of the incremental M-step")
            elif self.segments > 1 or self.n >= 2**31 or C.update_slice_width(self.dt, self.K, self.Dp, True) == 0:
                native.warn_once("incremental M-step unavailable for this shape/overlap mode; using full passes")
            else:
                cap = max(1, min(self.n, int(self.n * self.delta_cap)))
                self.delta = {
                    # labels the running totals correspond to (-1: none yet -> first pass is full)
                    "prev": torch.full((self.n,), -1, dtype=torch.int32, device=dev),
                    "list": torch.empty((cap, 2), dtype=torch.int32, device=dev),
                    "count": torch.zeros(1, dtype=torch.int32, device=dev),
                    "tot": torch.zeros(self.K * self.Dp + self.K, dtype=torch.int64, device=dev),
                }
                if self.n == 0:
                    self.delta = None

    def device_buffers(self) -> dict:
        """Allocator bytes of every device buffer the engine holds, under the names
        parallel/memplan.py plans them by (tests/test_memplan_gpu.py pins the two)."""
        from ..parallel.memplan import _r

        t = {"labels": self.labels, "xn": self.xn, "slab": self.slab, "cnt_slab": self.cnt_slab,
             "packed": self.packed, "C": self.C, "Cnew": self.Cnew, "shift": self.shift,
             "counts": self.counts, "pack": self.pk.pack, "cn": self.pk.cn, "slots": self.slots}
        if self.weights is not None:
            t["weights"] = self.weights
            t["wdot_scratch"] = self._wscratch
        if self.mind is not None:
            t["mind"] = self.mind
        if self.pk._keys is not None:
            t["split_keys"] = self.pk._keys
        if self.delta is not None:
            t.update(delta_prev=self.delta["prev"], delta_list=self.delta["list"],
                     delta_count=self.delta["count"], delta_tot=self.delta["tot"])
        if getattr(self, "bounded", False):
            t.update(bound_ub=self.ub, bound_lb=self.lb, bound_cand=self.cand, bound_rows=self._brows,
                     bound_count=self._bcount, bound_scratch=self._bscratch, bound_work=self._bwork,
                     bound_qshift=self.qshift)
            if self.oseed is not None:
                t["bound_oseed"] = self.oseed
        out = {k: _r(v.numel() * v.element_size()) for k, v in t.items()}
        for name in ("bufs", "stage"):          # streaming: two chunk / staging buffers
            bl = getattr(self, name, None)
            if bl:
                out["chunk_bufs" if name == "bufs" else "staging"] = sum(
                    _r(b.numel() * b.element_size()) for b in bl)
        if getattr(self, "part", None) is not None:
            out["packed"] += _r(self.part.numel() * 8)
        return out

    def reset_labels(self):
        """Unassign every point (the reference's Restart, app.mjs:167-178); the next
        step re-assigns from the current centres and counts every point as changed."""
        self.labels.fill_(-1)
        self._invalidate_bounds()
        return self

    def set_centers(self, centers: torch.Tensor):
        c = centers.to(device=self.device, dtype=torch.float32)
        if c.shape != (self.K, self.D):
            raise ValueError(f"centers must be [{self.K}, {self.D}], got {tuple(c.shape)}")
        if self.spherical:
            c = c / c.norm(dim=1, keepdim=True).clamp_min(1e-30)
        self.C.zero_()
        self.C[:, : self.D] = c
        if self.gpu:
            self.pk.finalize(0, None, self.C)
        self._invalidate_bounds()         # centres replaced: bounds no longer hold
        return self

    def _invalidate_bounds(self):
        """(bounded E-step) ub = inf: the next E-step re-assigns every row (device writes
        only, so a captured step replays it correctly after new centres or a label reset)."""
        if getattr(self, "bounded", False):
            self.ub.fill_(float("inf"))
            self.lb.zero_()
            self.cand.zero_()

    @property
    def centers(self) -> torch.Tensor:
        return self.C[:, : self.D]

    # ------------------------------------------------------------- iteration
    def step(self):
        """One Lloyd iteration (E-step on the current centres, M-step, all-reduce, finalize)."""
        graphs = getattr(self, "_graphs", None)
        if graphs is not None:
            # two graph launches around the (eager) collective: everything up to the packed
            # message, then everything after it for this centre-buffer parity
            graphs[2 * self._gphase].replay()
            self._collective()
            if self.empty_policy == "farthest":
                # (eager: the relocation reads the counts on the host, after the message's
                # post-collective fix-ups and before it overwrites an empty cluster's sums)
                self._post_reduce()
                self._relocate_empty()
            graphs[2 * self._gphase + 1].replay()
            self._gphase ^= 1
        elif self.gpu:
            self._step_gpu()
        else:
            self._step_cpu()
            if self.spherical:
                self._project_sphere()
        self.C, self.Cnew = self.Cnew, self.C
        self.iteration += 1

    def capture(self):
        """Record a Lloyd iteration as hipGraphs so each later :meth:`step` is two graph
        launches instead of ~6-12 kernel launches.  The graphs hold the device work on
        either side of the iteration's collective -- the packed message (assign, M-step,
        reduce) and the finalize, one pair per centre-buffer parity; the all-reduce and the
        'farthest' empty-cluster relocation (host reads) run eagerly between them.  So no
        RCCL call is ever recorded, and a host-staged communicator works too.

        A capture that fails (a capture-illegal call in a kernel launcher, an allocator
        refusal) is torn down before any further device work: the graphs are discarded, the
        pre-capture state is restored and the engine keeps stepping eagerly
        (``capture_error`` holds the reason).  The replay is bitwise the eager step
        (tests/test_gpu_rccl.py)."""
        self.capture_error = None
        if not self.gpu or not self.n or getattr(self, "_graphs", None) is not None:
            return self
        dev = self.device
        main = torch.cuda.current_stream(dev)
        C0, Cn0 = self.C.clone(), self.Cnew.clone()
        lab0 = self.labels.clone()
        state0 = self._capture_state()
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(main)
        try:
            # eager warm-up on the side stream: kernel attributes, workspaces, allocator
            with torch.cuda.stream(side):
                self._pre_collective()
                self._post_collective(relocate=False)
            torch.cuda.synchronize(dev)
            graphs = []
            # one (pre, post) pair per centre-buffer parity: C and Cnew swap every step, and
            # both halves may read them (the bounded E-step's tightening reads C)
            for part in ("pre", "post", "pre", "post"):
                g = torch.cuda.CUDAGraph()
                # thread_local: other threads (the RCCL watchdog polling earlier collectives)
                # may keep making calls that are illegal while a stream captures
                with torch.cuda.graph(g, stream=side, capture_error_mode="thread_local"):
                    if getattr(self, "_inject_capture_fault", False):
                        self.packed[:1].sum().item()    # tests: a capture-illegal host read
                    if part == "pre":
                        self._pre_collective()
                    else:
                        self._post_collective(relocate=False, reduce_part=self.empty_policy != "farthest")
                graphs.append(g)
                if part == "post":   # the next pair: the other centre-buffer parity
                    self.C, self.Cnew = self.Cnew, self.C
        except Exception as e:  # noqa: BLE001 -- any capture failure: eager from here on
            self.capture_error = f"{type(e).__name__}: {e}".splitlines()[0]
            native.warn_once(f"hipGraph capture failed ({self.capture_error}); eager steps")
            graphs = None
            # torch's graph context restores the caller's stream only after a successful
            # capture_end: a failed one leaves the (invalidated) capture stream current, and
            # every later launch on it fails "due to a previous error during capture".  End
            # any capture still open, make the caller's stream current again and never
            # touch the capture stream after this.
            self._C.capture_teardown(side.cuda_stream)
            torch.cuda.set_stream(main)
            side = torch.cuda.Stream(device=dev)
            torch.cuda.synchronize(dev)   # (a capture error is not sticky; a device fault would raise here)
        # the warm-up changed labels / slots / running totals: restore the pre-capture state
        main.wait_stream(side)
        self.C.copy_(C0)
        self.Cnew.copy_(Cn0)
        self.labels.copy_(lab0)
        self._restore_capture_state(state0)
        self.pk.finalize(0, None, self.C)
        torch.cuda.synchronize(dev)
        self._graphs = graphs
        self._gphase = 0
        return self

    def _capture_state(self) -> dict:
        """Device state a warm-up / captured step mutates besides C, Cnew and labels."""
        st = {"slots": self.slots.clone()}
        if self.delta is not None:
            st.update({k: v.clone() for k, v in self.delta.items()})
        if self.bounded:
            st.update(ub=self.ub.clone(), lb=self.lb.clone(), cand=self.cand.clone(), shift=self.shift.clone(),
                      qshift=self.qshift.clone())
        return st

    def _restore_capture_state(self, st: dict):
        self.slots.copy_(st["slots"])
        if self.delta is not None:
            for k, v in self.delta.items():
                v.copy_(st[k])
        if self.bounded:
            for k in ("ub", "lb", "cand", "shift", "qshift"):
                getattr(self, k).copy_(st[k])

    def _step_gpu(self):
        self._pre_collective()
        self._collective()
        self._post_collective()

    def _collective(self):
        with _phase("mikmeans.allreduce"):
            self.comm.allreduce_(self.packed)

    def _post_reduce(self):
        """The message's fix-ups right after the all-reduce: the wide columns' lo sums and,
        for the bounded E-step, the step's inertia from the sums."""
        if self.scales.nw:
            from ..ops import add_wide_lo

            add_wide_lo(self.packed, self.K, self.Dp, self.scales)
        if self.bounded:
            self._bounded_inertia()

    def _bounded_inertia(self):
        """packed[inertia] = sum_i w_i |x_i - c_{l_i}|^2 of the step's labels and centres C,
        as sxx + sum_k (n_k |c_k|^2 - 2 c_k . S_k) from the all-reduced sums S_k and counts n_k
        (f64; the bounded E-step assigns only some rows, so no per-row distances exist).  Global
        already: every rank writes the same value."""
        K, Dp = self.K, self.Dp
        KD = K * Dp
        S = self.packed[:KD].view(K, Dp)
        cnt = self.packed[KD : KD + K]
        c = self.C.double()
        t = cnt * (c * c).sum(1) - 2.0 * (c * S).sum(1)
        self.packed[KD + K : KD + K + 1].copy_(self._sxx + t.sum())

    def _post_collective(self, relocate: bool = True, reduce_part: bool = True):
        """Device work after the all-reduce: the message fix-ups (``reduce_part``),
        (relocation,) finalize, and the sphere projection of the cosine metric."""
        if reduce_part:
            self._post_reduce()
        with _phase("mikmeans.finalize"):
            if relocate:
                self._relocate_empty()
            self.pk.finalize(1, self.packed, self.C, self.Cnew, self.frozen, None, self.shift, self.counts,
                             self.qshift if self.bounded else None)
        if self.spherical:
            self._project_sphere()

    def _pre_collective(self):
        """Device work up to the packed message: assign, M-step, slab reduce."""
        C = self._C
        KD = self.K * self.Dp
        if self.n and self.segments > 1:
            self._assign_update_overlapped()
            C.reduce(self.slab, self.cnt_slab, self.n_chunks, self.K, self.Dp, self.slots, self.packed,
                     self.col_exp, self.cnt_exp)
            if self.weights is not None:
                self._weighted_inertia()
        elif self.n:
            with _phase("mikmeans.assign"):
                if self.bounded:
                    self._bounded_assign()
                else:
                    self.pk.assign(self.X, self.xn, self.labels, self.mind, self.slots, True)
            with _phase("mikmeans.update"):
                d = self.delta
                if d is not None:
                    if self.bounded:   # only the re-assigned candidates can have changed
                        C.label_delta_rows(self.labels, d["prev"], self._brows, self._bcount, d["list"], d["count"])
                    else:
                        C.label_delta(self.labels, d["prev"], d["list"], d["count"])
                    C.update_delta(self.X, self.labels, self.K, self.slab, self.cnt_slab, self.n_chunks,
                                   self.weights, self.col_exp, self.cnt_exp, d["list"], d["count"])
                    C.reduce_delta(self.slab, self.cnt_slab, self.n_chunks, self.K, self.Dp, self.slots,
                                   self.packed, self.col_exp, self.cnt_exp, d["tot"], d["count"],
                                   d["list"].shape[0])
                else:
                    C.update(self.X, self.labels, self.K, self.slab, self.cnt_slab, self.n_chunks,
                             self.weights, self.col_exp, self.cnt_exp, False)
                    C.reduce(self.slab, self.cnt_slab, self.n_chunks, self.K, self.Dp, self.slots,
                             self.packed, self.col_exp, self.cnt_exp)
            if self.weights is not None and not self.bounded:
                self._weighted_inertia()
        else:
            self.packed.zero_()
        sc = self.scales
        if sc.nw and self.n:  # residual (lo) pass of the wide-range columns into the message tail
            C.update(self.X, self.labels, self.K, self.slab, self.cnt_slab, self.n_chunks, self.weights,
                     self.col_exp, self.cnt_exp, False, col_exp2=sc.col_exp2)
            C.reduce_cols(self.slab, self.n_chunks, self.K, self.Dp, sc.wide_cols, sc.wide_exps,
                          self.packed[KD + self.K + 2:])

    def _bounded_assign(self):
        """E-step over the rows the Hamerly bounds cannot vouch for (every row after new
        centres or a label reset): bounds moved by the last shifts -> the flagged rows
        compacted in ascending order (count on the device) -> their exact distance to the
        label's centre (tightening) -> the rows still flagged compacted again -> a gathered
        assign that scatters labels and fresh bounds back to those rows.  No host read."""
        # (the bounds and shifts are the ranked centres' own: no quantisation term; the scores'
        # rounding slack is sized per row from |x|^2, its seed offset and D)
        self._C.bounds_update(self.labels, self.ub, self.lb, self.qshift, self.pk.cn, self.xn, self.cand,
                              self._bwork, self.oseed, self.D)
        self._C.compact(self.cand, self._brows, self._bcount, self._bscratch)
        if self.tighten:
            # Hamerly's second test: the exact distance to the label's centre; rows it clears
            # keep their label, the rest are compacted again for the full assign
            self._C.tighten(self.X, self.D, self.labels, self.C, self._brows, self._bcount, self.ub, self.lb,
                            self.cand, self.xn, self._bwork, self.oseed)
            self._C.compact(self.cand, self._brows, self._bcount, self._bscratch)
        self.pk.assign(self.X, self.xn, self.labels, None, self.slots, True, rows=self._brows, ub=self.ub,
                       lb=self.lb, scatter=True, count=self._bcount, oseed=self.oseed)

    @property
    def reassigned(self) -> int:
        """(bounded E-step) rows the last E-step re-assigned (a host read)."""
        return int(self._bcount.item()) if getattr(self, "bounded", False) else self.n

    def _weighted_inertia(self):
        """packed[inertia] = sum_i w_i mind_i (f64, one pass, no n x 8-byte temporaries)."""
        KD = self.K * self.Dp
        slot = self.packed[KD + self.K : KD + self.K + 1]
        slot.zero_()
        if getattr(self, "_wscratch", None) is None:
            self._wscratch = torch.empty(self._C.WDOT_SCRATCH, dtype=torch.float64, device=self.device)
        self._C.wdot(self.mind, self.weights, slot, self._wscratch)

    def _project_sphere(self):
        """Cnew <- Cnew / |Cnew| (empty / frozen rows are already unit or kept), then the
        shift against the previous centres and the packed copy for the next E-step."""
        Cn = self.Cnew[:, : self.D]
        Cn.div_(Cn.norm(dim=1, keepdim=True).clamp_min(1e-30))
        torch.sum((self.Cnew - self.C) ** 2, dim=1, out=self.shift)
        if getattr(self, "bounded", False):   # the ranked (quantised) centres' move
            q = self.dtype if self.dtype == torch.bfloat16 else torch.float32
            torch.sum((self.Cnew.to(q).float() - self.C.to(q).float()) ** 2, dim=1, out=self.qshift)
        if self.gpu:
            self.pk.finalize(0, None, self.Cnew)

    def _assign_update_overlapped(self):
        C = self._C
        main = torch.cuda.current_stream(self.device)
        self.side.wait_stream(main)  # slab / labels of the previous iteration are free
        kd, nc = self.K * self.Dp, self.seg_chunks
        for s, (r0, r1) in enumerate(self.seg_ranges):
            mind = self.mind[r0:r1] if self.mind is not None else None
            self.pk.assign(self.X[r0:r1], self.xn[r0:r1], self.labels[r0:r1], mind, self.slots, True)
            self.seg_events[s].record(main)
        C.set_update_max_sw(self.overlap_sw)
        try:
            with torch.cuda.stream(self.side):
                for s, (r0, r1) in enumerate(self.seg_ranges):
                    self.side.wait_event(self.seg_events[s])
                    w = self.weights[r0:r1] if self.weights is not None else None
                    C.update(self.X[r0:r1], self.labels[r0:r1], self.K, self.slab[s * nc * kd:],
                             self.cnt_slab[s * nc * self.K:], nc, w, self.col_exp, self.cnt_exp, False)
                self.side_done.record(self.side)
        finally:
            C.set_update_max_sw(0)
        main.wait_event(self.side_done)

    def _step_cpu(self):
        K, Dp = self.K, self.Dp
        KD = K * Dp
        old = self.labels.clone()
        lab, mind = cpu_ops.assign(self.X, self.C, xn=self.xn)
        self.labels = lab
        sums, counts = cpu_ops.cluster_sums(self.X, lab, K, self.weights)
        w = self.weights.double() if self.weights is not None else 1.0
        inertia = (mind.double() * w).sum() if self.n else torch.zeros((), dtype=torch.float64)
        self.packed[:KD] = sums.reshape(-1)
        self.packed[KD : KD + K] = counts
        self.packed[KD + K] = inertia
        self.packed[KD + K + 1] = float((old != lab).sum())
        self.mind = mind
        self.comm.allreduce_(self.packed)
        self._relocate_empty()
        s = self.packed[:KD].view(K, Dp)
        cnt = self.packed[KD : KD + K]
        upd = cnt > 0
        if self.frozen is not None:
            upd &= self.frozen == 0
        new = torch.where(upd[:, None], (s / cnt.clamp_min(1e-300)[:, None]).to(torch.float32), self.C)
        self.Cnew.copy_(new)
        self.shift.copy_(((new - self.C) ** 2).sum(1))
        self.counts.copy_(cnt.to(torch.float32))

    def _relocate_empty(self):
        """Empty-cluster policy 'farthest' (sklearn-like): an empty centre jumps to the
        point farthest from its centre.  Needs a host read of the counts; 'keep' (default)
        leaves empty centres where they are and stays sync-free."""
        if self.empty_policy != "farthest":
            return
        K, Dp = self.K, self.Dp
        KD = K * Dp
        cnt = self.packed[KD : KD + K]
        empty = torch.nonzero(cnt <= 0).flatten().tolist()
        if not empty:
            return
        if self.mind is None or getattr(self, "bounded", False):
            # (GPU engines with this policy allocate mind up front and every full step's assign
            # writes it under the step's centres, graph replays included: nothing to redo.  The
            # bounded E-step writes no distances: the full pass's, under the same packed centres)
            if self.mind is None:
                self.mind = torch.empty(self.n, dtype=torch.float32, device=self.device)
            if self.gpu and self.n:
                self._assign_into(self.mind)
        # global farthest points: every rank proposes its top-|empty| candidates
        m = len(empty)
        local = self.mind[: self.n] if self.n else torch.zeros(0, device=self.device)
        kk = min(m, local.numel())
        vals = torch.full((m,), -1.0, dtype=torch.float64, device=self.device)
        rows = torch.zeros((m, Dp), dtype=torch.float64, device=self.device)
        if kk:
            v, idx = torch.topk(local.double(), kk)
            vals[:kk] = v
            rows[:kk] = self._rows(idx)
        allv = self.comm.all_gather(vals).reshape(-1)
        allr = self.comm.all_gather(rows).reshape(-1, Dp)
        order = torch.argsort(allv, descending=True)[:m]
        for j, k in enumerate(empty):
            if self.frozen is not None and bool(self.frozen[k]):
                continue
            self.packed[k * Dp : (k + 1) * Dp] = allr[order[j]]
            self.packed[KD + k] = 1.0

    def _rows(self, idx: torch.Tensor) -> torch.Tensor:
        """Local rows ``idx`` as float64 ``[m, Dp]`` (the streaming engine fetches them from host)."""
        return self.X[idx.long()].double()

    def _assign_into(self, mind):
        labels = torch.empty_like(self.labels)
        self.pk.assign(self.X, self.xn, labels, mind)

    def last_stats(self) -> IterStats:
        """Host read of the last iteration's scalars (one small D2H copy)."""
        K, KD = self.K, self.K * self.Dp
        s = torch.stack([self.packed[KD + K], self.packed[KD + K + 1], self.shift.double().sum(),
                         self.shift.double().max()]).cpu().tolist()
        return IterStats(self.iteration, s[0], int(round(s[1])), s[2], s[3])

    def run(self, max_iter: int, tol: float = 0.0, *, check_every: int = 1, callback=None):
        """Iterate until ``shift <= tol`` (absolute), no label changes, or ``max_iter``.

        Returns ``(n_iter, converged, history)``; with ``check_every == 0`` the loop never
        synchronises with the host (benchmark mode) and only ``max_iter`` stops it.
        """
        history = []
        converged = False
        for it in range(max_iter):
            self.step()
            if check_every and ((it + 1) % check_every == 0 or it + 1 == max_iter):
                st = self.last_stats()
                history.append(st)
                if callback is not None:
                    callback(st)
                if st.n_changed == 0 and self.iteration > 1:
                    converged = True      # strict convergence: the E-step changed nothing
                    break
                if st.shift <= tol:
                    converged = True
                    break
        return self.iteration, converged, history

    # ----------------------------------------------------------- final E-step
    def assign(self, with_dist: bool = True):
        """Labels (and squared distances) of the local shard w.r.t. the current centres."""
        if self.gpu:
            labels = torch.empty(self.n, dtype=torch.int32, device=self.device)
            mind = torch.empty(self.n, dtype=torch.float32, device=self.device) if with_dist else None
            if self.n:
                xn = self.xn if with_dist else None
                self.pk.assign(self.X, xn, labels, mind)
            return labels, mind
        return cpu_ops.assign(self.X, self.C, with_dist=with_dist, xn=self.xn)

    def inertia(self) -> float:
        """Global inertia of the current centres (sum of squared distances, weighted)."""
        _, mind = self.assign(True)
        w = self.weights.double() if self.weights is not None else 1.0
        t = (mind.double() * w).sum().reshape(1) if self.n else torch.zeros(1, dtype=torch.float64,
                                                                            device=self.device)
        self.comm.allreduce_(t)
        return float(t.item())


def mean_variance(X: torch.Tensor, comm: Comm, n_global: int, D: int | None = None, stats=None) -> float:
    """Mean over the first ``D`` features of the global per-feature variance (sklearn's tol
    scale).  GPU shards use the column-statistics pass (f64 sums of x and x^2, no f32 copy
    of X); ``stats``: this rank's :class:`~mikmeans.ops.ColStats` when already computed."""
    from ..ops import col_stats

    d = int(D if D is not None else X.shape[1])
    if stats is None and X.shape[0] and X.is_cuda:
        stats = col_stats(X)
    if stats is not None:
        s = stats.sum[:d].to(device=comm.device, dtype=torch.float64)
        ss = stats.sumsq[:d].to(device=comm.device, dtype=torch.float64)
    elif X.shape[0]:
        s = torch.zeros(d, dtype=torch.float64, device=X.device)
        ss = torch.zeros_like(s)
        for i in range(0, X.shape[0], 1 << 16):
            xb = X[i : i + (1 << 16), :d].to(torch.float64)
            s += xb.sum(0)
            ss += (xb * xb).sum(0)
    else:
        s = torch.zeros(d, dtype=torch.float64, device=comm.device)
        ss = torch.zeros_like(s)
    t = torch.cat([s, ss]).to(comm.device)
    comm.allreduce_(t)
    mean = t[:d] / max(n_global, 1)
    var = t[d:] / max(n_global, 1) - mean * mean
    return float(var.clamp_min(0).mean().item()) if d else 0.0


def tol_to_abs(tol: float, X: torch.Tensor, comm: Comm, n_global: int, D: int | None = None,
               stats=None) -> float:
    if tol <= 0:
        return 0.0 if tol == 0 else -math.inf
    return tol * mean_variance(X, comm, n_global, D, stats)
