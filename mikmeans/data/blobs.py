"""Synthetic Gaussian blobs, deterministic by (seed, global row index).

Row ``i`` of a dataset is a pure function of ``(seed, i)`` (counter-based
Philox4x32-10), so every rank of a data-parallel job generates exactly its own
row range, on device, with no host traffic (BASELINE config 5 streams 1e9 rows:
PCIe at 63 GB/s would be ~100x too slow).  The GPU path is the HIP kernel K8
(csrc/kpp.hip); the CPU path below is a NumPy mirror of the same generator
(bit-identical integers; the device uses the hardware log2/sqrt/sin/cos, so the floats
agree to a few ulp before rounding).

Blob centres are uniform in ``[-box, box]^D`` (like sklearn's ``make_blobs``
``center_box=(-10, 10)``); the cluster of row i is ``mulhi(philox(i), n_centers)``.
"""
from __future__ import annotations

import numpy as np
import torch

from ..ops import native

M0, M1 = 0xD2511F53, 0xCD9E8D57
W0, W1 = 0x9E3779B9, 0xBB67AE85
MASK = 0xFFFFFFFF
TAG_CID, TAG_CTR, TAG_NRM = 0xC1D0, 0xCE27, 0x4E52


def philox4x32(c0, c1, c2, c3, seed: int):
    """Vectorised Philox4x32-10 over uint32 counter arrays (NumPy, uint64 math)."""
    c0, c1, c2, c3 = (np.asarray(c, dtype=np.uint64) & MASK for c in (c0, c1, c2, c3))
    c0, c1, c2, c3 = np.broadcast_arrays(c0, c1, c2, c3)
    k0 = np.uint64(seed & MASK)
    k1 = np.uint64((seed >> 32) & MASK)
    for _ in range(10):
        p0 = c0 * np.uint64(M0)
        p1 = c2 * np.uint64(M1)
        hi0, lo0 = p0 >> np.uint64(32), p0 & np.uint64(MASK)
        hi1, lo1 = p1 >> np.uint64(32), p1 & np.uint64(MASK)
        c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
        k0 = (k0 + np.uint64(W0)) & np.uint64(MASK)
        k1 = (k1 + np.uint64(W1)) & np.uint64(MASK)
    return c0, c1, c2, c3


def _u01(v):
    return ((v >> np.uint64(8)).astype(np.float32)) * np.float32(1.0 / 16777216.0)


def _u01_open0(v):
    return ((v >> np.uint64(8)) + np.uint64(1)).astype(np.float32) * np.float32(1.0 / 16777216.0)


def blob_centers_np(n_centers: int, d: int, box: float = 10.0, seed: int = 0) -> np.ndarray:
    c = np.arange(n_centers, dtype=np.uint64)[:, None]
    dd = np.arange(d, dtype=np.uint64)[None, :]
    r = philox4x32(c, dd >> np.uint64(2), TAG_CTR, 0, seed)
    lane = (dd & np.uint64(3)).astype(np.int64)
    v = np.choose(np.broadcast_to(lane, r[0].shape), r)
    return (np.float32(box) * (np.float32(2.0) * _u01(v) - np.float32(1.0))).astype(np.float32)


def blobs_np(i0: int, n: int, centers: np.ndarray, std: float = 1.0, seed: int = 0,
             return_labels: bool = False, bits16: bool = False):
    """Rows ``[i0, i0+n)`` of the blob dataset as float32 (NumPy mirror of K8).

    ``bits16``: the bf16 dataset's scheme -- 8 values per Philox call from 16-bit
    uniforms (radius from each word's low half, angle from its high half)."""
    nc, d = centers.shape
    gi = np.arange(i0, i0 + n, dtype=np.uint64)
    lo, hi = gi & np.uint64(MASK), gi >> np.uint64(32)
    rc = philox4x32(lo, hi, TAG_CID, 0, seed)[0]
    cid = ((rc * np.uint64(nc)) >> np.uint64(32)).astype(np.int64)
    el = 8 if bits16 else 4
    G = (d + el - 1) // el
    g = np.arange(G, dtype=np.uint64)[None, :]
    r0, r1, r2, r3 = philox4x32(lo[:, None], hi[:, None], g, TAG_NRM, seed)
    if bits16:
        zs = []
        for w in (r0, r1, r2, r3):
            u = ((w & np.uint64(0xFFFF)) + np.uint64(1)).astype(np.float32) * np.float32(1.0 / 65536.0)
            a = np.float32(2.0 * np.pi) * ((w >> np.uint64(16)).astype(np.float32) * np.float32(1.0 / 65536.0))
            rad = np.sqrt(np.float32(-2.0) * np.log(u)).astype(np.float32)
            zs += [rad * np.cos(a), rad * np.sin(a)]
        z = np.stack(zs, -1)
    else:
        rad0 = np.sqrt(np.float32(-2.0) * np.log(_u01_open0(r0))).astype(np.float32)
        rad1 = np.sqrt(np.float32(-2.0) * np.log(_u01_open0(r2))).astype(np.float32)
        a0 = np.float32(np.pi) * (np.float32(2.0) * _u01(r1))
        a1 = np.float32(np.pi) * (np.float32(2.0) * _u01(r3))
        z = np.stack([rad0 * np.cos(a0), rad0 * np.sin(a0), rad1 * np.cos(a1), rad1 * np.sin(a1)], -1)
    z = z.reshape(n, G * el)[:, :d].astype(np.float32)
    X = (centers[cid] + np.float32(std) * z).astype(np.float32)
    return (X, cid.astype(np.int32)) if return_labels else X


def blob_centers(n_centers: int, d: int, box: float = 10.0, seed: int = 0, device="cpu") -> torch.Tensor:
    device = torch.device(device)
    if device.type == "cuda":
        C = native.require()
        out = torch.empty((n_centers, d), dtype=torch.float32, device=device)
        C.blob_centers(out, float(box), int(seed))
        return out
    return torch.from_numpy(blob_centers_np(n_centers, d, box, seed))


def make_blobs(n: int, d: int, n_centers: int, *, std: float = 1.0, box: float = 10.0, seed: int = 0,
               i0: int = 0, dtype=torch.float32, device="cpu", return_labels: bool = False,
               centers: torch.Tensor | None = None, out: torch.Tensor | None = None,
               norms: torch.Tensor | None = None):
    """Rows ``[i0, i0+n)`` of the ``(seed, n_centers, d)`` blob dataset.

    On a GPU device the rows are generated in place by the HIP kernel (``out``
    may be a preallocated ``[n, ldx>=d]`` view, e.g. column-padded); ``norms``
    (float32 ``[n]``) receives the squared row norms of the stored values.
    """
    device = torch.device(device)
    if centers is None:
        centers = blob_centers(n_centers, d, box, seed, device=device)
    if device.type == "cuda":
        C = native.require()
        X = out if out is not None else torch.empty((n, d), dtype=dtype, device=device)
        y = torch.empty(n, dtype=torch.int32, device=device) if return_labels else None
        C.blobs(X, int(i0), centers.to(device=device, dtype=torch.float32).contiguous(), float(std),
                int(seed), y, norms)
        return (X, y) if return_labels else X
    res = blobs_np(i0, n, centers.cpu().numpy().astype(np.float32), std, seed, return_labels,
                   bits16=dtype == torch.bfloat16)
    Xn, y = (res if return_labels else (res, None))
    X = torch.from_numpy(Xn).to(dtype)
    if out is not None:
        out.copy_(X)
        X = out
    if norms is not None:
        norms.copy_(X.float().pow(2).sum(1))
    return (X, torch.from_numpy(y)) if return_labels else X


class BlobStream:
    """Endless (or bounded) stream of device-generated blob mini-batches.

    Batch j covers global rows ``[offset + j*batch*world + rank*batch, +batch)``:
    ranks interleave so the global stream is identical for any world size.
    """

    def __init__(self, n_total: int, d: int, n_centers: int, batch: int, *, std=1.0, box=10.0,
                 seed=0, dtype=torch.float32, device="cpu", rank=0, world=1, offset=0,
                 with_norms: bool = False, prefetch: bool = False):
        self.n_total, self.d, self.batch = n_total, d, batch
        self.std, self.seed, self.dtype, self.box = std, seed, dtype, box
        self.device = torch.device(device)
        self.rank, self.world, self.offset = rank, world, offset
        self.centers = blob_centers(n_centers, d, box, seed, device=self.device)
        self._buf = None
        self.with_norms = with_norms
        self._nbuf = None
        self.last_norms = None   # squared row norms of the last batch (with_norms=True)
        self.step = 0
        # prefetch (CUDA only): batch j+1 is generated on a side stream into the other of
        # two buffers while the caller's stream consumes batch j, so the VALU-bound
        # generator can share CUs with the LDS-bound M-step instead of running between
        # steps.  The side stream waits for the caller's stream to finish with a buffer
        # (event recorded when the next batch is requested) before overwriting it.
        self.prefetch = bool(prefetch) and self.device.type == "cuda"
        self._pf = None          # (X, norms, ready event) of the batch generated ahead
        self._pending = None     # step whose generation waits for kick()
        self._pool = []
        self._side = torch.cuda.Stream(device=self.device) if self.prefetch else None

    @property
    def value_bound(self) -> float:
        """A bound on |x| of every generated value: centres lie in [-box, box], the
        Box-Muller normals in [-5.78, 5.78] (uniforms are >= 2^-24, -2 ln 2^-24 < 33.3),
        plus one bf16 rounding step."""
        return float((self.box + 6.0 * abs(self.std)) * (1.0 + 2.0**-7))

    def position(self) -> int:
        """Global row offset of the next batch (rows consumed by every rank so far)."""
        return self.offset + self.step * self.world * self.batch

    def seek(self, pos: int) -> "BlobStream":
        """Continue the global row sequence at ``pos`` -- with any world size: a resumed
        job with the same global batch (``batch * world``) sees the same rows per step."""
        if self.prefetch and (self._pf is not None or self._pending is not None):
            raise RuntimeError("seek() before the first batch of a prefetching stream")
        self.offset, self.step = int(pos), 0
        return self

    def __iter__(self):
        return self

    def rows_for(self, step: int) -> tuple[int, int]:
        start = self.offset + (step * self.world + self.rank) * self.batch
        start %= max(self.n_total, 1)
        n = min(self.batch, self.n_total - start)
        return start, n

    def _bufs(self, slot: int):
        while len(self._pool) <= slot:
            X = torch.empty((self.batch, self.d), dtype=self.dtype, device=self.device)
            nb = torch.empty(self.batch, dtype=torch.float32, device=self.device) if self.with_norms else None
            self._pool.append((X, nb))
        return self._pool[slot]

    def _gen(self, step: int, slot: int):
        start, n = self.rows_for(step)
        Xb, nb = self._bufs(slot)
        nrm = nb[:n] if nb is not None else None
        X = make_blobs(n, self.d, 0, std=self.std, seed=self.seed, i0=start, dtype=self.dtype,
                       device=self.device, centers=self.centers, out=Xb[:n], norms=nrm)
        return X, nrm

    def kick(self) -> None:
        """Start generating the next batch now (prefetch streams; no-op otherwise).  The side
        stream starts once the caller's stream reaches this point, so a consumer that calls
        it between its matrix-core assign and its memory-bound M-step (``MiniBatchEngine.
        after_assign``) overlaps the VALU-bound generator with the M-step instead of racing
        the assign for the CUs.  Without a kick, the next batch starts when this one is taken."""
        if self._pending is None:
            return
        j = self._pending
        self._pending = None
        cur = torch.cuda.current_stream(self.device)
        # everything the caller enqueued on batch j-2 (slot j % 2) precedes this point
        freed = torch.cuda.Event()
        freed.record(cur)
        self._side.wait_event(freed)
        with torch.cuda.stream(self._side):
            Xn, nn = self._gen(j, j % 2)
            ready = torch.cuda.Event()
            ready.record(self._side)
        self._pf = (Xn, nn, ready)

    def _next_prefetch(self) -> torch.Tensor:
        cur = torch.cuda.current_stream(self.device)
        j = self.step
        self.kick()                               # (a batch not kicked yet starts now)
        if self._pf is None:                      # first batch: generate in order
            X, nrm = self._gen(j, j % 2)
        else:
            X, nrm, ev = self._pf
            cur.wait_event(ev)
        # batch j+1 goes to slot (j+1) % 2, batch j-1's: generated at the next kick(), when
        # the caller has enqueued all its work on batch j-1
        self._pending = j + 1
        self._pf = None
        self.step += 1
        self.last_norms = nrm
        return X

    def __next__(self) -> torch.Tensor:
        if self.prefetch:
            return self._next_prefetch()
        start, n = self.rows_for(self.step)
        self.step += 1
        if self._buf is None or self._buf.shape[0] < self.batch:
            self._buf = torch.empty((self.batch, self.d), dtype=self.dtype, device=self.device)
        X = self._buf[:n]
        nrm = None
        if self.with_norms:
            if self._nbuf is None or self._nbuf.shape[0] < self.batch:
                self._nbuf = torch.empty(self.batch, dtype=torch.float32, device=self.device)
            nrm = self._nbuf[:n]
        self.last_norms = nrm
        return make_blobs(n, self.d, 0, std=self.std, seed=self.seed, i0=start, dtype=self.dtype,
                          device=self.device, centers=self.centers, out=X, norms=nrm)
