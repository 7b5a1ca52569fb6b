"""Counter-based mini-batch row sampler (NumPy mirror of csrc/rows.hip ``sample_rows``).

Batch row ``j`` of step ``s`` on rank ``r`` is local row

    idx = min(floor(u * n), n - 1),   u = (w >> 11) * 2^-53,
    w = philox4x32-10(counter = (j, s, r, TAG_SMP), key = seed) words (x | y << 32)

(with replacement).  A pure function of (seed, rank, step, j): the step counter is the
sampler's whole state (checkpoint / resume), and the device kernel (device-resident
shards) and this mirror (host-resident shards, CPU fits) draw identical rows.  IEEE f64
arithmetic on both sides: ``(w >> 11)`` and the 2^-53 scaling are exact, the product
with n is one correctly rounded multiply.
"""
from __future__ import annotations

import numpy as np

from .blobs import philox4x32

TAG_SMP = 0x53414D50
TAG_KPAR = 0x4B504152


def sample_indices(n: int, b: int, seed: int, rank: int, step: int) -> np.ndarray:
    """Local row indices (int64 ``[b]``) of one mini-batch step."""
    if b <= 0:
        return np.zeros(0, dtype=np.int64)
    if n <= 0:
        raise ValueError("cannot sample from an empty shard")
    j = np.arange(b, dtype=np.uint64)
    r0, r1, _, _ = philox4x32(j, np.uint64(step & 0xFFFFFFFF), np.uint64(rank & 0xFFFFFFFF), TAG_SMP, int(seed))
    w = (r1 << np.uint64(32)) | r0
    u = (w >> np.uint64(11)).astype(np.float64) * 2.0**-53
    idx = (u * float(n)).astype(np.int64)
    return np.minimum(idx, n - 1)


def kpar_uniform(start: int, n: int, seed: int, rnd: int) -> np.ndarray:
    """k-means|| round ``rnd``: the f64 uniform of global rows start..start+n-1 (mirror of
    csrc/rows.hip kpar_select: philox(g_lo, g_hi, rnd, TAG_KPAR; seed), 53 bits)."""
    g = np.arange(start, start + n, dtype=np.uint64)
    r0, r1, _, _ = philox4x32(g & np.uint64(0xFFFFFFFF), g >> np.uint64(32), np.uint64(rnd & 0xFFFFFFFF),
                              TAG_KPAR, int(seed))
    w = (r1 << np.uint64(32)) | r0
    return (w >> np.uint64(11)).astype(np.float64) * 2.0**-53
