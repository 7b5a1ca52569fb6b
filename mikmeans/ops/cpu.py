"""Plain-PyTorch reference implementations of the kernel ops (CPU path / test oracle).

Semantics match the HIP kernels exactly where it matters for tests:
* bf16 points are scored against bf16-quantised centroids, with fp32 accumulation;
* ties in the argmin go to the lowest centroid index;
* sums and counts are accumulated in float64.
"""
from __future__ import annotations

import torch

_CHUNK = 1 << 16


def quantize_centers(centers: torch.Tensor, dtype: torch.dtype) -> torch.Tensor:
    c = centers.to(torch.float32)
    if dtype == torch.bfloat16:
        c = c.to(torch.bfloat16).to(torch.float32)
    return c


def row_sqnorm(X: torch.Tensor) -> torch.Tensor:
    Xf = X.to(torch.float32)
    return (Xf * Xf).sum(1)


def scores(X: torch.Tensor, centers: torch.Tensor) -> torch.Tensor:
    """``|c|^2 - 2 x.c`` in float32 (the quantity the assign kernel minimises)."""
    c = quantize_centers(centers, X.dtype)
    Xf = X.to(torch.float32)
    return (c * c).sum(1)[None, :] - 2.0 * (Xf @ c.T)


def assign(X: torch.Tensor, centers: torch.Tensor, *, with_dist: bool = True, xn=None):
    n = X.shape[0]
    labels = torch.empty(n, dtype=torch.int32, device=X.device)
    mind = torch.empty(n, dtype=torch.float32, device=X.device) if with_dist else None
    c = quantize_centers(centers, X.dtype)
    cn = (c * c).sum(1)
    for s in range(0, n, _CHUNK):
        xb = X[s : s + _CHUNK].to(torch.float32)
        sc = cn[None, :] - 2.0 * (xb @ c.T)
        m, idx = sc.min(1)
        labels[s : s + _CHUNK] = idx.to(torch.int32)
        if with_dist:
            xnb = xn[s : s + _CHUNK] if xn is not None else (xb * xb).sum(1)
            mind[s : s + _CHUNK] = (xnb + m).clamp_min(0.0)
    return labels, mind


def cluster_sums(X: torch.Tensor, labels: torch.Tensor, K: int, weights=None):
    lab = labels.to(torch.int64)
    Xd = X.to(torch.float64)
    if weights is not None:
        w = weights.to(torch.float64)
        Xd = Xd * w[:, None]
        counts = torch.zeros(K, dtype=torch.float64, device=X.device).index_add_(0, lab, w)
    else:
        counts = torch.bincount(lab, minlength=K).to(torch.float64)
    sums = torch.zeros((K, X.shape[1]), dtype=torch.float64, device=X.device).index_add_(0, lab, Xd)
    return sums, counts
