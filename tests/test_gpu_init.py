"""Seeding on the GPU: k-means|| (models/init.py init_kmeans_parallel, csrc/rows.hip
kpar_select) against its NumPy mirror and against k-means++ quality."""
import numpy as np
import pytest
import torch

from mikmeans.data import blobs as B
from mikmeans.parallel import Comm

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("start", [0, 1536 * 7, (1 << 32) - 5])
def test_kpar_select_matches_numpy_mirror(native, start):
    """The oversampling flags are u_g < l d2 / psi with the philox uniform of the global row g,
    bit for bit the NumPy mirror (also across the 2^32 row boundary)."""
    from mikmeans.data.sampler import kpar_uniform

    n = 100_003
    g = torch.Generator().manual_seed(3)
    d2 = (torch.rand(n, generator=g) ** 4 * 50).float()
    psi = float(d2.double().sum())
    ell = 2000.0
    cand = torch.empty(n, dtype=torch.uint8, device=DEV)
    native.kpar_select(d2.to(DEV), start, torch.tensor([psi], dtype=torch.float64, device=DEV), ell, 11, 3, cand)
    u = kpar_uniform(start, n, 11, 3)
    ref = u < ell * d2.double().numpy() / psi
    got = cand.cpu().numpy().astype(bool)
    assert np.array_equal(got, ref) and 0 < got.sum() < n


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_kmeans_parallel_gpu(native, dtype):
    """k-means|| on the MFMA assign: K distinct data rows, potential within 1.3x of
    k-means++ on blob data, and KMeans(init='k-means||') fits."""
    import mikmeans
    from mikmeans.models.init import init_kmeans_parallel, init_kmeanspp
    from mikmeans.ops import pad_columns

    n, d, k = 400_000, 64, 256
    X = pad_columns(B.make_blobs(n, d, 200, seed=5, dtype=dtype, device=DEV))
    C = init_kmeans_parallel(X, d, k, n, 0, Comm.local(DEV), seed=3)
    Cp = init_kmeanspp(X, d, k, n, 0, Comm.local(DEV), seed=3)
    Xf = X[:, :d].float()
    hit = torch.zeros(k, dtype=torch.bool, device=DEV)
    for i in range(0, n, 50_000):
        hit |= (C[:, None, :] == Xf[None, i:i + 50_000]).all(-1).any(1)
    assert bool(hit.all()) and torch.unique(C, dim=0).shape[0] == k

    def pot(c):
        return float(sum(torch.cdist(Xf[i:i + 50_000].double(), c.double()).min(1).values.pow(2).sum()
                         for i in range(0, n, 50_000)))

    assert pot(C) <= 1.3 * pot(Cp)
    km = mikmeans.KMeans(k, init="k-means||", dtype=dtype, max_iter=3, device=DEV).fit(X[:, :d].contiguous())
    assert km.cluster_centers_.shape == (k, d)


def test_weighted_kmeanspp_graph_equals_eager(native):
    """The k-means|| recluster replayed as hipGraphs of 64 steps gives the eager steps'
    centres bit for bit (the step index and the draws live on the device)."""
    from mikmeans.models.init import weighted_kmeanspp

    g = torch.Generator().manual_seed(2)
    C = torch.randn(5000, 24, generator=g).to(DEV)
    w = torch.randint(0, 50, (5000,), generator=g).double().to(DEV)
    u = torch.rand(300, generator=g, dtype=torch.float64).to(DEV)
    a = weighted_kmeanspp(C, w, 300, u, graph_steps=0)
    b = weighted_kmeanspp(C, w, 300, u, graph_steps=64)
    torch.cuda.synchronize()
    assert torch.equal(a, b)
    assert torch.unique(b, dim=0).shape[0] == 300


@pytest.mark.parametrize("M,D,K", [(300, 8, 40), (41_000, 64, 512), (5_000, 130, 300), (257, 3, 257)])
def test_native_weighted_recluster_matches_torch(native, M, D, K):
    """The k-means|| recluster on the framework's kernels (csrc/kpp.hip wkpp: f64 d2 update +
    block scans, one-workgroup pick) draws the same candidates as the PyTorch oracle
    (cumsum / searchsorted) -- draw for draw, the prefix sums agree except within f64 rounding
    of a boundary -- never a zero-weight candidate, identically on a second run."""
    from mikmeans.models.init import weighted_kmeanspp

    g = torch.Generator().manual_seed(M + K)
    C = (torch.randn(M, D, generator=g) * 3).to("cuda")
    w = torch.randint(0, 20, (M,), generator=g).double().to("cuda")
    if 2 * K >= M:
        w.clamp_min_(1.0)                                             # (every draw finds weight)
    u = torch.rand(K, generator=g, dtype=torch.float64).to("cuda")
    a = weighted_kmeanspp(C, w, K, u)
    b = weighted_kmeanspp(C, w, K, u, native_kernels=False)
    a2 = weighted_kmeanspp(C, w, K, u)
    assert torch.equal(a, a2)
    ia = torch.cdist(a.double(), C.double()).argmin(1)
    ib = torch.cdist(b.double(), C.double()).argmin(1)
    agree = (ia == ib).float().mean().item()
    assert agree == 1.0, agree
    assert bool((w[ia] > 0).all())
