"""Property-based sweeps of the HIP kernels over random shapes (1 GPU; hypothesis with a fixed
seed, so every run draws the same cases): the assign kernel's labels are (near-)optimal and its
distances right for any (rows, features, centres, dtype, data offset) -- ragged tails, features
off the 16-byte grid, centre counts off the 16-centre tile grid, the centre-split path of small
batches and the wide-row kernels included; the M-step's counts are exact and its sums within
the fixed-point bound for any shape, with unassigned (-1) rows."""
import pytest
import torch

from mikmeans import ops
from mikmeans.ops import cpu as ref

from .test_gpu_kernels import _check_assign

hyp = pytest.importorskip("hypothesis")
from hypothesis import HealthCheck, given, settings, strategies as st  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = "cuda"
_SET = dict(max_examples=150, deadline=None, derandomize=True, suppress_health_check=list(HealthCheck))


@settings(**_SET)
@given(n=st.integers(1, 4000), d=st.one_of(st.integers(1, 160), st.integers(161, 1024)),
       k=st.one_of(st.integers(1, 64), st.integers(65, 2048)), bf16=st.booleans(),
       offset=st.sampled_from([0.0, 40.0]), seed=st.integers(0, 2**20))
def test_assign_random_shapes(native, n, d, k, bf16, offset, seed):
    dtype = torch.bfloat16 if bf16 else torch.float32
    g = torch.Generator().manual_seed(seed)
    X = (torch.randn(n, d, generator=g) + offset).to(dtype)
    C = torch.randn(k, d, generator=g) + offset
    labels, mind = ops.assign(X.to(DEV), C.to(DEV), with_dist=True)
    assert labels.shape == (n,) and int(labels.min()) >= 0 and int(labels.max()) < k
    _check_assign(X, C, labels, mind, rel=3e-5 if bf16 else 2e-5)


@settings(**_SET)
@given(n=st.integers(1, 20000), d=st.integers(1, 300), k=st.integers(1, 3000), bf16=st.booleans(),
       unassigned=st.floats(0.0, 0.5), seed=st.integers(0, 2**20))
def test_cluster_sums_random_shapes(native, n, d, k, bf16, unassigned, seed):
    dtype = torch.bfloat16 if bf16 else torch.float32
    g = torch.Generator().manual_seed(seed)
    X = (torch.randn(n, d, generator=g) * 3).to(dtype)
    lab = torch.randint(0, k, (n,), generator=g, dtype=torch.int32)
    lab[torch.rand(n, generator=g) < unassigned] = -1
    sums, counts = ops.cluster_sums(X.to(DEV), lab.to(DEV), k)
    valid = lab >= 0
    es, ec = ref.cluster_sums(X[valid], lab[valid], k)
    torch.testing.assert_close(counts.cpu(), ec, rtol=0, atol=0)
    # fixed point: every contribution within 2^-20 of its column's max |x|
    colmax = X.double().abs().amax(0).clamp_min(1e-30)   # (over every row: the scale's own basis)
    bound = ec.double()[:, None] * colmax[None, :] * 2.0**-19 + 1e-12
    assert bool(((sums.cpu().double() - es.double()).abs() <= bound).all())


@settings(**{**_SET, "max_examples": 30})
@given(n=st.integers(70_000, 200_000), d=st.sampled_from([16, 40, 64, 128, 200, 256]),
       k=st.integers(32, 600), bf16=st.booleans(), init=st.sampled_from(["random", "k-means++"]),
       seed=st.integers(0, 2**16))
def test_bounded_estep_equals_lloyd_random_problems(native, n, d, k, bf16, init, seed):
    """The exact bounded (Hamerly) E-step -- the default algorithm='auto' takes it here -- gives
    the full E-step's labels, centres and iteration count bit for bit on random blob problems."""
    from mikmeans import KMeans
    from mikmeans.data import blobs as B

    dtype = torch.bfloat16 if bf16 else torch.float32
    X = B.make_blobs(n, d, max(2, k // 2), seed=seed, dtype=dtype, device=DEV)
    kw = dict(init=init, max_iter=12, tol=1e-6, seed=seed, dtype=dtype)
    a = KMeans(k, **kw).fit(X)
    f = KMeans(k, algorithm="lloyd", **kw).fit(X)
    assert a.algorithm_ == "hamerly" and f.algorithm_ == "lloyd"
    assert a.n_iter_ == f.n_iter_
    assert torch.equal(a.cluster_centers_, f.cluster_centers_)
    assert torch.equal(a.labels_, f.labels_)


@settings(**{**_SET, "max_examples": 80})
@given(n=st.integers(1, 3000), d=st.integers(1, 600), k=st.integers(1, 700), bf16=st.booleans(),
       seed=st.integers(0, 2**20))
def test_transform_random_shapes(native, n, d, k, bf16, seed):
    """The MFMA transform kernel's [n, K] distances against torch.cdist on the quantised
    centres, and its argmin is a nearest centre."""
    dtype = torch.bfloat16 if bf16 else torch.float32
    g = torch.Generator().manual_seed(seed)
    X = (torch.randn(n, d, generator=g) * 2).to(dtype)
    C = torch.randn(k, d, generator=g) * 2
    got = ops.transform(X.to(DEV), C.to(DEV)).cpu()
    exp = torch.cdist(X.float(), ref.quantize_centers(C, dtype))
    scale = float((X.float() ** 2).sum(1).max() + (C ** 2).sum(1).max()) ** 0.5
    assert got.shape == (n, k)
    torch.testing.assert_close(got, exp, rtol=2e-3, atol=2e-3 * scale)


@settings(**{**_SET, "max_examples": 60})
@given(n=st.integers(1, 40_000), d=st.integers(1, 1100), bf16=st.booleans(), sparse=st.booleans(),
       seed=st.integers(0, 2**20))
def test_col_stats_random_shapes(native, n, d, bf16, sparse, seed):
    """Column statistics (max |x|, nonzero counts, lowest-bit exponents exact; f64 sums to
    rounding) against torch for any shape -- rows wider than one launch's 64 pieces too."""
    dtype = torch.bfloat16 if bf16 else torch.float32
    g = torch.Generator().manual_seed(seed)
    X = torch.randn(n, d, generator=g) * torch.logspace(-2, 2, d)
    if sparse:
        X[torch.rand(n, d, generator=g) < 0.7] = 0.0
    X = X.to(dtype)
    st_ = ops.col_stats(ops.pad_columns(X.to(DEV)))
    rf = ops.col_stats(X)
    assert torch.equal(st_.absmax.cpu()[:d], rf.absmax)
    assert torch.equal(st_.nnz.cpu()[:d], rf.nnz)
    assert torch.equal(st_.lowbit.cpu()[:d], rf.lowbit)
    for key in ("sumabs", "sum", "sumsq"):
        a, b = getattr(st_, key).cpu()[:d], getattr(rf, key)
        tol = 1e-12 * rf.sumabs.abs() if key == "sum" else 1e-12 * b.abs()
        assert bool(((a - b).abs() <= tol + 1e-300).all()), key


@settings(**{**_SET, "max_examples": 40})
@given(n=st.integers(1, 3000), d=st.integers(1, 300), centres=st.integers(1, 64), bf16=st.booleans(),
       i0=st.integers(0, 2**40), seed=st.integers(0, 2**32 - 1))
def test_blobs_match_mirror_random(native, n, d, centres, bf16, i0, seed):
    """The on-device blob generator against its NumPy mirror for any (row offset, shape, seed):
    identical cluster ids, values within the hardware transcendentals' few ulp (bf16: one
    rounding step)."""
    import numpy as np

    from mikmeans.data import blobs as B

    dtype = torch.bfloat16 if bf16 else torch.float32
    Cg = B.blob_centers(centres, d, 10.0, seed=seed, device=DEV)
    Cn = B.blob_centers_np(centres, d, 10.0, seed=seed)
    Xg, yg = B.make_blobs(n, d, centres, seed=seed, i0=i0, dtype=dtype, device=DEV, return_labels=True,
                          centers=Cg)
    Xn, yn = B.blobs_np(i0, n, Cn, 1.0, seed, True, bits16=bf16)
    assert np.array_equal(yg.cpu().numpy(), yn)
    tol = 1e-4 if not bf16 else 8e-2
    np.testing.assert_allclose(Xg.float().cpu().numpy(), Xn, rtol=0, atol=tol)


@settings(**{**_SET, "max_examples": 20})
@given(n=st.integers(20_000, 120_000), d=st.sampled_from([8, 30, 64, 128, 256, 300]),
       k=st.integers(2, 300), bf16=st.booleans(), chunk_units=st.integers(2, 12), seed=st.integers(0, 2**16))
def test_streamed_fit_equals_resident_random(native, n, d, k, bf16, chunk_units, seed):
    """An out-of-core (streamed) fit from host rows is the resident fit bit for bit, for any
    chunk size on the 1536-row grid (every chunk resolves near-ties as the resident pass does)."""
    import mikmeans
    from mikmeans.data import blobs as B

    X = B.make_blobs(n, d, max(2, k), seed=seed, dtype=torch.float32, device="cpu")
    Xh = X.to(torch.bfloat16) if bf16 else X
    kw = dict(init=X[:k].clone(), dtype="bfloat16" if bf16 else "float32", max_iter=4, tol=0, device=DEV,
              algorithm="lloyd")
    res = mikmeans.KMeans(k, **kw).fit(Xh.to(DEV))
    strm = mikmeans.KMeans(k, chunk_rows=1536 * chunk_units, **kw).fit(Xh)
    assert strm.memory_plan_["mode"] == "streaming"
    assert torch.equal(strm.cluster_centers_, res.cluster_centers_)
    assert torch.equal(strm.labels_, res.labels_)
