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
