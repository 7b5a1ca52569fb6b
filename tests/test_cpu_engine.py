"""CPU path: Lloyd / k-means++ / mini-batch / API against scikit-learn and invariants."""
import numpy as np
import pytest
import torch

import mikmeans
from mikmeans.data import blobs as B
from mikmeans.models.init import floyd_sample, init_kmeanspp
from mikmeans.models.lloyd import LloydEngine, tol_to_abs
from mikmeans.parallel import Comm, plan, shard_range, shard_sizes

sk_cluster = pytest.importorskip("sklearn.cluster")


def blobs(n=3000, d=8, k=5, seed=1):
    return B.make_blobs(n, d, k, seed=seed, return_labels=True)


def test_config1_parity_with_sklearn():
    """BASELINE config 1: N=1000, D=2, K=3 fp32 on the CPU path."""
    X, _ = blobs(1000, 2, 3, seed=3)
    init = X[:3].numpy()
    km = mikmeans.KMeans(3, init=init, max_iter=100, tol=1e-4, device="cpu").fit(X.numpy())
    sk = sk_cluster.KMeans(3, init=init, n_init=1, max_iter=100, tol=1e-4, algorithm="lloyd").fit(X.numpy())
    assert np.array_equal(km.labels_, sk.labels_)
    np.testing.assert_allclose(km.cluster_centers_.numpy(), sk.cluster_centers_, rtol=1e-5, atol=1e-5)
    assert km.inertia_ == pytest.approx(sk.inertia_, rel=1e-5)
    assert isinstance(km.labels_, np.ndarray) or torch.is_tensor(km.labels_)


def test_lloyd_engine_matches_sklearn_iterates():
    X, _ = blobs(5000, 16, 20, seed=5)
    init = X[:20].numpy().copy()
    eng = LloydEngine(X, 20).set_centers(torch.from_numpy(init))
    eng.run(7, tol=-1, check_every=1)
    sk = sk_cluster.KMeans(20, init=init, n_init=1, max_iter=7, tol=0, algorithm="lloyd").fit(X.numpy())
    np.testing.assert_allclose(eng.centers.numpy(), sk.cluster_centers_, rtol=1e-5, atol=1e-5)


def test_functional_fit_predict_numpy_io():
    X, y = blobs()
    C, lab = mikmeans.fit(X.numpy(), 5, device="cpu", seed=0)
    assert isinstance(C, np.ndarray) and C.shape == (5, 8)
    lab2 = mikmeans.predict(X.numpy(), C)
    assert isinstance(lab2, np.ndarray)
    assert np.array_equal(lab, lab2)
    from sklearn.metrics import adjusted_rand_score

    assert adjusted_rand_score(y.numpy(), lab) > 0.99


def test_kmeans_methods_and_metrics():
    X, _ = blobs()
    km = mikmeans.KMeans(5, device="cpu", seed=0).fit(X)
    assert km.predict(X).dtype == torch.int32
    d = km.transform(X[:10])
    assert d.shape == (10, 5)
    assert km.score(X) == pytest.approx(-km.inertia_, rel=1e-5)
    m = km.metrics()
    assert m["k"] == 5 and sum(m["counts"]) == 3000 and m["balance"]["gap"] == max(m["counts"]) - min(m["counts"])
    assert km.n_iter_ >= 1 and km.converged_
    ft = mikmeans.KMeans(5, device="cpu", seed=0).fit_transform(X)
    assert ft.shape == (3000, 5)
    torch.testing.assert_close(ft.argmin(1).to(torch.int32), km.predict(X))
    with pytest.raises(RuntimeError, match="not fitted"):
        mikmeans.MiniBatchKMeans(3).predict(X)


def test_sample_weight_matches_sklearn():
    X, _ = blobs(2000, 4, 4, seed=9)
    w = np.random.default_rng(0).uniform(0.1, 2.0, 2000).astype(np.float32)
    init = X[:4].numpy()
    km = mikmeans.KMeans(4, init=init, max_iter=50, tol=0, device="cpu").fit(X.numpy(), sample_weight=w)
    sk = sk_cluster.KMeans(4, init=init, n_init=1, max_iter=50, tol=0, algorithm="lloyd").fit(
        X.numpy(), sample_weight=w)
    np.testing.assert_allclose(km.cluster_centers_.numpy(), sk.cluster_centers_, rtol=1e-4, atol=1e-4)
    assert km.inertia_ == pytest.approx(sk.inertia_, rel=1e-4)


def test_frozen_and_empty_policies():
    X, _ = blobs(1000, 2, 2, seed=2)
    far = np.array([[1e4, 1e4]], dtype=np.float32)
    init = np.concatenate([X[:2].numpy(), far])
    km = mikmeans.KMeans(3, init=init, frozen=[0, 0, 1], max_iter=20, device="cpu").fit(X)
    np.testing.assert_array_equal(km.cluster_centers_[2].numpy(), far[0])
    keep = mikmeans.KMeans(3, init=init, max_iter=20, device="cpu").fit(X)
    assert keep.counts_[2] == 0  # empty centre stays put
    np.testing.assert_array_equal(keep.cluster_centers_[2].numpy(), far[0])
    moved = mikmeans.KMeans(3, init=init, max_iter=20, empty_cluster="farthest", device="cpu").fit(X)
    assert moved.counts_.min() > 0


def test_n_init_keeps_best():
    X, _ = blobs(3000, 4, 8, seed=4)
    one = mikmeans.KMeans(8, init="random", n_init=1, seed=0, device="cpu").fit(X)
    many = mikmeans.KMeans(8, init="random", n_init=5, seed=0, device="cpu").fit(X)
    assert many.inertia_ <= one.inertia_ + 1e-6


def test_floyd_sample_distinct_and_deterministic():
    rng = np.random.default_rng(3)
    s = floyd_sample(10**9, 1000, rng)
    assert len(set(s.tolist())) == 1000 and s.min() >= 0 and s.max() < 10**9
    assert np.array_equal(s, floyd_sample(10**9, 1000, np.random.default_rng(3)))
    with pytest.raises(ValueError):
        floyd_sample(5, 6, rng)


@pytest.mark.parametrize("trials", [1, 3])
def test_kmeanspp_cpu(trials):
    X, _ = blobs(4000, 8, 10, seed=6)
    C = init_kmeanspp(X, 8, 10, 4000, 0, Comm.local(), seed=5, n_local_trials=trials)
    d = ((C[:, None, :] - X[None]) ** 2).sum(-1).min(1).values
    assert float(d.max()) == 0.0          # every centre is a data row
    assert len(set(map(tuple, C.numpy().round(4).tolist()))) == 10
    C2 = init_kmeanspp(X, 8, 10, 4000, 0, Comm.local(), seed=5, n_local_trials=trials)
    assert torch.equal(C, C2)


def test_kmeanspp_beats_random_on_blobs():
    X, _ = blobs(6000, 8, 30, seed=8)
    a = mikmeans.KMeans(30, init="k-means++", max_iter=1, tol=-1, seed=0, device="cpu").fit(X).inertia_
    b = mikmeans.KMeans(30, init="random", max_iter=1, tol=-1, seed=0, device="cpu").fit(X).inertia_
    assert a < b


def test_minibatch_cpu_converges():
    X, y = blobs(20000, 8, 6, seed=10)
    mb = mikmeans.MiniBatchKMeans(6, batch_size=1024, max_iter=5, device="cpu", seed=0).fit(X)
    full = mikmeans.KMeans(6, device="cpu", seed=0).fit(X)
    assert mb.score(X) >= 1.05 * full.score(X)   # scores are negative inertias
    assert mb.n_steps_ > 0 and float(mb.counts_.sum()) == pytest.approx(mb.n_steps_ * 1024)
    lab = mb.predict(X)
    torch.testing.assert_close(mb.transform(X).argmin(1).to(torch.int32), lab)
    mb2 = mikmeans.MiniBatchKMeans(6, batch_size=1024, max_iter=5, device="cpu", seed=0)
    assert torch.equal(mb2.fit_predict(X), lab)


def test_minibatch_partial_fit_stream():
    stream = B.BlobStream(10**6, 8, 5, 512, seed=1)
    mb = mikmeans.MiniBatchKMeans(5, batch_size=512, device="cpu")
    mb.fit_stream(stream, steps=20)
    X, _ = blobs(2000, 8, 5, seed=1)
    assert np.isfinite(mb.score(X))


def test_tol_scaling():
    X, _ = blobs(1000, 4, 3)
    var = X.double().var(0, unbiased=False).mean().item()
    assert tol_to_abs(1e-4, X, Comm.local(), 1000) == pytest.approx(1e-4 * var, rel=1e-6)
    assert tol_to_abs(-1, X, Comm.local(), 1000) == float("-inf")


def test_blobs_shard_invariance():
    C = B.blob_centers_np(7, 5, 10.0, 3)
    for b16 in (False, True):
        whole = B.blobs_np(0, 1000, C, 1.0, 3, bits16=b16)
        parts = np.concatenate([B.blobs_np(s, e - s, C, 1.0, 3, bits16=b16)
                                for s, e in (shard_range(1000, r, 3) for r in range(3))])
        assert np.array_equal(whole, parts)
        z = whole - C[B.blobs_np(0, 1000, C, 1.0, 3, True, bits16=b16)[1]]   # unit normals
        assert abs(float(z.mean())) < 0.05 and abs(float(z.std()) - 1.0) < 0.05


def test_shard_plan():
    assert shard_sizes(10, 3) == [10, 0, 0]                  # one 1536-row unit
    assert [shard_range(10, r, 3, align=1) for r in range(3)] == [(0, 4), (4, 7), (7, 10)]
    assert [shard_range(4000, r, 3) for r in range(3)] == [(0, 1536), (1536, 3072), (3072, 4000)]
    assert shard_sizes(10**8, 8)[0] % 1536 == 0 and sum(shard_sizes(10**8, 8)) == 10**8
    p = plan(10**8, 128, 1024, world=1, itemsize=2)
    assert p.fits and p.bytes_points == 25_600_000_000
    big = plan(10**9, 256, 512, world=1, itemsize=2)
    assert not big.fits and big.batch_rows > 0
    assert plan(10**9, 256, 512, world=8, itemsize=2).fits


def test_config_roundtrip_and_argparse():
    import argparse

    cfg = mikmeans.KMeansConfig(n_clusters=7, dtype="bf16", max_iter=3)
    km = mikmeans.KMeans.from_config(cfg)
    assert km.n_clusters == 7 and km.dtype == torch.bfloat16
    ap = mikmeans.KMeansConfig.add_arguments(argparse.ArgumentParser())
    ns = ap.parse_args(["--n-clusters", "4", "--init", "random", "--tol", "0"])
    c2 = mikmeans.KMeansConfig.from_args(ns)
    assert c2.n_clusters == 4 and c2.init == "random" and c2.tol == 0.0
    assert mikmeans.KMeansConfig.from_dict(c2.to_dict()) == c2


def test_bf16_cpu_path_quantises_like_kernel():
    X, _ = blobs(2000, 8, 4, seed=12)
    km = mikmeans.KMeans(4, dtype="bfloat16", device="cpu", seed=0).fit(X)
    assert km.cluster_centers_.dtype == torch.float32
    assert np.isfinite(km.inertia_)


def test_chunk_rows_on_cpu_is_the_resident_fit():
    # out-of-core streaming needs a GPU; on the CPU the option leaves the fit unchanged
    X, _ = blobs(4000, 6, 5, seed=3)
    a = mikmeans.KMeans(5, device="cpu", seed=0).fit(X)
    b = mikmeans.KMeans(5, device="cpu", seed=0, chunk_rows=512).fit(X)
    assert torch.equal(a.cluster_centers_, b.cluster_centers_)
    assert b.get_config().chunk_rows == 512


def test_algorithm_option_cpu():
    """algorithm='hamerly' (alias 'elkan') is the GPU bounded E-step; on the CPU path every
    row is assigned each step, so the fit is Lloyd's, bit for bit."""
    X, _ = blobs(3000, 8, 6, seed=5)
    a = mikmeans.KMeans(6, device="cpu", seed=1).fit(X)
    b = mikmeans.KMeans(6, device="cpu", seed=1, algorithm="elkan").fit(X)
    assert b.algorithm == "hamerly" and b.get_config().algorithm == "hamerly"
    assert a.algorithm == "auto" and a.algorithm_ == "lloyd"      # (the CPU path assigns every row)
    assert torch.equal(a.cluster_centers_, b.cluster_centers_) and a.inertia_ == b.inertia_
    assert mikmeans.KMeans.from_config(b.get_config()).algorithm == "hamerly"
    with pytest.raises(ValueError):
        mikmeans.KMeans(3, algorithm="exact")


def _spherical_reference(X, C0, iters):
    """Plain NumPy spherical k-means (Dhillon & Modha): unit rows, cosine argmax, mean, renormalise."""
    Xn = X / np.linalg.norm(X, axis=1, keepdims=True)
    C = C0 / np.linalg.norm(C0, axis=1, keepdims=True)
    for _ in range(iters):
        lab = (Xn @ C.T).argmax(1)
        for k in range(C.shape[0]):
            m = Xn[lab == k]
            if len(m):
                s = m.sum(0)
                C[k] = s / np.linalg.norm(s)
    return C, lab


def test_cosine_metric_is_spherical_kmeans():
    X, _ = blobs(3000, 8, 6, seed=8)
    X = X.numpy().astype(np.float64)
    X *= np.random.default_rng(0).uniform(0.2, 5.0, size=(len(X), 1))   # row scale must not matter
    C0 = X[:6].copy()
    km = mikmeans.KMeans(6, init=C0.astype(np.float32), metric="cosine", max_iter=10, tol=0, device="cpu").fit(X)
    C = km.cluster_centers_.double().numpy()
    np.testing.assert_allclose(np.linalg.norm(C, axis=1), 1.0, rtol=1e-5)
    ref_C, _ = _spherical_reference(X, C0, km.n_iter_)
    np.testing.assert_allclose(C, ref_C, atol=2e-5)
    Xn = X / np.linalg.norm(X, axis=1, keepdims=True)
    assert np.array_equal(np.asarray(km.predict(X)), (Xn @ C.T).argmax(1))
    km2 = mikmeans.KMeans(6, init=C0.astype(np.float32), metric="cosine", max_iter=10, tol=0,
                          device="cpu").fit(X * 7.0)
    np.testing.assert_allclose(km2.cluster_centers_.numpy(), km.cluster_centers_.numpy(), atol=1e-6)
    with pytest.raises(ValueError):
        mikmeans.KMeans(3, metric="manhattan")


def test_sklearn_params_protocol():
    """get_params / set_params / clone-by-constructor round trip (the scikit-learn estimator
    protocol), normalised values kept, unknown names refused, repr of non-defaults."""
    km = mikmeans.KMeans(16, dtype="bf16", algorithm="elkan", max_iter=10, seed=3)
    p = km.get_params()
    assert p["n_clusters"] == 16 and p["algorithm"] == "hamerly" and p["dtype"] == torch.bfloat16
    k2 = mikmeans.KMeans(**p)
    assert k2.get_params() == p
    assert km.set_params(n_clusters=4, tol=0.0) is km and km.n_clusters == 4 and km.tol == 0.0
    with pytest.raises(ValueError):
        km.set_params(bogus=1)
    with pytest.raises(ValueError):
        km.set_params(algorithm="nope")
    assert repr(km) == "KMeans(n_clusters=4, max_iter=10, tol=0.0, seed=3, dtype='bfloat16', algorithm='hamerly')" \
        or repr(km).startswith("KMeans(n_clusters=4")
    mb = mikmeans.MiniBatchKMeans(8, batch_size=256)
    assert repr(mb) == "MiniBatchKMeans(n_clusters=8, batch_size=256)"
    X, _ = blobs(600, 4, 3, seed=1)
    a = mikmeans.KMeans(3, device="cpu", seed=2).fit(X)
    b = mikmeans.KMeans(**a.get_params()).fit(X)
    assert torch.equal(a.cluster_centers_, b.cluster_centers_)


def test_kmeans_parallel_init_quality_and_weights():
    """k-means|| (init='k-means||'): K distinct data rows whose potential is as good as
    k-means++'s on blob data (within 1.5x); the weighted recluster never picks a zero-weight
    candidate; the NumPy uniform mirror is a pure function of the global row."""
    from mikmeans.data.sampler import kpar_uniform
    from mikmeans.models.init import init_kmeanspp, weighted_kmeanspp
    from mikmeans.parallel import Comm

    X, _ = blobs(6000, 8, 25, seed=7)
    X = torch.as_tensor(X)
    km = mikmeans.KMeans(25, init="k-means||", device="cpu", max_iter=1, seed=2).fit(X)
    C = mikmeans.models.init.init_kmeans_parallel(X, 8, 25, 6000, 0, Comm.local(), seed=2)
    hit = (C[:, None, :] == X.float()[None]).all(-1).any(1)
    assert bool(hit.all()) and torch.unique(C, dim=0).shape[0] == 25
    Cp = init_kmeanspp(X, 8, 25, 6000, 0, Comm.local(), seed=2)
    pot = lambda c: float(torch.cdist(X.double(), c.double()).min(1).values.pow(2).sum())  # noqa: E731
    assert pot(C) <= 1.5 * pot(Cp)
    assert km.cluster_centers_.shape == (25, 8)
    Cc = torch.randn(40, 3)
    w = torch.zeros(40, dtype=torch.float64)
    w[[2, 5, 8, 13, 21]] = 1.0
    out = weighted_kmeanspp(Cc, w, 5, torch.rand(5, dtype=torch.float64))
    got = sorted(int(((Cc - o).abs().sum(1) == 0).nonzero()[0]) for o in out)
    assert got == [2, 5, 8, 13, 21]
    a = kpar_uniform(100, 50, 9, 2)
    b = kpar_uniform(0, 200, 9, 2)[100:150]
    assert np.array_equal(a, b) and ((a >= 0) & (a < 1)).all()


def test_kmeans_parallel_too_few_candidates_keeps_caller_options(monkeypatch):
    """ Data with fewer distinct rows than K: k-means|| collects fewer than K
    candidates and falls back to k-means++ -- with the caller's n_local_trials and sampling,
    not the defaults -- and still returns K data rows."""
    from mikmeans.models import init as I
    from mikmeans.parallel import Comm

    # 2 distinct rows (small integers: duplicates sit at d2 = 0 exactly): the first pick is
    # row 0, round 1 adds row 9, and psi = 0 ends the rounds with 2 < K candidates
    base = torch.tensor([[1.0, 2.0, 3.0, 4.0], [5.0, 6.0, 7.0, 9.0]])
    X = base[torch.tensor([0] * 9 + [1])]
    seen = {}
    real = I.init_kmeanspp

    def spy(*a, **kw):
        seen["trials"] = a[7] if len(a) > 7 else kw.get("n_local_trials")
        seen["sampling"] = kw.get("sampling")
        return real(*a, **kw)

    monkeypatch.setattr(I, "init_kmeanspp", spy)
    assert int(np.random.default_rng(1).integers(0, 10)) < 9          # (seed 1: the first pick is row 0)
    C = I.resolve_init("k-means||", X, 4, 3, 10, 0, Comm.local(), 1, n_local_trials=4, sampling="two-stage")
    assert seen == {"trials": 4, "sampling": "two-stage"}
    assert C.shape == (3, 4)
    assert bool((C[:, None, :] == X[None]).all(-1).any(1).all())


def test_auto_algorithm_votes():
    """algorithm='auto' (the default) votes for the bounded E-step only for the option set it
    reproduces bit for bit and problems big enough for the bounds to pay; the memory plan with
    the bounds is what decides on a GPU (tests/test_gpu_bounded.py: the fits equal 'lloyd')."""
    from mikmeans.parallel import memplan

    km = mikmeans.KMeans(1024)
    n = 1 << 20
    assert km._auto_bounded_ok(n, weighted=False)
    assert not km._auto_bounded_ok(n, weighted=True)
    assert not km._auto_bounded_ok(1000, weighted=False)
    assert not mikmeans.KMeans(8)._auto_bounded_ok(n, weighted=False)
    assert not mikmeans.KMeans(1024, metric="cosine")._auto_bounded_ok(n, weighted=False)
    assert not mikmeans.KMeans(1024, empty_cluster="farthest")._auto_bounded_ok(n, weighted=False)
    assert not mikmeans.KMeans(1024, chunk_rows=1 << 16)._auto_bounded_ok(n, weighted=False)
    # the headline shape: the bounds (~21 B/row) fit beside a resident 1e8 x 128 bf16 shard
    b = memplan.plan_fit(100_000_000, 128, 1024, "bfloat16", budget=280 << 30, x_on_device=True, bounded=True)
    p = memplan.plan_fit(100_000_000, 128, 1024, "bfloat16", budget=280 << 30, x_on_device=True)
    assert b.mode == "resident" and b.fits
    assert 15 * 100_000_000 <= b.peak - p.peak <= 30 * 100_000_000
    # a budget the plain shard fits and the bounds do not: auto falls back to lloyd
    tight = (p.peak + b.peak) // 2
    with pytest.raises(memplan.HBMCapacityError):
        memplan.plan_fit(100_000_000, 128, 1024, "bfloat16", budget=tight, x_on_device=True, bounded=True)
    assert memplan.plan_fit(100_000_000, 128, 1024, "bfloat16", budget=tight, x_on_device=True).fits
