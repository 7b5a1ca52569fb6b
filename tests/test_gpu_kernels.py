"""Numerics of every HIP kernel against the plain-PyTorch fp32/f64 reference (1 GPU)."""
import numpy as np
import pytest
import torch

import mikmeans
from mikmeans import ops
from mikmeans.data import blobs as B
from mikmeans.ops import cpu as ref
from mikmeans.ops.native import slot_totals

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _points(n, d, dtype, seed=0, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(n, d, generator=g) * scale).to(dtype)


def _check_assign(X, C, labels, mind, rel=2e-5):
    """Tie-tolerant: the chosen centre must be (near-)optimal for every point."""
    Xc = X.cpu()
    sc = ref.scores(Xc, C.cpu())                       # |c|^2 - 2 x.c on quantised centres
    best = sc.min(1).values
    got = sc.gather(1, labels.cpu().long()[:, None])[:, 0]
    scale = (Xc.float() ** 2).sum(1) + (ref.quantize_centers(C.cpu(), X.dtype) ** 2).sum(1).max()
    bad = (got - best) > rel * scale + 1e-6
    assert int(bad.sum()) == 0, f"{int(bad.sum())} suboptimal labels of {len(bad)}"
    if mind is not None:
        xn = (Xc.float() ** 2).sum(1)
        exp = (xn + got).clamp_min(0)
        torch.testing.assert_close(mind.cpu(), exp, rtol=1e-3, atol=1e-3 * float(scale.max()) ** 0.5)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("n,d", [(1, 8), (1000, 2), (4097, 64), (20000, 128), (3000, 256), (777, 30)])
def test_row_sqnorm(native, dtype, n, d):
    X = _points(n, d, dtype, seed=n + d)
    got = ops.row_sqnorm(X.to(DEV)).cpu()
    torch.testing.assert_close(got, ref.row_sqnorm(X), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("n,d,k", [(1000, 2, 3), (513, 16, 37), (20000, 128, 256), (9000, 128, 1024),
                                   (4096, 64, 4096), (3000, 256, 512), (255, 100, 70), (70000, 32, 9),
                                   # wide rows (DPAD 384 / 512 / 768 / 1024 kernels)
                                   (3000, 300, 77), (2500, 500, 130), (2000, 768, 1024), (1500, 1000, 300),
                                   (1200, 1024, 33), (300_001, 768, 64)])
def test_assign_matches_reference(native, dtype, n, d, k):
    X = _points(n, d, dtype, seed=k)
    C = _points(k, d, torch.float32, seed=k + 1)
    labels, mind = ops.assign(X.to(DEV), C.to(DEV), with_dist=True)
    _check_assign(X, C, labels, mind, rel=2e-5 if dtype == torch.float32 else 3e-5)


def _first_argmin(sc):
    """Lowest index among the exact minima of each row (f64 scores)."""
    m = sc.min(1, keepdim=True).values
    idx = torch.arange(sc.shape[1], dtype=torch.int64).expand_as(sc)
    return torch.where(sc == m, idx, sc.shape[1]).min(1).values


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("n,d,k", [(5000, 64, 1300), (3000, 128, 1024), (2000, 32, 300), (4000, 128, 2048),
                                   (60_000, 128, 4096)])
def test_assign_exact_ties_lowest_index(native, dtype, n, d, k):
    """Integer data: every score is exact in f32, so labels must equal the f64 argmin with
    the LOWEST index on exact ties -- every row, ties included (duplicated centres, negative
    and positive scores)."""
    g = torch.Generator().manual_seed(3 + d)
    X = torch.randint(-8, 8, (n, d), generator=g).float()
    C = torch.randint(-8, 8, (k, d), generator=g).float()
    C[17] = C[5]       # exact duplicate centres: the lower index must win
    C[k - 100] = C[40]
    C[k - 1] = C[300 % k]
    X[:50] = C[5]      # rows sitting exactly on a duplicated centre (score -|x|^2 < 0)
    X[50:100] = C[40]
    labels, _ = ops.assign(X.to(dtype).to(DEV), C.to(DEV), with_dist=False)
    sc = ref.scores(X.double(), C.double())
    exp = _first_argmin(sc)
    got = labels.cpu().long()
    if dtype == torch.float32:
        assert torch.equal(got, exp)
    else:
        # bf16 keys: scores are exact too, but the per-point seed offset is added in f32, so
        # two DISTINCT centres with equal exact scores may split by one rounding; the label
        # must be optimal, and among bitwise-equal centres the lowest index
        assert torch.equal(sc.gather(1, got[:, None]), sc.gather(1, exp[:, None]))
        same = (C[got] == C[exp]).all(1)
        assert torch.equal(got[same], exp[same])
        assert torch.equal(got[:100], exp[:100])


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_assign_offset_data_resolution(native, dtype):
    """Data far from the origin (x + 100): labels equal the f64 argmin on the (quantised)
    centres except where the f64 gap to the runner-up is below the fp32 arithmetic of the
    expanded form, 2^-20 (|x|^2 + |c|^2); duplicated centres keep the lowest index."""
    n, d, k = 20000, 128, 512
    g = torch.Generator().manual_seed(11)
    C = torch.randn(k, d, generator=g) * 2.0 + 100.0
    C[7] = C[3]
    X = (C[torch.randint(0, k, (n,), generator=g)] + torch.randn(n, d, generator=g)).to(dtype)
    labels, _ = ops.assign(X.to(DEV), C.to(DEV), with_dist=False)
    Cq = ref.quantize_centers(C, dtype).double()
    Xd = X.double()
    dist = (Xd * Xd).sum(1, keepdim=True) - 2 * Xd @ Cq.T + (Cq * Cq).sum(1)[None]
    exp = _first_argmin(dist)
    srt = dist.sort(1).values
    uniq_gap = torch.where(srt > srt[:, :1], srt, torch.inf).min(1).values - srt[:, 0]
    tol = 2.0**-20 * ((Xd * Xd).sum(1) + (Cq * Cq).sum(1).max())
    ok = uniq_gap > tol
    assert ok.float().mean() > 0.95
    got = labels.cpu().long()
    bad = (got != exp) & ok
    assert int(bad.sum()) == 0, f"{int(bad.sum())} wrong labels of {int(ok.sum())} resolvable rows"
    assert not (got == 7).any()   # the duplicate of centre 3 never wins


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("n,d,k", [(10000, 128, 1024), (50000, 64, 4096), (7000, 256, 512), (999, 8, 3),
                                   (30000, 128, 256), (4000, 128, 20000)])
def test_cluster_sums(native, dtype, n, d, k):
    X = _points(n, d, dtype, seed=d)
    g = torch.Generator().manual_seed(k)
    lab = torch.randint(0, k, (n,), generator=g, dtype=torch.int32)
    sums, counts = ops.cluster_sums(X.to(DEV), lab.to(DEV), k)
    es, ec = ref.cluster_sums(X, lab, k)
    torch.testing.assert_close(counts.cpu(), ec, rtol=0, atol=0)
    torch.testing.assert_close(sums.cpu(), es, rtol=1e-5, atol=1e-4)


def test_cluster_sums_weighted(native):
    X = _points(5000, 32, torch.float32)
    lab = torch.randint(0, 50, (5000,), dtype=torch.int32)
    w = torch.rand(5000)
    sums, counts = ops.cluster_sums(X.to(DEV), lab.to(DEV), 50, w.to(DEV))
    es, ec = ref.cluster_sums(X, lab, 50, w)
    torch.testing.assert_close(counts.cpu(), ec, rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(sums.cpu(), es, rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("case", ["one_label", "two_labels", "uniform", "wide_range"])
def test_cluster_sums_fixed_point_bound(native, case):
    """Packed-pair fixed point (csrc/update.hip): every sum within count * 2^-20 * colmax of
    the f64 sum, bitwise reproducible, including labels that force a flush every period."""
    n, d, k = 300_000, 40, 64
    g = torch.Generator().manual_seed(1)
    X = torch.randn(n, d, generator=g)
    if case == "wide_range":
        X = X * torch.logspace(-6, 6, d)            # per-column exponents must cope
    lab = torch.randint(0, k, (n,), generator=g, dtype=torch.int32)
    if case == "one_label":
        lab.zero_()                                   # every period hits the flush threshold
    elif case == "two_labels":
        lab = (lab % 2).to(torch.int32)
    Xd, ld = X.to(DEV), lab.to(DEV)
    sums, counts = ops.cluster_sums(Xd, ld, k)
    es, ec = ref.cluster_sums(X, lab, k)
    assert torch.equal(counts.cpu(), ec)
    colmax = X.abs().amax(0).double()
    bound = ec[:, None] * colmax[None, :] * 2.0 ** -20
    assert bool(((sums.cpu() - es).abs() <= bound).all())
    again, _ = ops.cluster_sums(Xd, ld, k)          # atomics in another order: same bits
    assert torch.equal(again, sums)


@pytest.mark.parametrize("k,weighted", [(4096, False), (3500, True), (2048, False), (9000, True)])
def test_cluster_sums_large_k_layouts(native, k, weighted):
    """Unpadded + swizzled LDS layout (and the weighted-count variant) at large K."""
    n, d = 200_000, 64
    g = torch.Generator().manual_seed(k)
    X = torch.randn(n, d, generator=g).to(torch.bfloat16)
    lab = torch.randint(0, k, (n,), generator=g, dtype=torch.int32)
    w = torch.rand(n, generator=g) if weighted else None
    sums, counts = ops.cluster_sums(X.to(DEV), lab.to(DEV), k, w.to(DEV) if weighted else None)
    es, ec = ref.cluster_sums(X, lab, k, w)
    if weighted:
        torch.testing.assert_close(counts.cpu(), ec, rtol=1e-5, atol=1e-4)
        torch.testing.assert_close(sums.cpu(), es, rtol=1e-5, atol=1e-3)
    else:
        assert torch.equal(counts.cpu(), ec)
        colmax = X.float().abs().amax(0).double()
        assert bool(((sums.cpu() - es).abs() <= ec[:, None] * colmax[None, :] * 2.0 ** -20).all())


def test_cluster_sums_integer_data_exact(native):
    g = torch.Generator().manual_seed(5)
    X = torch.randint(-1000, 1000, (100_000, 64), generator=g).float()
    lab = torch.randint(0, 300, (100_000,), generator=g, dtype=torch.int32)
    sums, counts = ops.cluster_sums(X.to(DEV), lab.to(DEV), 300)
    es, ec = ref.cluster_sums(X, lab, 300)
    assert torch.equal(sums.cpu(), es) and torch.equal(counts.cpu(), ec)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_blobs_match_numpy_mirror(native, dtype):
    Cg = B.blob_centers(16, 40, 10.0, seed=11, device=DEV)
    Cn = B.blob_centers_np(16, 40, 10.0, seed=11)
    np.testing.assert_allclose(Cg.cpu().numpy(), Cn, rtol=0, atol=0)
    Xg, yg = B.make_blobs(5000, 40, 16, seed=11, i0=123456789, dtype=dtype, device=DEV,
                          return_labels=True, centers=Cg)
    Xn, yn = B.blobs_np(123456789, 5000, Cn, 1.0, 11, True, bits16=dtype == torch.bfloat16)
    assert np.array_equal(yg.cpu().numpy(), yn)
    tol = 1e-4 if dtype == torch.float32 else 8e-2
    np.testing.assert_allclose(Xg.float().cpu().numpy(), Xn, rtol=0, atol=tol)
    # fused squared norms of the stored values, strided (non-16-byte) output rows too
    nrm = torch.empty(5000, dtype=torch.float32, device=DEV)
    Xs = torch.empty((5000, 41), dtype=dtype, device=DEV)[:, :40]
    B.make_blobs(5000, 40, 16, seed=11, i0=123456789, dtype=dtype, device=DEV, centers=Cg, out=Xs, norms=nrm)
    assert torch.equal(Xs, Xg)
    torch.testing.assert_close(nrm, Xg.float().pow(2).sum(1), rtol=1e-5, atol=1e-3)


def test_blob_stream_prefetch_is_identical(native):
    """Side-stream prefetch (bench cfg5) yields the same batches and the same mini-batch fit --
    also when the engine kicks the next batch's generation between its assign and M-step."""
    from mikmeans.models.minibatch import MiniBatchEngine

    D, K, b = 64, 32, 4096
    res = []
    for pf, kick in ((False, False), (True, False), (True, True)):
        s = B.BlobStream(10**6, D, K, b, seed=5, dtype=torch.bfloat16, device=DEV, with_norms=True, prefetch=pf)
        eng = MiniBatchEngine(K, D, b, dtype=torch.bfloat16, device=DEV)
        if kick:
            eng.after_assign = s.kick
        X0 = next(s)
        eng.set_centers(X0[:K].float())
        batches = [X0.clone()]
        for _ in range(6):
            Xb = next(s)
            batches.append(Xb.clone())
            eng.partial_fit(Xb, s.last_norms)
        torch.cuda.synchronize()
        res.append((batches, eng.C.clone()))
    for r in res[1:]:
        for a, c in zip(res[0][0], r[0]):
            assert torch.equal(a, c)
        assert torch.equal(res[0][1], r[1])


def _resolvable_argmin(X, C, rel=1e-5):
    """f64 argmin of every row (lowest index on ties) and the rows whose gap to the
    runner-up exceeds ``rel`` (|x|^2 + max |c|^2): fp32 arithmetic cannot flip those."""
    Xd, Cd = X.double().cpu(), C.double().cpu()
    xx = (Xd * Xd).sum(1)
    dist = xx[:, None] - 2 * Xd @ Cd.T + (Cd * Cd).sum(1)[None]
    srt = dist.sort(1).values
    ok = (srt[:, 1] - srt[:, 0]) > rel * (xx + (Cd * Cd).sum(1).max())
    return _first_argmin(dist), ok


def test_lloyd_gpu_matches_cpu_engine(native):
    """f32 Lloyd on the GPU (exact-f32 MFMA) against the CPU engine: every row whose
    f64 gap to the runner-up is resolvable gets the f64 argmin label on BOTH engines,
    every step; centres from identical labels agree to f32 rounding."""
    from mikmeans.models.lloyd import LloydEngine

    X = B.make_blobs(20000, 64, 50, seed=5)
    C0 = X[:50].clone()
    ec = LloydEngine(X, 50).set_centers(C0)
    eg = LloydEngine(X.to(DEV), 50).set_centers(C0)
    exp, ok = _resolvable_argmin(X, C0)
    assert ok.float().mean() > 0.99
    ec.step()
    eg.step()
    gl = eg.labels.cpu().long()
    assert torch.equal(gl[ok], exp[ok]) and torch.equal(ec.labels.long()[ok], exp[ok])
    diff = gl != ec.labels.long()
    same = torch.ones(50, dtype=torch.bool)
    same[ec.labels[diff].long()] = False
    same[gl[diff]] = False
    torch.testing.assert_close(eg.centers.cpu()[same], ec.centers[same], rtol=1e-5, atol=1e-5)
    # afterwards the trajectories may part at near-ties: each engine's labels must still be
    # the resolvable f64 argmin of its own previous centres, and the objectives agree
    for _ in range(5):
        cg, cc = eg.centers.cpu().clone(), ec.centers.clone()
        ec.step()
        eg.step()
        eg_exp, eg_ok = _resolvable_argmin(X, cg)
        ec_exp, ec_ok = _resolvable_argmin(X, cc)
        assert torch.equal(eg.labels.cpu().long()[eg_ok], eg_exp[eg_ok])
        assert torch.equal(ec.labels.long()[ec_ok], ec_exp[ec_ok])
    sc, sg = ec.last_stats(), eg.last_stats()
    assert abs(sc.inertia - sg.inertia) <= 1e-3 * abs(sc.inertia)


def test_kmeans_fit_bf16_blobs(native):
    from sklearn.metrics import adjusted_rand_score

    X, y = B.make_blobs(200000, 128, 64, seed=2, dtype=torch.bfloat16, device=DEV, return_labels=True)
    km = mikmeans.KMeans(64, init="greedy-k-means++", dtype="bfloat16", seed=0, max_iter=50).fit(X)
    assert km.cluster_centers_.shape == (64, 128)
    ari = adjusted_rand_score(y.cpu().numpy(), km.labels_.cpu().numpy())
    assert ari > 0.9, ari
    assert np.isfinite(km.inertia_)


def test_kmeanspp_gpu_picks_data_rows(native):
    X = B.make_blobs(30000, 32, 20, seed=9, device=DEV)
    C = mikmeans.kmeans_plusplus(X, 20, seed=4)
    d = ((C.float()[:, None, :] - X.float()[None]) ** 2).sum(-1).min(1).values  # exact, unlike cdist
    assert float(d.max()) == 0.0
    # k-means++ on well separated blobs hits (almost) every blob
    _, y = B.make_blobs(30000, 32, 20, seed=9, device=DEV, return_labels=True)
    lab, _ = ops.assign(C, B.blob_centers(20, 32, 10.0, 9, device=DEV), with_dist=False)
    assert len(set(lab.cpu().tolist())) >= 17


@pytest.mark.parametrize("dtype,d,trials", [(torch.bfloat16, 64, 1), (torch.float32, 32, 1),
                                            (torch.bfloat16, 128, 3)])
def test_kmeanspp_pruned_is_bitwise_unpruned(native, dtype, d, trials):
    """The triangle-inequality pruned D^2 passes must reproduce the unpruned seeding bit for bit."""
    from mikmeans.models.init import init_kmeanspp
    from mikmeans.parallel import Comm

    n, k = 60000, 96
    X = B.make_blobs(n, d, 40, seed=11, dtype=dtype, device=DEV)
    comm = Comm.local(DEV)
    a = init_kmeanspp(X, d, k, n, 0, comm, seed=2, n_local_trials=trials, prune=True)
    b = init_kmeanspp(X, d, k, n, 0, comm, seed=2, n_local_trials=trials, prune=False)
    assert torch.equal(a, b)


def test_kmeanspp_gpu_cpu_same_seed_same_first_center(native):
    X = B.make_blobs(5000, 16, 8, seed=1)
    Cg = mikmeans.kmeans_plusplus(X.to(DEV), 8, seed=7).cpu()
    Cc = mikmeans.kmeans_plusplus(X, 8, seed=7)
    torch.testing.assert_close(Cg[0], Cc[0])


def test_minibatch_gpu_vs_cpu(native):
    from mikmeans.models.minibatch import MiniBatchEngine

    X = B.make_blobs(8192, 32, 10, seed=3)
    C0 = X[:10].clone()
    ec = MiniBatchEngine(10, 32, 1024)
    eg = MiniBatchEngine(10, 32, 1024, device=DEV)
    ec.set_centers(C0)
    eg.set_centers(C0)
    for s in range(8):
        xb = X[s * 1024 : (s + 1) * 1024]
        ec.partial_fit(xb)
        eg.partial_fit(xb.to(DEV))
    torch.testing.assert_close(eg.centers.cpu(), ec.centers, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(eg.vcount.cpu(), ec.vcount)


def test_frozen_centers_stay(native):
    X = B.make_blobs(10000, 16, 4, seed=8, device=DEV)
    C0 = X[:4].clone().float()
    km = mikmeans.KMeans(4, init=C0, frozen=[1, 0, 0, 1], max_iter=10, tol=0).fit(X)
    torch.testing.assert_close(km.cluster_centers_[0], C0[0])
    torch.testing.assert_close(km.cluster_centers_[3], C0[3])


def test_native_extension_is_loaded(native):
    import sys

    assert "mikmeans._C" in sys.modules
    maps = open("/proc/self/maps").read()
    hip = {l.split()[-1] for l in maps.splitlines() if "libamdhip64" in l}
    assert len(hip) == 1, hip  # exactly one HIP runtime (torch's)


@pytest.mark.parametrize("weighted", [False, True])
def test_lloyd_graph_replay_matches_eager(native, weighted):
    """hipGraph-captured iterations (LloydEngine.capture) are bitwise the eager ones."""
    from mikmeans.models.lloyd import LloydEngine

    X = B.make_blobs(50_000, 64, 40, seed=9, dtype=torch.bfloat16, device=DEV)
    w = torch.rand(50_000, device=DEV) if weighted else None
    C0 = X[:40].float()
    ea = LloydEngine(X, 40, sample_weight=w).set_centers(C0)
    eb = LloydEngine(X, 40, sample_weight=w).set_centers(C0).capture()
    assert eb._graphs is not None
    for _ in range(5):
        ea.step()
        eb.step()
        torch.cuda.synchronize()
        assert torch.equal(ea.centers, eb.centers)
        sa, sb = ea.last_stats(), eb.last_stats()
        assert sa.n_changed == sb.n_changed and sa.inertia == sb.inertia
    eb.set_centers(C0)
    ea.set_centers(C0)
    ea.step()
    eb.step()
    assert torch.equal(ea.centers, eb.centers)


@pytest.mark.parametrize("cap", [0, 7, 5000, 200_000])
def test_label_delta_list(native, cap):
    """Changed-row list of the incremental M-step: every changed row once, with its old label."""
    n = 100_003
    g = torch.Generator().manual_seed(cap)
    prev0 = torch.randint(-1, 50, (n,), generator=g, dtype=torch.int32)
    lab = prev0.clone()
    flip = torch.rand(n, generator=g) < 0.03
    lab[flip] = torch.randint(0, 50, (int(flip.sum()),), generator=g, dtype=torch.int32)
    changed = (lab != prev0).nonzero().flatten()
    prev = prev0.to(DEV)
    lst = torch.full((max(cap, 1), 2), -7, dtype=torch.int32, device=DEV)[: cap] if cap else \
        torch.empty((0, 2), dtype=torch.int32, device=DEV)
    cnt = torch.full((1,), 123, dtype=torch.int32, device=DEV)
    native.label_delta(lab.to(DEV), prev, lst, cnt)
    assert int(cnt) == changed.numel()
    assert torch.equal(prev.cpu(), lab)
    m = min(cap, changed.numel())
    got = lst[:m].cpu()
    rows = got[:, 0].long()
    assert rows.unique().numel() == m
    assert torch.equal(got[:, 1], prev0[rows])
    assert bool((lab[rows] != prev0[rows]).all())
    if cap >= changed.numel():
        assert torch.equal(rows.sort().values, changed)


@pytest.mark.parametrize("weighted", [False, True])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("delta_cap", [0.0001, 0.125, 1.0])
def test_incremental_mstep_bitwise(native, weighted, dtype, delta_cap):
    """LloydEngine(incremental=True) re-scatters only changed rows into running integer
    totals; centres, counts and the message must equal the full M-step bit for bit,
    through list overflow (tiny cap), label resets and re-seeding."""
    from mikmeans.models.lloyd import LloydEngine

    n, D, K = 120_000, 64, 48
    X = B.make_blobs(n, D, K, seed=3, dtype=dtype, device=DEV)
    w = torch.rand(n, device=DEV) + 0.5 if weighted else None
    C0 = X[:K].float()
    ea = LloydEngine(X, K, sample_weight=w).set_centers(C0)
    eb = LloydEngine(X, K, sample_weight=w, incremental=True, delta_cap=delta_cap).set_centers(C0)
    assert eb.delta is not None
    KD = K * ea.Dp
    for it in range(10):
        if it == 6:  # re-seed: most labels change -> overflow / full pass
            C1 = X[K: 2 * K].float()
            ea.set_centers(C1)
            eb.set_centers(C1)
        if it == 8:
            ea.reset_labels()
            eb.reset_labels()
        ea.step()
        eb.step()
        torch.cuda.synchronize()
        assert torch.equal(ea.packed[: KD + K], eb.packed[: KD + K]), it
        assert torch.equal(ea.centers, eb.centers), it
        sa, sb = ea.last_stats(), eb.last_stats()
        assert sa.n_changed == sb.n_changed and sa.inertia == sb.inertia


def test_incremental_mstep_graph(native):
    """The incremental step is sync-free, so it captures into the Lloyd hipGraph too."""
    from mikmeans.models.lloyd import LloydEngine

    X = B.make_blobs(80_000, 128, 64, seed=5, dtype=torch.bfloat16, device=DEV)
    C0 = X[:64].float()
    ea = LloydEngine(X, 64).set_centers(C0)
    eb = LloydEngine(X, 64, incremental=True).set_centers(C0).capture()
    assert eb._graphs is not None
    for _ in range(8):
        ea.step()
        eb.step()
        torch.cuda.synchronize()
        assert torch.equal(ea.centers, eb.centers)


@pytest.mark.parametrize("d", [300, 768, 1024])
def test_wide_features_run_native_kernels(native, d):
    """D = 300 / 768 / 1024: fit, predict and mini-batch run the wide-row MFMA kernels (no
    PyTorch GEMM fallback) and agree with the CPU engine."""
    from mikmeans import KMeans, MiniBatchKMeans

    X = B.make_blobs(6000, d, 8, seed=4)
    kg = KMeans(8, init="random", seed=1, max_iter=10, tol=-1.0, device=DEV, dtype="float32").fit(X.to(DEV))
    assert kg._engine.gpu and kg._engine.pk.dpad == ops.dpad_for(d, torch.float32)
    kc = KMeans(8, init="random", seed=1, max_iter=10, tol=-1.0, device="cpu").fit(X)
    lab = kg.predict(X.to(DEV))
    mb = MiniBatchKMeans(8, batch_size=1000, max_iter=5, device=DEV, seed=0).fit(X.to(DEV))
    assert mb._eng.gpu
    assert lab.is_cuda and torch.equal(lab.cpu(), kg.labels_.cpu())
    agree = (kg.labels_.cpu() == kc.labels_).float().mean().item()
    assert agree > 0.99
    assert abs(kg.inertia_ - kc.inertia_) <= 1e-3 * kc.inertia_
    assert mb.cluster_centers_.shape == (8, d)
    kb = KMeans(8, init="random", seed=1, max_iter=10, tol=-1.0, device=DEV, dtype="bfloat16").fit(X.to(DEV))
    # (bf16 rows: a different rounding of the same trajectory -- measured 98.3 % at D = 300)
    assert kb._engine.gpu and (kb.labels_.cpu() == kc.labels_).float().mean().item() > 0.97
    assert abs(kb.inertia_ - kc.inertia_) <= 2e-2 * kc.inertia_


def test_features_past_1024_use_gemm_path(native):
    """D > 1024 (wider than the widest MFMA kernel): the PyTorch GEMM path on the device."""
    import warnings

    from mikmeans import KMeans

    X = B.make_blobs(3000, 1100, 6, seed=4)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        kg = KMeans(6, init="random", seed=1, max_iter=6, tol=-1.0, device=DEV).fit(X.to(DEV))
    kc = KMeans(6, init="random", seed=1, max_iter=6, tol=-1.0, device="cpu").fit(X)
    assert not kg._engine.gpu
    assert (kg.labels_.cpu() == kc.labels_).float().mean().item() > 0.99


@pytest.mark.parametrize("dtype", ["bfloat16", "float32"])
def test_streamed_fit_d768_matches_resident(native, dtype):
    """An out-of-core fit at D=768 (wide-row kernels, chunks of 7680 rows) is the resident
    fit bit for bit."""
    import mikmeans

    n, d, k = 40_000, 768, 32
    X = B.make_blobs(n, d, k, seed=12, dtype=torch.float32, device="cpu")
    Xh = X.to(torch.bfloat16) if dtype == "bfloat16" else X
    kw = dict(init=X[:k].clone(), dtype=dtype, max_iter=5, tol=0, device=DEV)
    ref = mikmeans.KMeans(k, **kw).fit(Xh.to(DEV))
    st = mikmeans.KMeans(k, chunk_rows=7_680, **kw).fit(Xh)
    assert st.memory_plan_["mode"] == "streaming" and ref._engine.gpu
    assert torch.equal(st.cluster_centers_, ref.cluster_centers_)
    assert torch.equal(st.labels_, ref.labels_)


def test_predict_reuses_pack_until_centres_change(native):
    km = mikmeans.KMeans(64, dtype="bfloat16", max_iter=3).fit(
        B.make_blobs(20000, 32, 64, seed=2, dtype=torch.bfloat16, device=DEV))
    X = B.make_blobs(5000, 32, 64, seed=3, dtype=torch.bfloat16, device=DEV)
    l0 = km.predict(X)
    pk = km._pack_cache[2]
    assert torch.equal(km.predict(X), l0) and km._pack_cache[2] is pk      # reused
    with torch.no_grad():                                                  # in-place edit
        km.cluster_centers_[[0, 1]] = km.cluster_centers_[[1, 0]]
    l1 = km.predict(X)
    assert km._pack_cache[2] is not pk
    sw = l0.clone()
    sw[l0 == 0], sw[l0 == 1] = 1, 0
    assert torch.equal(l1, sw)
    km.cluster_centers_ = km.cluster_centers_.clone()                      # new tensor
    assert torch.equal(km.predict(X), l1) and km._pack_cache[0] is km.cluster_centers_


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("n,d,k", [(1, 128, 1024), (1000, 128, 1024), (16384, 64, 4096), (3000, 256, 512),
                                   (70000, 32, 300), (5000, 128, 70)])
def test_assign_centre_split_small_batches(native, dtype, n, d, k):
    """Small batches split the centre range over workgroups; labels, distances and the
    inertia / changed counters equal the one-pass kernel's, calls reuse the scratch."""
    X = _points(n, d, dtype, seed=n + k)
    C = _points(k, d, torch.float32, seed=k + 11)
    Xp = ops.pad_columns(X.to(DEV))
    pk = ops.pack_centers(C.to(DEV), Xp.shape[1], Xp.dtype, DEV)
    assert n <= ops.SPLIT_MAX_ROWS
    xn = ops.row_sqnorm(Xp)
    res = []
    for split in (False, True, True):
        lab = torch.full((n,), 7, dtype=torch.int32, device=DEV)
        mind = torch.empty(n, dtype=torch.float32, device=DEV)
        slots = torch.zeros(native.NSLOT * native.SLOT_STRIDE, dtype=torch.float64, device=DEV)
        if split:
            pk.assign(Xp, xn, lab, mind, slots, True)
        else:
            native.assign(Xp, pk.pack, pk.cn, xn, lab, mind, slots, pk.Kpad, pk.dpad, True, None)
        inert, changed = slot_totals(slots)
        res.append((lab.cpu(), mind.cpu(), inert, changed))
    assert int((pk._keys[:n] != -1).sum()) == 0          # scratch restored to all-ones
    for lab, mind, inert, changed in res[1:]:
        assert torch.equal(lab, res[0][0])
        assert torch.equal(mind, res[0][1])
        assert changed == res[0][3] == float((res[0][0] != 7).sum())
        assert inert == pytest.approx(res[0][2], rel=1e-6)
    _check_assign(X, C, res[1][0], res[1][1], rel=2e-5 if dtype == torch.float32 else 3e-5)


@pytest.mark.parametrize("dtype", ["bfloat16", "float32"])
def test_streaming_fit_matches_resident(native, dtype):
    """Out-of-core Lloyd (host rows streamed in chunks, copy/compute overlap) gives the
    device-resident fit's centres and labels bit for bit (integer M-step, same scales)."""
    X = B.make_blobs(50_000, 60, 32, seed=21, dtype=torch.float32, device=DEV)
    C0 = X[:32].cpu()
    ref = mikmeans.KMeans(32, init=C0, dtype=dtype, max_iter=6, tol=0, device=DEV).fit(X)
    st = mikmeans.KMeans(32, init=C0, dtype=dtype, max_iter=6, tol=0, device=DEV, chunk_rows=6_000).fit(X.cpu())
    from mikmeans.models.streaming import StreamingLloydEngine
    from mikmeans.parallel.shard import ROW_ALIGN

    R = -(-6_000 // ROW_ALIGN) * ROW_ALIGN     # chunks start on the shard grid
    assert isinstance(st._engine, StreamingLloydEngine) and len(st._engine.ranges) == -(-50_000 // R)
    assert st.n_iter_ == ref.n_iter_
    assert torch.equal(st.cluster_centers_, ref.cluster_centers_)
    assert torch.equal(st.labels_, ref.labels_)
    assert st.inertia_ == pytest.approx(ref.inertia_, rel=1e-9)
    torch.testing.assert_close(st.predict(X), ref.predict(X))


def test_streaming_copy_stream_waits_for_buffer_init(native):
    """The chunk copies run on a side stream: they must start behind the caller's queued
    work, including the chunk buffers' own zero fill.  With the caller's stream busy (a
    spin kernel), a copy that raced ahead was overwritten by that fill, and chunk 0's row
    norms and column statistics came out as zeros."""
    from mikmeans.models.streaming import StreamingLloydEngine

    X = B.make_blobs(40_000, 32, 16, seed=5, dtype=torch.bfloat16, device="cpu")
    torch.cuda._sleep(200_000_000)          # ~0.1 s of queued work on the current stream
    eng = StreamingLloydEngine(X, 16, chunk_rows=1 << 13, device=DEV, dtype=torch.bfloat16)
    Xd = X.to(DEV).float()
    torch.testing.assert_close(eng.xn, Xd.pow(2).sum(1), rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(eng.stats.sum[:32], Xd.double().sum(0), rtol=1e-9, atol=1e-6)
    torch.testing.assert_close(eng.stats.sumsq[:32], Xd.double().pow(2).sum(0), rtol=1e-9, atol=1e-6)
    eng.close()


def test_streaming_fit_kmeanspp_sample_init(native):
    # k-means++ runs on a device-resident sample of init_size rows (seeded, sorted draw);
    # the resident fit started from the same seeding must give the same model
    from mikmeans.models.init import resolve_init
    from mikmeans.parallel import Comm

    X = B.make_blobs(40_000, 32, 16, seed=5, dtype=torch.bfloat16, device="cpu")
    km = mikmeans.KMeans(16, dtype="bfloat16", max_iter=20, device=DEV, chunk_rows=1 << 13,
                         init_size=4096).fit(X)
    idx = torch.randperm(40_000, generator=torch.Generator().manual_seed(0))[:4096].sort().values
    C0 = resolve_init("k-means++", X[idx].to(DEV), 32, 16, 4096, 0, Comm.local(torch.device(DEV)), 0)
    ref = mikmeans.KMeans(16, init=C0.cpu(), dtype="bfloat16", max_iter=20, device=DEV).fit(X.to(DEV))
    assert km.labels_.is_cuda and km.labels_.shape == (40_000,)
    from mikmeans.models.lloyd import tol_to_abs

    loc = Comm.local(torch.device(DEV))
    tk = tol_to_abs(1e-4, None, loc, 40_000, 32, stats=km._engine.stats)
    tr = tol_to_abs(1e-4, None, loc, 40_000, 32, stats=ref._engine.stats)
    why = (f"n_iter {km.n_iter_} vs {ref.n_iter_}; tol {tk!r} vs {tr!r}; "
           f"km {[(h['n_changed'], h['shift']) for h in km.history_]} "
           f"ref {[(h['n_changed'], h['shift']) for h in ref.history_]}")
    assert torch.equal(km.cluster_centers_, ref.cluster_centers_), why
    assert km.n_iter_ == ref.n_iter_, why


def test_cosine_metric_gpu(native):
    """Spherical k-means on the MFMA path: unit centres, matches the CPU path from the same
    start up to near-ties, and hipGraph replay equals eager execution bit for bit."""
    from mikmeans.models.lloyd import LloydEngine

    X = B.make_blobs(30_000, 48, 12, seed=13, dtype=torch.float32, device=DEV)
    X = X * torch.rand(30_000, 1, device=DEV).add_(0.5)
    C0 = X[:12].cpu()
    for iters in (1, 8):
        g = mikmeans.KMeans(12, init=C0, metric="cosine", max_iter=iters, tol=0, device=DEV).fit(X)
        c = mikmeans.KMeans(12, init=C0, metric="cosine", max_iter=iters, tol=0, device="cpu").fit(X.cpu())
        torch.testing.assert_close(g.cluster_centers_.norm(dim=1).cpu(), torch.ones(12), rtol=1e-5, atol=1e-5)
        if iters == 1:   # one step from the same start: equal up to the 20-bit fixed point
            torch.testing.assert_close(g.cluster_centers_.cpu(), c.cluster_centers_, rtol=0, atol=2e-4)
        else:            # trajectories may part at near-ties; the objective must agree
            assert g.inertia_ == pytest.approx(c.inertia_, rel=1e-4)
    Xn = (X / X.norm(dim=1, keepdim=True)).to(torch.bfloat16)
    ea = LloydEngine(Xn, 12, spherical=True).set_centers(C0.to(DEV))
    eb = LloydEngine(Xn, 12, spherical=True).set_centers(C0.to(DEV)).capture()
    for _ in range(4):
        ea.step()
        eb.step()
    torch.cuda.synchronize()
    assert torch.equal(ea.centers, eb.centers) and torch.equal(ea.labels, eb.labels)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("n,d", [(1, 64), (1000, 8), (12345, 128), (70001, 256), (3000, 512), (4000, 768),
                                 (2001, 1024), (999, 1504)])
def test_col_absmax_matches_torch(native, dtype, n, d):
    """Native per-column max |x| (fixed-point M-step scales) vs torch.aminmax; strided rows too."""
    from mikmeans.ops import col_max_abs

    # (rows wider than 64 16-B pieces go through the kernel in column blocks)
    g = torch.Generator(device=DEV).manual_seed(n + d)
    X = (torch.randn(n, d, device=DEV, generator=g) * torch.linspace(0.1, 50, d, device=DEV)).to(dtype)
    ref = X.float().abs().amax(0).double()
    assert torch.equal(col_max_abs(X), ref)
    Xs = torch.zeros(n, d + 16, device=DEV, dtype=dtype)[:, 8:8 + d] if dtype == torch.bfloat16 \
        else torch.zeros(n, d + 8, device=DEV, dtype=dtype)[:, 4:4 + d]
    Xs.copy_(X)
    assert torch.equal(col_max_abs(Xs), ref)
    X[n // 2, d // 3] = float("nan")
    assert torch.isnan(col_max_abs(X)[d // 3]) and not torch.isnan(col_max_abs(X)[d // 3 + 1])


def _bf16_dist(Xb, C):
    Cq = ref.quantize_centers(C, torch.bfloat16).double()
    Xd = Xb.double()
    xx = (Xd * Xd).sum(1)
    return xx, Cq, xx[:, None] - 2 * Xd @ Cq.T + (Cq * Cq).sum(1)[None]


@pytest.mark.parametrize("n", [20_000, 300_000])
def test_assign_bf16_outlier_row_keeps_neighbours_resolved(native, n):
    """One row with |x|^2 ~1e6x its workgroup neighbours' must not coarsen their keys: the
    workgroup switches to per-point seed offsets (csrc/assign16.hip), so every other row
    still resolves at 2^-17 of its own distance scale (split and one-pass grids)."""
    d, k = 128, 256
    g = torch.Generator().manual_seed(7)
    X = torch.randn(n, d, generator=g)
    C = torch.randn(k, d, generator=g)
    X[5] *= 1000.0
    X[n // 2 + 3] *= 1000.0
    Xb = X.to(torch.bfloat16)
    labels, mind = ops.assign(Xb.to(DEV), C.to(DEV), with_dist=True)
    xx, Cq, dist = _bf16_dist(Xb, C)
    exp = _first_argmin(dist)
    srt = dist.sort(1).values
    cmax = (Cq * Cq).sum(1).max()
    tol = 2.0**-16 * (srt[:, 0].clamp_min(0) + 3 * xx) + 2.0**-20 * (xx + cmax)
    ok = (srt[:, 1] - srt[:, 0]) > tol
    assert ok.float().mean() > 0.95
    got = labels.cpu().long()
    bad = (got != exp) & ok
    assert int(bad.sum()) == 0, f"{int(bad.sum())} wrong labels of {int(ok.sum())} resolvable rows"
    # distances of the neighbours at their own scale too
    dg = dist.gather(1, got[:, None])[:, 0]
    nb = torch.ones(n, dtype=torch.bool)
    nb[[5, n // 2 + 3]] = False
    err = (mind.cpu().double() - dg.clamp_min(0)).abs()
    assert bool((err[nb] <= tol[nb] + 1e-6).all())


def test_assign_bf16_key_resolution_distance_relative(native):
    """The documented bf16 key resolution: 2^-17 of (|x - c|^2 + the spread of |x|^2 in the
    point's workgroup of 256 rows at D=128), plus the fp32 arithmetic floor; rows whose f64
    gap exceeds twice that get the exact f64 argmin label."""
    n, d, k, wg = 102_400, 128, 1024, 256
    g = torch.Generator().manual_seed(23)
    X = torch.randn(n, d, generator=g)
    C = torch.randn(k, d, generator=g) * 0.7
    Xb = X.to(torch.bfloat16)
    labels, _ = ops.assign(Xb.to(DEV), C.to(DEV), with_dist=False)
    xx, Cq, dist = _bf16_dist(Xb, C)
    exp = _first_argmin(dist)
    srt = dist.sort(1).values
    spread = xx.view(-1, wg).max(1, keepdim=True).values.expand(-1, wg).reshape(-1) - xx
    tol = 2.0**-16 * (srt[:, 0].clamp_min(0) + spread) + 2.0**-20 * (xx + (Cq * Cq).sum(1).max())
    ok = (srt[:, 1] - srt[:, 0]) > tol
    assert ok.float().mean() > 0.9
    bad = (labels.cpu().long() != exp) & ok
    assert int(bad.sum()) == 0, f"{int(bad.sum())} wrong labels of {int(ok.sum())} resolvable rows"


@pytest.mark.parametrize("pmaj", ["0", "1"])
@pytest.mark.parametrize("varg", ["0", "1"])
def test_assign_per_point_offset_seeds_repeatable(native, kvariant, pmaj, varg):
    """Per-point-offset workgroups (N(0,1) rows at D=32: most workgroups) under both MFMA
    issue orders and both epilogues, launched repeatedly with other kernels in between (they
    leave their own data in LDS and registers): every launch gives the same labels, and no
    row with a clear f64 gap (> 1e-3) takes another label.  Packed v_pk_add_f32 seeds got one
    point block wrong in 5 of 12 launches here (profiles/r3_15_ppo_seed_race.md)."""
    n, d, k = 300_000, 32, 1024
    g = torch.Generator().manual_seed(11 + n + d)
    X = torch.randn(n, d, generator=g)
    C = torch.randn(k, d, generator=g) * 0.8
    Xb = X.to(torch.bfloat16)
    xx, Cq, dist = _bf16_dist(Xb, C)
    exp = _first_argmin(dist)
    srt = dist.sort(1).values
    clear = (srt[:, 1] - srt[:, 0]) > 1e-3
    kvariant("assign_pmaj", pmaj)
    kvariant("assign_varg", varg)
    Xd, Cd = Xb.to(DEV), C.to(DEV)
    first = None
    for r in range(6):
        if r % 2:   # another kernel's LDS / register history before the next launch
            Y = torch.randn(200_000, 256, device=DEV, dtype=torch.bfloat16) * 100
            ops.assign(Y, torch.randn(512, 256, device=DEV) * 50, with_dist=True)
        lab = ops.assign(Xd, Cd, with_dist=False)[0].cpu().long()
        bad = (lab != exp) & clear
        assert int(bad.sum()) == 0, f"launch {r}: {int(bad.sum())} rows off the f64 argmin"
        if first is None:
            first = lab
        assert torch.equal(lab, first), f"launch {r} differs from launch 0"


@pytest.mark.parametrize("n,outlier,d,k", [(20_000, False, 64, 4096), (300_000, False, 64, 4096),
                                           (300_000, True, 64, 4096), (40_000, True, 64, 4096),
                                           (300_000, False, 32, 1024), (30_000, True, 32, 1024)])
def test_assign_value_argmin_d64(native, kvariant, n, outlier, d, k):
    """The value-only argmin (bf16 D=64 K >= 2048, D=32 K >= 1024: running minimum + tile in the main loop,
    the row inside the winning tile recovered on the matrix cores afterwards) gives the f64
    argmin on every row resolvable at fp32 resolution of the seeded score, on the split and
    one-pass grids and in per-point-offset workgroups, and distances of the same accuracy;
    where the packed keys resolve a row, both epilogues agree."""
    wg = 512 if d == 64 else 256           # workgroup points (csrc/assign16.hip launch16_d)
    g = torch.Generator().manual_seed(11 + n + d)
    X = torch.randn(n, d, generator=g)
    C = torch.randn(k, d, generator=g) * 0.8
    if outlier:
        X[7] *= 300.0
    Xb = X.to(torch.bfloat16)
    kvariant("assign_varg", "1")
    lv, dv = ops.assign(Xb.to(DEV), C.to(DEV), with_dist=True)
    kvariant("assign_varg", "0")
    lk, _ = ops.assign(Xb.to(DEV), C.to(DEV), with_dist=False)
    xx, Cq, dist = _bf16_dist(Xb, C)
    exp = _first_argmin(dist)
    srt = dist.sort(1).values
    pad = (-n) % wg
    xw = torch.cat([xx, xx[-1:].expand(pad)]).view(-1, wg).max(1, keepdim=True).values.expand(-1, wg)
    off = xw.reshape(-1)[:n] * (1 + 2**-12)          # the workgroup's seed offset scale
    scale = srt[:, 0].clamp_min(0) + off + (Cq * Cq).sum(1).max()
    ok = (srt[:, 1] - srt[:, 0]) > 2.0**-20 * scale
    assert ok.float().mean() > 0.9
    bad = (lv.cpu().long() != exp) & ok
    assert int(bad.sum()) == 0, f"{int(bad.sum())} wrong labels of {int(ok.sum())} resolvable rows"
    torch.testing.assert_close(dv.cpu().double(), srt[:, 0].clamp_min(0), rtol=0,
                               atol=float(2.0**-19 * scale.max()))
    okk = (srt[:, 1] - srt[:, 0]) > 2.0**-15 * scale    # resolvable by the 2^-17 keys too
    assert torch.equal(lv.cpu()[okk], lk.cpu()[okk])


@pytest.mark.parametrize("n,segments", [(3000, 4), (5000, 4), (60_000, 3)])
def test_overlapped_segments_match_plain_step(native, n, segments):
    """The overlapped M-step (assign of segment s+1 on the main stream while segment s is
    scattered on a side stream) equals the plain step bit for bit, also when the 1536-row
    grid leaves some of the requested segments empty (small shards)."""
    from mikmeans.models.lloyd import LloydEngine

    X = B.make_blobs(n, 64, 24, seed=n, dtype=torch.bfloat16, device=DEV)
    C0 = X[:24].float()
    ea = LloydEngine(X, 24).set_centers(C0)
    eb = LloydEngine(X, 24, segments=segments).set_centers(C0)
    assert 1 < eb.segments <= segments and all(e > s for s, e in eb.seg_ranges)
    for _ in range(4):
        ea.step()
        eb.step()
        torch.cuda.synchronize()
        assert torch.equal(ea.centers, eb.centers) and torch.equal(ea.labels, eb.labels)
        assert ea.last_stats().n_changed == eb.last_stats().n_changed


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("n,d,k", [(1000, 2, 3), (20001, 128, 1024), (5000, 64, 4097), (3000, 256, 77),
                                   (2000, 768, 100), (1500, 1024, 16), (777, 30, 513)])
def test_transform_kernel_matches_reference(native, dtype, n, d, k):
    """KMeans.transform's MFMA kernel: every row's distance to every centre against the f64
    distances to the quantised centres; argmin of the row equals the assign's label on rows
    the scores resolve."""
    X = _points(n, d, dtype, seed=n + k)
    C = _points(k, d, torch.float32, seed=k + 3)
    got = ops.transform(X.to(DEV), C.to(DEV))
    assert got.shape == (n, k) and got.dtype == torch.float32
    Cq = ref.quantize_centers(C, dtype).double()
    exp = torch.cdist(X.double(), Cq)
    scale = (X.double() ** 2).sum(1, keepdim=True).sqrt() + Cq.norm(dim=1).max()
    err = (got.cpu().double() - exp).abs()
    tol = (3e-5 if dtype == torch.float32 else 1e-4) * scale + 1e-3
    assert bool((err <= tol).all()), float((err - tol).max())
    sq = ops.transform(X.to(DEV), C.to(DEV), squared=True)
    torch.testing.assert_close(sq.sqrt(), got, rtol=1e-5, atol=1e-5)


def test_kmeans_transform_uses_kernel(native):
    import mikmeans

    X = B.make_blobs(30_000, 96, 12, seed=2, dtype=torch.bfloat16, device=DEV)
    km = mikmeans.KMeans(12, dtype="bfloat16", seed=0, max_iter=10).fit(X)
    D = km.transform(X)
    lab = km.predict(X)
    # the argmin of the distances is the label wherever the best two are apart
    top2 = D.topk(2, largest=False)
    clear = (top2.values[:, 1] - top2.values[:, 0]) > 1e-3
    assert torch.equal(top2.indices[:, 0][clear].int(), lab[clear])
    Dn = km.transform(X[:100].cpu().float().numpy())
    assert Dn.shape == (100, 12)


@pytest.mark.parametrize("n,d,k,outlier", [(300_007, 128, 1024, False), (70_001, 256, 512, True),
                                           (100_003, 64, 4096, True), (5000, 128, 256, False)])
def test_assign_prologue_switches_bitwise(native, kvariant, n, d, k, outlier):
    """The early prologue (norms first, fragments in flight across the seed-offset barrier;
    one norm load per 4 blocks) and the epilogue-read prefetch change only when loads are
    issued and waited for: labels, distances, inertia and changed count are bitwise those of
    the plain prologue -- on ragged N, with an outlier row (per-point-offset workgroups)."""
    from mikmeans.ops import pad_columns

    g = torch.Generator().manual_seed(n + d)
    X = torch.randn(n, d, generator=g)
    if outlier:
        X[n // 2] *= 300.0
    Xb = pad_columns(X.to(torch.bfloat16).to(DEV))
    C = torch.randn(k, d, generator=g) * 0.8
    pk = ops.pack_centers(C.to(DEV), Xb.shape[1], torch.bfloat16, DEV)
    xn = ops.row_sqnorm(Xb)
    out = {}
    for arm in ((0, 0), (0, 1), (1, 1)):
        kvariant("assign_early", arm[0])
        kvariant("assign_epi", arm[1])
        lab = torch.full((n,), 3, dtype=torch.int32, device=DEV)
        mind = torch.empty(n, device=DEV)
        slots = torch.zeros(native.NSLOT * native.SLOT_STRIDE, dtype=torch.float64, device=DEV)
        pk.assign(Xb, xn, lab, mind, slots, True)
        torch.cuda.synchronize()
        out[arm] = (lab, mind, slot_totals(slots))
    ref = out[(0, 0)]
    for arm, o in out.items():
        assert torch.equal(o[0], ref[0]) and torch.equal(o[1], ref[1]), arm
        assert o[2] == ref[2], arm   # (order-free slots: the inertia bitwise too)


def test_assign_timeline_hook(native):
    """set_assign_timeline: every workgroup of the next launches stamps entry <= loop start <=
    epilogue start <= exit (real-time ticks) and its CU; disarmed, launches write nothing."""
    from mikmeans.ops import pad_columns

    n, d, k = 300_000, 128, 256    # (one-pass grid: small batches split the centres instead)
    Xb = pad_columns(torch.randn(n, d, device=DEV).to(torch.bfloat16))
    pk = ops.pack_centers(torch.randn(k, d, device=DEV), Xb.shape[1], torch.bfloat16, DEV)
    xn = ops.row_sqnorm(Xb)
    lab = torch.zeros(n, dtype=torch.int32, device=DEV)
    buf = torch.zeros((n // 16 + 1) * 8, dtype=torch.int64, device=DEV)
    native.set_assign_timeline(buf)
    try:
        pk.assign(Xb, xn, lab)
        torch.cuda.synchronize()
    finally:
        native.set_assign_timeline(None)
    t = buf.view(-1, 8).cpu()
    t = t[t[:, 0] > 0]
    assert len(t) > 0
    assert bool((t[:, 0] <= t[:, 1]).all() and (t[:, 1] <= t[:, 2]).all() and (t[:, 2] <= t[:, 3]).all())
    buf.zero_()
    pk.assign(Xb, xn, lab)
    torch.cuda.synchronize()
    assert int(buf.abs().sum()) == 0
