"""M-step robustness on the GPU: wide-range (outlier) columns, mini-batch scale growth.

The fixed-point scatter-add (csrc/update.hip) quantises every contribution on a
per-column grid derived from the column maximum.  These tests pin the two ways that
grid can be wrong -- a single huge outlier coarsening every other row of its column
(residual lo pass) and a streamed batch exceeding the first batch's range (device
clamp count + rescale) -- against float64 oracles.
"""
import pytest
import torch

from mikmeans import ops
from mikmeans.data import blobs as B

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _oracle_means(X, labels, K):
    Xd = X.double().cpu()
    lab = labels.long().cpu()
    s = torch.zeros(K, X.shape[1], dtype=torch.float64).index_add_(0, lab, Xd)
    c = torch.bincount(lab, minlength=K).double()
    return s, c


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("weighted", [False, True])
def test_outlier_column_sums_exact(native, dtype, weighted):
    n, d, K = 100_000, 64, 16
    g = torch.Generator().manual_seed(0)
    X = torch.randn(n, d, generator=g)
    X[1234, 3] = 1.0e6            # one outlier in an N(0,1) column
    X[777, 40] = -3.0e5
    X = X.to(dtype)
    labels = torch.randint(0, K, (n,), generator=g, dtype=torch.int32)
    w = torch.rand(n, generator=g) + 0.5 if weighted else None
    sc = ops.mstep_scales(X.to(DEV), w.to(DEV) if w is not None else None, n_global=n)
    assert sorted(sc.wide_cols.cpu().tolist()) == [3, 40]
    s, c = ops.cluster_sums(X.to(DEV), labels.to(DEV), K, w.to(DEV) if w is not None else None)
    Xd = X.double() * (w.double()[:, None] if weighted else 1.0)
    s_ref = torch.zeros(K, d, dtype=torch.float64).index_add_(0, labels.long(), Xd)
    c_ref = torch.zeros(K, dtype=torch.float64).index_add_(0, labels.long(),
                                                           w.double() if weighted else torch.ones(n, dtype=torch.float64))
    # centroid error (sum / count) within 1e-5 absolute of the f64 oracle in every column
    err = ((s.cpu() / c.cpu()[:, None]) - (s_ref / c_ref[:, None])).abs().max().item()
    assert err <= 1e-5, err
    torch.testing.assert_close(c.cpu(), c_ref, rtol=1e-6, atol=1e-6)


def test_outlier_lloyd_step_matches_f64(native):
    from mikmeans.models.lloyd import LloydEngine

    n, d, K = 60_000, 32, 8
    X = B.make_blobs(n, d, K, seed=4)
    X[100, 5] = 1.0e6
    C0 = X[torch.arange(K) * 1000 + 7].clone()
    eng = LloydEngine(X.to(DEV), K, incremental=False).set_centers(C0)
    assert eng.scales.nw == 1
    eng.step()
    labels = eng.labels.cpu()
    s, c = _oracle_means(X, labels, K)
    exp = torch.where(c[:, None] > 0, s / c.clamp_min(1)[:, None], C0.double())
    # within 1e-5 of the f64 oracle, beyond the f32 rounding of the centre itself
    err = ((eng.centers.cpu().double() - exp).abs() - exp.abs() * 2.0**-24).max().item()
    assert err <= 1e-5, err
    # the incremental default falls back to full passes with wide columns and agrees bitwise
    eng2 = LloydEngine(X.to(DEV), K, incremental=True).set_centers(C0)
    eng2.step()
    assert torch.equal(eng.centers, eng2.centers)


def test_outlier_lloyd_graph_replay(native):
    from mikmeans.models.lloyd import LloydEngine

    X = B.make_blobs(40_000, 64, 10, seed=6, dtype=torch.bfloat16, device=DEV)
    X[5, 9] = 5.0e5
    C0 = X[:10].float()
    ea = LloydEngine(X, 10).set_centers(C0)
    eb = LloydEngine(X, 10).set_centers(C0).capture()
    for _ in range(3):
        ea.step()
        eb.step()
    torch.cuda.synchronize()
    assert ea.scales.nw == 1 and torch.equal(ea.centers, eb.centers)


def test_update_clamp_count(native):
    C = native
    n, d, K = 20_000, 32, 4
    X = torch.randn(n, d, device=DEV)
    lab = torch.randint(0, K, (n,), device=DEV, dtype=torch.int32)
    nch = C.update_n_chunks(ops.dtype_code(torch.float32), K, d, n, False)
    slab = torch.empty(nch * K * d, dtype=torch.int64, device=DEV)
    cnt = torch.empty(nch * K, dtype=torch.int64, device=DEV)
    # scale made for |x| <= 0.5: rows beyond it are clamped and counted, rows within are not
    col_exp, _ = ops.fixed_exps(X[:1], None, bound=torch.full((d,), 0.5, dtype=torch.float64))
    cc = torch.zeros(1, dtype=torch.int32, device=DEV)
    C.update(X, lab, K, slab, cnt, nch, None, col_exp, 0, True, clamp_count=cc)
    assert int(cc.item()) > 0
    cc.zero_()
    col_exp, _ = ops.fixed_exps(X, None)
    C.update(X, lab, K, slab, cnt, nch, None, col_exp, 0, True, clamp_count=cc)
    assert int(cc.item()) == 0


@pytest.mark.parametrize("case", ["growing", "zero_first"])
def test_minibatch_rescales_instead_of_saturating(native, case):
    """A later batch 20x the first batch's range, or a column that is all zero in the
    first batch: the GPU engine must match the CPU engine (no silent saturation)."""
    from mikmeans.models.minibatch import MiniBatchEngine

    d, K, b = 32, 6, 2048
    g = torch.Generator().manual_seed(1)
    batches = [torch.randn(b, d, generator=g) for _ in range(8)]
    if case == "growing":
        batches[4] = batches[4] * 20.0
    else:
        batches[0][:, 7] = 0.0
    C0 = batches[0][:K].clone()
    ec = MiniBatchEngine(K, d, b)
    eg = MiniBatchEngine(K, d, b, device=DEV)
    ec.set_centers(C0)
    eg.set_centers(C0)
    for xb in batches:
        ec.partial_fit(xb)
        eg.partial_fit(xb.to(DEV))
    assert eg.rescales >= 1
    torch.testing.assert_close(eg.centers.cpu(), ec.centers, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("case", ["uniform", "one_label", "sorted", "unassigned"])
@pytest.mark.parametrize("d,k", [(128, 1024), (64, 4096)])
def test_cluster_sums_ksplit_matches_slice_kernel(native, case, d, k):
    """The K-split M-step (plain full passes at shapes whose column slices are under 128 B,
    csrc/update.hip update_ks_kernel) against the column-slice kernel, which unit weights
    select: the same fixed-point contributions, so the sums must agree bit for bit --
    through hot-label flushes (one label), whole-wave matches that overflow the in-flight
    row groups (sorted labels) and rows without a label (-1)."""
    C = native
    assert C.update_slice_width(ops.dtype_code(torch.bfloat16), k, d, False) * 2 < 128
    n = 300_000
    g = torch.Generator().manual_seed(d + k)
    X = (torch.randn(n, d, generator=g) * 3 + 1).to(torch.bfloat16)
    lab = torch.randint(0, k, (n,), generator=g, dtype=torch.int32)
    if case == "one_label":
        lab.fill_(k - 1)
    elif case == "sorted":
        lab = lab.sort().values
    elif case == "unassigned":
        lab[::3] = -1
    Xd, ld = X.to(DEV), lab.to(DEV)
    sums, counts = ops.cluster_sums(Xd, ld, k)
    ws, _ = ops.cluster_sums(Xd, ld, k, torch.ones(n, device=DEV))
    assert torch.equal(sums, ws)
    valid = lab >= 0
    assert torch.equal(counts.cpu().long(), torch.bincount(lab[valid].long(), minlength=k))
    again, _ = ops.cluster_sums(Xd, ld, k)          # atomics in another order: same bits
    assert torch.equal(again, sums)


def test_ksplit_clamp_count(native):
    """Clamped K-split pass (mini-batch streams): out-of-range rows are counted."""
    C = native
    n, d, K = 50_000, 128, 1024
    X = torch.randn(n, d, device=DEV).to(torch.bfloat16)
    lab = torch.randint(0, K, (n,), device=DEV, dtype=torch.int32)
    dt = ops.dtype_code(torch.bfloat16)
    assert C.update_slice_width(dt, K, d, False) * 2 < 128
    nch = C.update_n_chunks(dt, K, d, n, False)
    slab = torch.empty(nch * K * d, dtype=torch.int64, device=DEV)
    cnt = torch.empty(nch * K, dtype=torch.int64, device=DEV)
    col_exp, _ = ops.fixed_exps(X[:1], None, bound=torch.full((d,), 0.5, dtype=torch.float64))
    cc = torch.zeros(1, dtype=torch.int32, device=DEV)
    C.update(X, lab, K, slab, cnt, nch, None, col_exp, 0, True, clamp_count=cc)
    assert int(cc.item()) > 0
    cc.zero_()
    col_exp, _ = ops.fixed_exps(X, None)
    C.update(X, lab, K, slab, cnt, nch, None, col_exp, 0, True, clamp_count=cc)
    assert int(cc.item()) == 0
    assert int(cnt.view(nch, K).sum()) == n


@pytest.mark.parametrize("dtype,d,k", [(torch.bfloat16, 256, 1024), (torch.bfloat16, 96, 2048),
                                       (torch.float32, 128, 2048), (torch.float32, 256, 1024)])
def test_cluster_sums_ksplit_other_widths_vs_f64(native, dtype, d, k):
    """K-split M-step at 32 / 64 lanes per row and a column-padded width (96 -> 128): each
    lane's column pairs sit one cell per lane group (csrc/update.hip update_ks_kernel), so
    a wrong pair <-> cell map would move sums between columns.  Means against f64."""
    C = native
    es = 2 if dtype == torch.bfloat16 else 4
    dt = ops.dtype_code(dtype)
    dp = ops.pad_columns(torch.zeros(1, d, dtype=dtype)).shape[1]
    sw = C.update_slice_width(dt, k, dp, False)
    if not (0 < sw < dp and sw * es < 128):
        pytest.skip("shape not routed to the K-split kernel")
    n = 200_000
    g = torch.Generator().manual_seed(d * 7 + k)
    X = (torch.randn(n, d, generator=g) * 2 + torch.arange(d) * 0.25).to(dtype)
    lab = torch.randint(0, k, (n,), generator=g, dtype=torch.int32)
    sums, counts = ops.cluster_sums(X.to(DEV), lab.to(DEV), k)
    s_ref, c_ref = _oracle_means(X, lab, k)
    assert torch.equal(counts.cpu().double(), c_ref)
    colmax = X.double().abs().amax(0)
    m = c_ref > 0
    err = ((sums.cpu().double()[m] - s_ref[m]) / c_ref[m][:, None]).abs() / colmax
    assert err.max().item() <= 2.0**-19, err.max().item()


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_col_stats_native_matches_torch(native, dtype):
    """Native column statistics (max |x|, sum |x|, nonzero count, lowest-bit exponent)
    against the torch reference path of the same pass, subnormals and zero columns too."""
    n, d = 50_001, 64
    g = torch.Generator().manual_seed(3)
    X = torch.randn(n, d, generator=g) * torch.logspace(-3, 3, d)
    X[:, 5] = 0.0                                           # all-zero column
    X[:, 6] = (torch.rand(n, generator=g) < 0.01).float()  # one-hot-like
    X[::7, 7] = 0.0
    X[3, 8] = 1e-40                                         # f32 subnormal (bf16 keeps it too)
    X = X.to(dtype)
    st = ops.col_stats(X.to(DEV))
    ref = ops.col_stats(X)                                  # CPU: the torch implementation
    assert torch.equal(st.absmax.cpu(), ref.absmax)
    assert torch.equal(st.nnz.cpu(), ref.nnz)
    assert torch.equal(st.lowbit.cpu(), ref.lowbit)
    torch.testing.assert_close(st.sumabs.cpu(), ref.sumabs, rtol=1e-5, atol=0)
    assert int(st.nnz[5]) == 0 and int(st.lowbit[5]) == ops.ColStats.LOWBIT_NONE
    assert int(st.lowbit[6]) == 0


@pytest.mark.parametrize("d", [8, 48, 128, 512])
def test_col_stats_bf16_edge_values(native, d):
    """The bf16 statistics pass (packed max / nonzero count, lowest-bit exponent recomputed only
    for row groups that could lower it) against the torch reference on values that stress the
    screen: magnitudes falling row by row down through the bf16 subnormals to zero (the exact
    path runs on most groups), +-inf, NaN, -0, an all-zero column, one huge value, a sparse
    column; row counts with ragged tails.  Max / counts / lowest bits exact, f64 sums to
    rounding, fused row norms bitwise row_sqnorm's."""
    from mikmeans.ops import pad_columns

    n = 70_001 + d
    g = torch.Generator().manual_seed(d)
    X = torch.randn(n, d, generator=g) * torch.logspace(-3, 3, d)
    i = torch.arange(n, dtype=torch.float64)
    X[:, 0] = (2.0 ** (-(i % 20_000) / 100.0)).float()        # falls to 2^-200: subnormals, then 0
    X[:, 1 % d] = -X[:, 0]
    if d > 2:
        X[:, 2] = 0.0
        X[7, 2] = -0.0
    if d > 4:
        X[:, 3] = torch.where(torch.rand(n, generator=g) < 0.003, torch.randn(n, generator=g), torch.zeros(n))
        X[11, 4] = float("inf")
        X[12, 4] = float("-inf")
        X[13, 4] = float("nan")
    if d > 5:
        X[n - 1, 5] = 3.0e38
    Xb = X.to(torch.bfloat16)
    Xg = pad_columns(Xb.to(DEV))
    xn = torch.full((n,), -1.0, device=DEV)
    st = ops.col_stats(Xg, xn=xn) if ops.fused_norms_ok(Xg) else ops.col_stats(Xg)
    ref = ops.col_stats(Xb)
    torch.testing.assert_close(st.absmax.cpu()[:d], ref.absmax, rtol=0, atol=0, equal_nan=True)
    assert torch.equal(st.nnz.cpu()[:d], ref.nnz)
    assert torch.equal(st.lowbit.cpu()[:d], ref.lowbit)
    for k in ("sumabs", "sum", "sumsq"):
        a, b = getattr(st, k).cpu()[:d], getattr(ref, k)
        fin = torch.isfinite(b)
        assert torch.equal(torch.isnan(a), torch.isnan(b)) and torch.equal(a[torch.isinf(b)], b[torch.isinf(b)]), k
        torch.testing.assert_close(a[fin], b[fin], rtol=1e-12, atol=0, msg=k)
    if ops.fused_norms_ok(Xg):   # (row 13 holds the NaN)
        torch.testing.assert_close(xn, ops.row_sqnorm(Xg), rtol=0, atol=0, equal_nan=True)


def test_sparse_and_grid_exact_columns_stay_single_pass(native):
    """One-hot columns, sparse continuous columns and small-integer columns with a huge
    value are exact on the hi grid or have a nonzero mean near their max: no residual
    pass (and the incremental M-step stays on).  A dense column with one outlier still
    gets it."""
    from mikmeans.models.lloyd import LloydEngine

    n, d, K = 200_000, 32, 8
    g = torch.Generator().manual_seed(5)
    X = torch.randn(n, d, generator=g)
    hot = torch.randint(0, 1000, (n,), generator=g)
    X[:, 0] = (hot == 0).float()                          # one-hot, 0.1 % nonzero
    X[:, 1] = (hot == 1).float() * 3.0
    sp = torch.rand(n, generator=g) < 0.002
    X[:, 2] = torch.where(sp, torch.randn(n, generator=g) * 2.0, torch.zeros(n))  # sparse continuous
    X[:, 3] = torch.randint(0, 4, (n,), generator=g).float()
    X[17, 3] = 10_000.0                                   # small integers + one huge integer
    X[99, 9] = 4.0e5                                      # dense N(0,1) column with an outlier
    sc = ops.mstep_scales(X.to(DEV), n_global=n)
    assert sc.wide_cols.cpu().tolist() == [9]
    Xs = X.clone()
    Xs[99, 9] = 0.5
    eng = LloydEngine(Xs.to(DEV), K, incremental=True).set_centers(Xs[:K])
    assert eng.scales.nw == 0 and eng.delta is not None


@pytest.mark.parametrize("dtype,d", [(torch.bfloat16, 48), (torch.bfloat16, 128), (torch.bfloat16, 256),
                                     (torch.bfloat16, 512), (torch.float32, 8), (torch.float32, 64),
                                     (torch.float32, 256)])
def test_col_stats_reproducible_with_fused_row_norms(native, dtype, d):
    """(verdict r4) The column statistics' f64 sums are per-block partials summed in a fixed
    order: five launches give bitwise the same sums; the same pass writes every row's |x|^2
    bitwise as row_sqnorm does (one read of X for a fit's setup, canonical order for D up to
    64 pieces); the sums match f64 torch to rounding."""
    from mikmeans.ops import pad_columns

    n = 300_001
    g = torch.Generator().manual_seed(d)
    X = pad_columns((torch.randn(n, d, generator=g) * torch.logspace(-2, 2, d)).to(dtype).to(DEV))
    assert ops.fused_norms_ok(X)
    runs = []
    for _ in range(5):
        xn = torch.full((n,), -1.0, device=DEV)
        runs.append((ops.col_stats(X, xn=xn), xn))
    for st, xn in runs[1:]:
        for k in ("absmax", "sumabs", "sum", "sumsq", "nnz", "lowbit"):
            assert torch.equal(getattr(st, k), getattr(runs[0][0], k)), k
        assert torch.equal(xn, runs[0][1])
    assert torch.equal(runs[0][1], ops.row_sqnorm(X))
    Xd = X.double().cpu()
    torch.testing.assert_close(runs[0][0].sumsq.cpu(), (Xd * Xd).sum(0), rtol=1e-12, atol=0)
    torch.testing.assert_close(runs[0][0].sum.cpu(), Xd.sum(0), rtol=1e-9, atol=1e-9 * float(Xd.abs().sum()))


def test_resident_and_streamed_fit_agree_at_the_wide_column_threshold(native):
    """(verdict r4) A column whose max is exactly WIDE_RATIO x its nonzero mean (off the hi
    pass's grid, so the knife-edge decides the residual pass): the statistics are
    reproducible, the decision the same on every launch, and the resident and streamed fits
    agree bitwise -- the claim of models/streaming.py."""
    import mikmeans

    n, d, K = 262_144, 32, 16
    g = torch.Generator().manual_seed(2)
    X = torch.randn(n, d, generator=g) * 3.0
    col = torch.zeros(n)
    col[:256] = 1.0 + 2.0 ** -7          # off the hi grid (lowbit -7 < -col_exp)
    col[256] = 66048.0                   # = 256 x the nonzero mean 258, exactly
    X[:, 0] = col[torch.randperm(n, generator=g)]
    X = X.to(torch.bfloat16)
    decisions = {int(ops.mstep_scales(X.to(DEV), n_global=n).nw) for _ in range(5)}
    assert decisions == {0}, decisions
    X[int((X[:, 0] == 66048.0).nonzero()[0]), 0] = 66560.0   # the next bf16 up: past the edge, wide
    assert int(ops.mstep_scales(X.to(DEV), n_global=n).nw) == 1
    X[int((X[:, 0] == 66560.0).nonzero()[0]), 0] = 66048.0
    kw = dict(init="random", dtype="bfloat16", max_iter=6, tol=0.0, seed=3, device=DEV)
    a = mikmeans.KMeans(K, **kw).fit(X.to(DEV))
    b = mikmeans.KMeans(K, chunk_rows=65_536, **kw).fit(X)
    assert b.memory_plan_["mode"] == "streaming"
    assert torch.equal(a.cluster_centers_, b.cluster_centers_)
    assert torch.equal(a.labels_.cpu(), torch.as_tensor(b.labels_).cpu())
