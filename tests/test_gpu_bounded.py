"""Bounded (Hamerly) E-step on the GPU (models/lloyd.py ``bounded``; csrc/assign16.hip TOP2,
csrc/rows.hip bounds_update / seed_offsets): the bounds the kernels keep are valid bounds on
the true distances, the rows they cannot vouch for are the only ones re-assigned, a
re-assigned row gets bitwise the full pass's score and label, and so the fit's iterates --
labels, centres, changed counts -- are bitwise the full E-step's."""
import pytest
import torch

from mikmeans import KMeans, ops
from mikmeans.data import blobs as B
from mikmeans.models.lloyd import LloydEngine
from mikmeans.ops import cpu as ref
from mikmeans.ops.native import slot_totals

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _true_dists(X, C, dtype):
    """Distances of every row to every (quantised) centre, f64 on the host."""
    Cq = ref.quantize_centers(C.cpu(), dtype).double()
    return torch.cdist(X.cpu().double(), Cq)


@pytest.mark.parametrize("dtype,d,k", [(torch.float32, 64, 100), (torch.bfloat16, 128, 256),
                                       (torch.bfloat16, 32, 40)])
def test_full_assign_writes_nearest_and_second_distances(native, dtype, d, k):
    """The first (full) bounded E-step: ub = distance to the label's centre, lb = distance to
    the second nearest centre, both against the quantised centres the kernel ranks."""
    X = B.make_blobs(60_000, d, 16, seed=k, dtype=dtype, device=DEV)
    C0 = X[:k].float() + 0.1
    e = LloydEngine(X, k, bounded=True).set_centers(C0)
    e._bounded_assign()
    torch.cuda.synchronize()
    dist = _true_dists(X, C0, dtype)
    two = dist.topk(2, dim=1, largest=False).values
    lab = e.labels.cpu().long()
    scale = (X.cpu().double() ** 2).sum(1).sqrt() + dist.max()
    assert (dist.gather(1, lab[:, None])[:, 0] - two[:, 0]).abs().max() <= 1e-3 * scale.max()
    torch.testing.assert_close(e.ub.cpu().double(), two[:, 0], rtol=2e-3, atol=2e-3 * float(scale.mean()))
    torch.testing.assert_close(e.lb.cpu().double(), two[:, 1], rtol=2e-3, atol=2e-3 * float(scale.mean()))


@pytest.mark.parametrize("dtype,tighten", [(torch.float32, False), (torch.bfloat16, False),
                                           (torch.bfloat16, True)])
def test_bounds_stay_valid_and_skip_rows(native, dtype, tighten):
    """After every step: every row the bounds vouch for (not a candidate) really is nearest to
    its label's centre, ub >= its distance, lb <= the second distance; and once the centres
    settle, most rows are skipped."""
    X = B.make_blobs(200_000, 64, 32, seed=3, dtype=dtype, device=DEV)
    K = 48
    C0 = X[:K].float()
    e = LloydEngine(X, K, bounded=True, tighten=tighten).set_centers(C0)
    skipped = []
    for it in range(12):
        e.step()
        torch.cuda.synchronize()
        C = e.centers.clone()
        if it >= 1:
            skipped.append(1.0 - e.reassigned / e.n)
        # bounds of the step's labels against the centres that step assigned with (its C0)
        dist = _true_dists(X, C0, dtype)
        lab = e.labels.cpu().long()
        dl = dist.gather(1, lab[:, None])[:, 0]
        masked = dist.clone()
        masked.scatter_(1, lab[:, None], float("inf"))
        d2 = masked.min(1).values
        slack = 1e-3 * ((X.cpu().double() ** 2).sum(1).sqrt() + dist.max())
        assert bool((e.ub.cpu().double() >= dl - slack).all()), it
        assert bool((e.lb.cpu().double() <= d2 + slack).all()), it
        assert bool((dl <= d2 + slack).all()), it            # the label is (near-)nearest
        C0 = C
    assert skipped[-1] > 0.5, skipped


def _spread_rows(n, d, seed, dtype):
    """Rows whose norms span ~1-900x: some 1536-row workgroups take the shared seed offset,
    others per-point offsets (csrc/assign16.hip), so a gathered row's workgroup offset almost
    never equals its full-pass one."""
    g = torch.Generator().manual_seed(seed)
    X = torch.randn(n, d, generator=g)
    X[: n // 2] *= 1.0 + 29.0 * torch.rand(n // 2, 1, generator=g)
    return X.to(dtype).to(DEV)


@pytest.mark.parametrize("d,k", [(64, 96), (128, 256), (256, 64), (512, 40), (64, 2048), (32, 1024), (128, 1024),
                                 (256, 512), (100, 77)])
def test_gathered_assign_with_seed_offsets_is_the_full_pass(native, d, k):
    """csrc/rows.hip seed_offsets + AssignArgs::oseed: a scattering gathered TOP2 assign over a
    random subset of rows writes bitwise the full pass's distances and labels at those rows --
    also where the full pass ranks by value (VARG: D=64 K>=2048, D=32 K>=1024), which the TOP2
    kernel then mirrors with its exact epilogue.  Without the offsets the distances differ."""
    from mikmeans.ops import pad_columns

    n = 120_000
    Xb = pad_columns(_spread_rows(n, d, d + k, torch.bfloat16))
    C = Xb[torch.randperm(n, generator=torch.Generator().manual_seed(k))[:k].to(DEV), :d].float() * 0.7
    pk = ops.pack_centers(C, Xb.shape[1], torch.bfloat16, DEV)
    xn = ops.row_sqnorm(Xb)
    lab_f = torch.empty(n, dtype=torch.int32, device=DEV)
    mind_f = torch.empty(n, device=DEV)
    pk.assign(Xb, xn, lab_f, mind_f)
    oseed = pk.seed_offsets(xn)
    g = torch.Generator().manual_seed(7)
    rows = torch.randperm(n, generator=g)[: n // 3].sort().values.to(DEV)
    out = {}
    for use in (True, False):
        lab = torch.full((n,), -1, dtype=torch.int32, device=DEV)
        mind = torch.full((n,), -1.0, device=DEV)
        ub = torch.zeros(n, device=DEV)
        lb = torch.zeros(n, device=DEV)
        slots = torch.zeros(native.NSLOT * native.SLOT_STRIDE, dtype=torch.float64, device=DEV)
        pk.assign(Xb, xn, lab, mind, slots, True, rows=rows, ub=ub, lb=lb, scatter=True,
                  oseed=oseed if use else None)
        out[use] = (lab, mind, ub, lb)
    lab, mind, ub, lb = out[True]
    assert torch.equal(lab[rows], lab_f[rows])
    assert torch.equal(mind[rows], mind_f[rows])
    assert bool((lb[rows] >= ub[rows]).all())
    # (the sensitivity check: the gathered workgroups' own offsets round the scores differently)
    assert not torch.equal(out[False][1][rows], mind_f[rows])


@pytest.mark.parametrize("dtype,d,k,init,spread", [
    (torch.bfloat16, 64, 96, "random", False),
    (torch.bfloat16, 128, 256, "random", True),
    (torch.bfloat16, 256, 64, "random", False),
    (torch.bfloat16, 128, 200, "k-means||", False),
    (torch.bfloat16, 64, 2048, "random", False),
    (torch.float32, 64, 100, "random", False),
    (torch.float32, 128, 64, "k-means||", True),
])
def test_bounded_trajectory_bitwise(native, dtype, d, k, init, spread):
    """30 Lloyd iterations with the bounded E-step and with the full one from the same start:
    labels, centres and changed counts equal bit for bit after every step, the inertia agrees
    (sums formula vs per-row distances), and the bounded engine re-assigns few rows late on."""
    from mikmeans.models.init import init_kmeans_parallel, init_random
    from mikmeans.parallel import Comm

    n = 400_000
    X = _spread_rows(n, d, k, dtype) if spread else B.make_blobs(n, d, k, seed=k, dtype=dtype, device=DEV)
    comm = Comm.local(torch.device(DEV))
    if init == "random":
        C0 = init_random(X, d, k, n, 0, comm, 3)
    else:
        C0 = init_kmeans_parallel(X, d, k, n, 0, comm, 3)
    ea = LloydEngine(X, k, comm=comm).set_centers(C0)
    eb = LloydEngine(X, k, comm=comm, bounded=True).set_centers(C0)
    re = []
    for it in range(30):
        ea.step()
        eb.step()
        sa, sb = ea.last_stats(), eb.last_stats()
        assert torch.equal(ea.labels, eb.labels), it
        assert torch.equal(ea.centers, eb.centers), it
        assert sa.n_changed == sb.n_changed, it
        assert sb.inertia == pytest.approx(sa.inertia, rel=1e-4), it
        re.append(eb.reassigned)
    print("reassigned per step", re)
    assert re[0] == n
    if not spread:      # (structureless rows keep every centre moving: no bound settles)
        assert min(re) < 0.6 * n, re


def test_kmeans_hamerly_fit(native):
    X = B.make_blobs(400_000, 64, 50, seed=2, dtype=torch.float32, device=DEV)
    ka = KMeans(50, init="random", seed=4, max_iter=40, tol=1e-6, device=DEV, algorithm="lloyd").fit(X)
    kb = KMeans(50, init="random", seed=4, max_iter=40, tol=1e-6, device=DEV, algorithm="hamerly").fit(X)
    assert kb._engine.bounded and not ka._engine.bounded
    assert kb.inertia_ == pytest.approx(ka.inertia_, rel=1e-5)
    assert torch.equal(kb.labels_, ka.labels_) and torch.equal(kb.cluster_centers_, ka.cluster_centers_)
    assert kb.n_iter_ == ka.n_iter_
    for ha, hb in zip(ka.history_, kb.history_):   # every step's inertia, from the M-step's sums
        assert hb["inertia"] == pytest.approx(ha["inertia"], rel=1e-5)
    re = [h["reassigned"] for h in kb.history_]
    assert re[0] == X.shape[0] and min(re) < X.shape[0] // 10
    assert KMeans(4, algorithm="elkan").algorithm == "hamerly"
    with pytest.raises(ValueError):
        KMeans(4, algorithm="bogus")


@pytest.mark.parametrize("n", [1, 15, 16, 4095, 4097, 1_000_003])
@pytest.mark.parametrize("density", [0.0, 0.003, 0.5, 1.0])
def test_compact_matches_nonzero(native, n, density):
    """csrc/rows.hip compaction: the flagged rows in ascending order and their count, both on
    the device, for ragged sizes (16-flag thread groups, 4096-flag blocks, a multi-slice scan)."""
    g = torch.Generator(device="cpu").manual_seed(n)
    cand = (torch.rand(n, generator=g) < density).to(torch.uint8).to(DEV)
    rows = torch.full((n,), -7, dtype=torch.int64, device=DEV)
    count = torch.full((1,), -1, dtype=torch.int64, device=DEV)
    scratch = torch.empty(max(1, native.compact_blocks(n)), dtype=torch.int64, device=DEV)
    native.compact(cand, rows, count, scratch)
    ref = torch.nonzero(cand).flatten()
    assert int(count) == ref.numel()
    assert torch.equal(rows[: ref.numel()], ref)


def test_device_count_assign_matches_host_count(native):
    """A gathered assign bounded by a device count equals the one over rows[:count]."""
    X = B.make_blobs(50_000, 64, 20, seed=1, dtype=torch.bfloat16, device=DEV)
    from mikmeans.ops import pad_columns

    X = pad_columns(X)
    pk = ops.pack_centers(X[:300, :64].float(), X.shape[1], torch.bfloat16, DEV)
    xn = ops.row_sqnorm(X)
    rows = torch.randperm(50_000, device=DEV)[:20_000].sort().values
    for m in (0, 1, 777, 20_000):
        out = []
        for use_count in (False, True):
            lab = torch.full((50_000,), 5, dtype=torch.int32, device=DEV)
            ub = torch.zeros(50_000, device=DEV)
            lb = torch.zeros(50_000, device=DEV)
            slots = torch.zeros(native.NSLOT * native.SLOT_STRIDE, dtype=torch.float64, device=DEV)
            if use_count:
                pk.assign(X, xn, lab, None, slots, True, rows=rows, ub=ub, lb=lb, scatter=True,
                          count=torch.tensor([m], dtype=torch.int64, device=DEV))
            elif m:
                pk.assign(X, xn, lab, None, slots, True, rows=rows[:m].contiguous(), ub=ub, lb=lb, scatter=True)
            out.append((lab, ub, lb, slot_totals(slots)[1]))
        a, b = out
        assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1]) and torch.equal(a[2], b[2]), m
        assert float(a[3]) == float(b[3])


def test_bounded_graph_replay_matches_eager(native):
    """The bounded E-step is sync-free, so it captures into the Lloyd hipGraph; replays give
    the eager bounded engine's centres and labels bit for bit, also across set_centers."""
    X = B.make_blobs(120_000, 64, 24, seed=5, dtype=torch.bfloat16, device=DEV)
    C0 = X[:24].float()
    ea = LloydEngine(X, 24, bounded=True).set_centers(C0)
    eb = LloydEngine(X, 24, bounded=True).set_centers(C0).capture()
    assert eb._graphs is not None, eb.capture_error
    for it in range(10):
        if it == 6:          # new centres: bounds invalidated by device writes the graph sees
            ea.set_centers(X[100:124].float())
            eb.set_centers(X[100:124].float())
        ea.step()
        eb.step()
        torch.cuda.synchronize()
        assert torch.equal(ea.centers, eb.centers), it
        assert torch.equal(ea.labels, eb.labels), it
        assert ea.reassigned == eb.reassigned, it


def test_scatter_assign_uses_row_norms(native):
    """A scattering gathered assign (the bounded E-step's) seeds each workgroup's keys from
    the caller norms at the X rows: on rows whose norms span 1-900x it gives bitwise the
    labels of the plain gathered assign fed the gathered norms (same workgroups, same
    offsets), (near-)optimal labels, and ub = the gathered assign's distance."""
    from mikmeans.ops import pad_columns

    n, d, k = 60_000, 64, 96
    g = torch.Generator().manual_seed(4)
    X = torch.randn(n, d, generator=g) * (1.0 + 29.0 * torch.rand(n, 1, generator=g))
    Xb = pad_columns(X.to(torch.bfloat16).to(DEV))
    C = X[:k].float() * 0.5
    pk = ops.pack_centers(C, Xb.shape[1], torch.bfloat16, DEV)
    xn = ops.row_sqnorm(Xb)
    rows = torch.randperm(n, generator=g)[: n // 2].sort().values.to(DEV)
    m = rows.numel()
    lab = torch.full((n,), -1, dtype=torch.int32, device=DEV)
    ub = torch.zeros(n, device=DEV)
    lb = torch.zeros(n, device=DEV)
    slots = torch.zeros(native.NSLOT * native.SLOT_STRIDE, dtype=torch.float64, device=DEV)
    pk.assign(Xb, xn, lab, None, slots, True, rows=rows, ub=ub, lb=lb, scatter=True)
    glab = torch.empty(m, dtype=torch.int32, device=DEV)
    gmind = torch.empty(m, device=DEV)
    pk.assign(Xb, xn[rows].contiguous(), glab, gmind, None, False, rows=rows)
    assert torch.equal(lab[rows], glab)
    assert bool((lab[torch.ones(n, dtype=torch.bool, device=DEV).index_fill_(0, rows, False)] == -1).all())
    torch.testing.assert_close(ub[rows], gmind.sqrt(), rtol=1e-6, atol=1e-6)
    r = rows.cpu()
    Xc = Xb[:, :d].float().cpu()[r]
    sc = ref.scores(Xb[:, :d].cpu()[r], C)          # (bf16 rows: against the bf16-quantised centres)
    got = sc.gather(1, glab.cpu().long()[:, None])[:, 0]
    best = sc.min(1).values
    # (a key resolves 2^-17 (|x - c|^2 + 3|x|^2) or better)
    scale = (Xc ** 2).sum(1) + (ref.quantize_centers(C, torch.bfloat16) ** 2).sum(1).max()
    assert int(((got - best) > 4e-5 * scale + 1e-6).sum()) == 0


@pytest.mark.parametrize("dtype,d", [(torch.bfloat16, 128), (torch.bfloat16, 40), (torch.float32, 77)])
def test_tighten_exact_distance(native, dtype, d):
    """Hamerly's tightening (csrc/rows.hip tighten_kernel): for the listed candidates ub
    becomes |x - C[label]| (f32 centres, direct sum of squares), the flag clears where that
    is below lb, unlisted and unassigned rows are untouched."""
    from mikmeans.ops import pad_columns

    n, k = 50_000, 37
    g = torch.Generator().manual_seed(d)
    X = pad_columns((torch.randn(n, d, generator=g) * 3).to(dtype).to(DEV))
    C = torch.zeros(k, X.shape[1], device=DEV)
    C[:, :d] = torch.randn(k, d, generator=g).to(DEV)
    lab = torch.randint(0, k, (n,), generator=g, dtype=torch.int32).to(DEV)
    lab[5] = -1
    rows = torch.randperm(n, generator=g)[:20_000].sort().values.to(DEV)
    rows[0] = 5
    rows = rows.sort().values
    count = torch.tensor([rows.numel() - 100], dtype=torch.int64, device=DEV)   # the tail is not listed
    ub = torch.full((n,), -1.0, device=DEV)
    lb = torch.where(torch.arange(n, device=DEV) % 2 == 0, torch.full((n,), 1e9, device=DEV),
                     torch.zeros(n, device=DEV))
    cand = torch.ones(n, dtype=torch.uint8, device=DEV)
    xn = ops.row_sqnorm(X)
    work = torch.zeros(4, device=DEV)        # (no shifts, |c|max 0: the slack is the rows' own)
    native.tighten(X, d, lab, C, rows, count, ub, lb, cand, xn, work, None)
    torch.cuda.synchronize()
    listed = rows[: int(count)]
    listed = listed[lab[listed] >= 0]
    Cq = C.to(dtype).double() if dtype == torch.bfloat16 else C.double()   # (the centres the assign ranks)
    ref = (X[listed, :d].double() - Cq[lab[listed].long(), :d]).norm(dim=1)
    torch.testing.assert_close(ub[listed].double(), ref, rtol=2e-6, atol=1e-6)
    even = (listed % 2 == 0)
    assert bool((cand[listed[even]] == 0).all()) and bool((cand[listed[~even]] == 1).all())
    mask = torch.ones(n, dtype=torch.bool, device=DEV)
    mask[listed] = False
    assert bool((ub[mask] == -1.0).all()) and bool((cand[mask] == 1).all())


@pytest.mark.parametrize("dtype,d,k,spherical,frozen", [
    (torch.float32, 40, 77, False, False),
    (torch.bfloat16, 96, 50, True, False),
    (torch.bfloat16, 64, 40, False, True),
])
def test_bounded_option_combinations(native, dtype, d, k, spherical, frozen):
    """The bounded E-step with ragged K / D, the cosine metric's sphere projection and frozen
    centres: it follows the full-E-step engine, and frozen centres never move."""
    n = 150_000
    X = B.make_blobs(n, d, 30, seed=k, dtype=dtype, device=DEV)
    if spherical:
        from mikmeans.ops import pad_columns

        X = pad_columns(X).clone()
        native.row_normalize(X)
        X = X[:, :d] if X.shape[1] != d else X
    C0 = X[:k, :d].float()
    fz = None
    if frozen:
        fz = torch.zeros(k, dtype=torch.int32, device=DEV)
        fz[::5] = 1
    ea = LloydEngine(X, k, spherical=spherical, frozen=fz, n_features=d).set_centers(C0)
    eb = LloydEngine(X, k, spherical=spherical, frozen=fz, n_features=d, bounded=True).set_centers(C0)
    assert eb.bounded
    for it in range(8):
        ea.step()
        eb.step()
        assert torch.equal(ea.labels, eb.labels), it
        assert torch.equal(ea.centers, eb.centers), it
    assert eb.inertia() == ea.inertia()
    if frozen:
        assert torch.equal(eb.centers[::5], C0[::5])


def test_bounded_incremental_mstep_bitwise(native):
    """Bounded E-step + incremental M-step (its changed-row list built over the candidates
    only, label_delta_rows) gives bitwise the bounded E-step + full M-step engine's centres
    and labels, across a centre reset too."""
    X = B.make_blobs(250_000, 64, 40, seed=8, dtype=torch.bfloat16, device=DEV)
    C0 = X[:48].float()
    ea = LloydEngine(X, 48, bounded=True, incremental=False).set_centers(C0)
    eb = LloydEngine(X, 48, bounded=True, incremental=True).set_centers(C0)
    assert eb.delta is not None
    for it in range(12):
        if it == 7:
            ea.set_centers(X[1000:1048].float())
            eb.set_centers(X[1000:1048].float())
        ea.step()
        eb.step()
        torch.cuda.synchronize()
        assert torch.equal(ea.labels, eb.labels), it
        assert torch.equal(ea.centers, eb.centers), it


@pytest.mark.parametrize("policy,weighted", [("farthest", False), ("keep", True), ("farthest", True)])
def test_bounded_weights_and_farthest_bitwise(native, policy, weighted):
    """Sample weights and the 'farthest' empty-cluster policy keep the bounded E-step (no
    fallback): bitwise the full engine's labels and centres, empty clusters relocated alike,
    and each step's inertia (weighted) from the sums."""
    n, d, k = 200_000, 64, 80
    X = B.make_blobs(n, d, 20, seed=11, dtype=torch.bfloat16, device=DEV)
    g = torch.Generator().manual_seed(5)
    w = (0.25 + 2 * torch.rand(n, generator=g)).to(DEV) if weighted else None
    C0 = X[:k].float()
    C0[-6:] = 1e3                      # far-away centres: empty after the first E-step
    ea = LloydEngine(X, k, sample_weight=w, empty_policy=policy).set_centers(C0)
    eb = LloydEngine(X, k, sample_weight=w, empty_policy=policy, bounded=True).set_centers(C0)
    assert eb.bounded
    for it in range(12):
        ea.step()
        eb.step()
        sa, sb = ea.last_stats(), eb.last_stats()
        assert torch.equal(ea.labels, eb.labels), it
        assert torch.equal(ea.centers, eb.centers), it
        assert sb.inertia == pytest.approx(sa.inertia, rel=1e-4), it
    if policy == "farthest":
        assert float(eb.centers[-6:].abs().max()) < 1e2     # relocated onto data rows


def test_bounded_graph_farthest_matches_eager(native):
    """Captured bounded steps with the 'farthest' policy (the eager relocation between the two
    graphs re-computes the distances the bounded E-step does not write) equal the eager ones."""
    X = B.make_blobs(100_000, 64, 16, seed=6, dtype=torch.bfloat16, device=DEV)
    C0 = X[:30].float()
    C0[-4:] = 5e2
    ea = LloydEngine(X, 30, empty_policy="farthest", bounded=True).set_centers(C0)
    eb = LloydEngine(X, 30, empty_policy="farthest", bounded=True).set_centers(C0).capture()
    assert eb._graphs is not None, eb.capture_error
    for it in range(8):
        ea.step()
        eb.step()
        assert torch.equal(ea.centers, eb.centers), it
        assert torch.equal(ea.labels, eb.labels), it
        assert ea.last_stats().inertia == eb.last_stats().inertia, it


@pytest.mark.parametrize("dtype,d,k,init", [(torch.bfloat16, 128, 256, "random"), (torch.bfloat16, 64, 96, "k-means||"),
                                            (torch.float32, 128, 64, "random"), (torch.float32, 64, 128, "k-means||")])
def test_auto_algorithm_is_bounded_and_equals_lloyd(native, dtype, d, k, init):
    """KMeans' default algorithm='auto' takes the bounded E-step where the bounds fit resident
    and gives 'lloyd's centres, labels and n_iter_ bit for bit; history_ carries the inertia."""
    X = B.make_blobs(300_000, d, k, seed=d + k, dtype=dtype, device=DEV)
    kw = dict(init=init, max_iter=40, tol=1e-6, seed=5, dtype=dtype)
    a = KMeans(k, **kw).fit(X)
    f = KMeans(k, algorithm="lloyd", **kw).fit(X)
    assert a.algorithm == "auto" and a.algorithm_ == "hamerly" and f.algorithm_ == "lloyd"
    assert a.n_iter_ == f.n_iter_
    assert torch.equal(a.cluster_centers_, f.cluster_centers_)
    assert torch.equal(a.labels_, f.labels_)
    assert a.inertia_ == f.inertia_
    assert len(a.history_) == a.n_iter_ and all(h["inertia"] > 0 for h in a.history_)
    for ha, hf in zip(a.history_, f.history_):
        assert ha["n_changed"] == hf["n_changed"]
        # (the bounded step's inertia comes from the sums, sxx + sum_k (n_k |c_k|^2 - 2 c_k.S_k), the
        # full step's from the per-row f32 scores: two roundings of the same quantity)
        assert ha["inertia"] == pytest.approx(hf["inertia"], rel=1e-4)
    # small problems stay on the full E-step
    s = KMeans(k, **kw).fit(X[:20_000])
    assert s.algorithm_ == "lloyd"
