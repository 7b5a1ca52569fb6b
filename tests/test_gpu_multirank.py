"""Multi-rank GPU execution on one MI355X: W = 2 / 4 / 8 processes share cuda:0 over a
host-staged gloo group (parallel/comm.py ``staged``) and run the real HIP kernels
through every distributed code path -- the reference's several participants meshed on one
board (app.mjs:70-118) -- and every case must give bitwise the W = 1 GPU result.

RCCL refuses two ranks on one GPU, so the collectives here go device -> host -> gloo; the
kernels, the sharding on the 1536-row grid, the k-means++ owner selection with real
non-owner ranks (csrc/kpp.hip mode 2), the memory-plan agreement, the per-rank device
sampler, the 'farthest' relocation across ranks and the W=2 -> W=4 resume are the ones
the 8-GPU RCCL job runs.  W = 8 is the target node's world size: one 1536-row grid unit per
rank (the last one short), five empty tail ranks on the small set, the 8-way owner draw, the
8-rank device sampler, and a W = 8 checkpoint resumed at W = 2.  One spawn per world size
runs all of its cases (each rank is a fresh process: ~5 s of start-up).
"""
import os

import pytest
import torch

from mikmeans.parallel import shard_range
from mikmeans.parallel.launch import spawn_local

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)

N, D, K = 12_000, 48, 24          # 8 units of the 1536-row grid: W=2 -> 4+4, W=4 -> 2+2+2+2, W=8 -> 1 each
N_EMPTY = 4_000                   # 3 units: at W=4 the last rank holds no rows, at W=8 the last five


def _data(dtype=torch.bfloat16, n=N, device=None):
    from mikmeans.data import blobs as B

    return B.make_blobs(n, D, K, seed=11, dtype=dtype, device=device or DEV)


def _shard(comm, X):
    s, e = shard_range(X.shape[0], comm.rank, comm.world)
    return X[s:e], s


def _far_init(X):
    C0 = X[:K].float().clone()
    C0[3:7] = 1.0e4                  # far-away centres: empty after the first E-step
    return C0


# ----------------------------------------------------------------------------- cases
def _lloyd(comm, dtype, init):
    from mikmeans.models.init import resolve_init
    from mikmeans.models.lloyd import LloydEngine

    X = _data(dtype)
    Xl, s = _shard(comm, X)
    C0 = resolve_init(init, Xl, D, K, N, s, comm, seed=3)
    eng = LloydEngine(Xl, K, comm=comm).set_centers(C0)
    eng.run(5, tol=-1, check_every=1)
    st = eng.last_stats()
    return {"C0": C0, "C": eng.centers.clone(), "labels": eng.labels.clone(), "counts": eng.counts.clone(),
            "inertia": st.inertia, "changed": st.n_changed}


def case_lloyd_random_bf16(comm):
    return _lloyd(comm, torch.bfloat16, "random")


def case_lloyd_random_f32(comm):
    return _lloyd(comm, torch.float32, "random")


def case_lloyd_kpp(comm):
    return _lloyd(comm, torch.bfloat16, "k-means++")


def case_kpp_greedy(comm):
    from mikmeans.models.init import init_kmeanspp
    from mikmeans.ops import pad_columns

    X = pad_columns(_data())
    Xl, s = _shard(comm, X)
    # world > 1: the owner path (all-gather of the potentials, kpp_sample mode 2 writes the
    # drawn row on its owner and zeros elsewhere, all-reduce of the L candidates)
    return {"C": init_kmeanspp(Xl, D, K, N, s, comm, seed=9, n_local_trials=3)}


def case_kpp_two_stage(comm):
    """sampling='two-stage': one all-gather per centre (the drawn rows ride with the
    potentials); rank-count dependent, so checked for replica agreement, not W=1 equality."""
    from mikmeans.models.init import init_kmeanspp
    from mikmeans.ops import pad_columns

    X = pad_columns(_data())
    Xl, s = _shard(comm, X)
    return {f"C{t}": init_kmeanspp(Xl, D, K, N, s, comm, seed=9, n_local_trials=t, sampling="two-stage")
            for t in (1, 3)}


def case_kpar(comm):
    """k-means||: candidates keyed by the global row -> the W=1 centres on real ranks."""
    from mikmeans.models.init import init_kmeans_parallel
    from mikmeans.ops import pad_columns

    X = pad_columns(_data())
    Xl, s = _shard(comm, X)
    return {"C": init_kmeans_parallel(Xl, D, K, N, s, comm, seed=6)}


def _fit(comm, **kw):
    import mikmeans

    X = _data(kw.pop("dtype_", torch.bfloat16))
    Xl, s = _shard(comm, X)
    w = None
    if kw.pop("weighted", False):
        i = torch.arange(N, device=DEV)
        w = (0.5 + (i % 7).float() / 7.0)[s : s + Xl.shape[0]]
    init = _far_init(X) if kw.pop("far", False) else "random"
    km = mikmeans.KMeans(K, init=init, dtype=X.dtype, max_iter=8, seed=2, comm=comm, **kw).fit(
        Xl, sample_weight=w)
    return {"C": km.cluster_centers_, "labels": km.labels_, "n_iter": km.n_iter_, "inertia": km.inertia_,
            "counts": km.counts_}


def case_fit_farthest(comm):
    return _fit(comm, far=True, empty_cluster="farthest")


def case_fit_weighted(comm):
    return _fit(comm, weighted=True)


def case_fit_cosine(comm):
    return _fit(comm, metric="cosine")


def case_fit_hamerly(comm):
    """The bounded E-step (bitwise the full one) on real ranks: every shard starts on the
    1536-row grid, so each row's full-pass seed offset is the W=1 one."""
    return _fit(comm, algorithm="hamerly")


def case_fit_graph(comm):
    """hipGraph replay with the host-staged collective between the graphs."""
    return _fit(comm, graph=True, incremental=False)


def _fit_kpp(comm):
    import mikmeans

    X = _data(torch.float32)
    Xl, _ = _shard(comm, X)
    km = mikmeans.KMeans(K, init="greedy-k-means++", n_local_trials=3, dtype="float32", max_iter=6, seed=4,
                         comm=comm).fit(Xl)
    return {"C": km.cluster_centers_, "labels": km.labels_}


def case_stream_agreement(comm):
    """Rank 1's HBM budget is below its resident need: every rank streams its (host) shard
    with the resident fit's result (memory-plan agreement, api.KMeans._memory_plan)."""
    import mikmeans
    from mikmeans.parallel import memplan

    X = _data().cpu()
    Xl, _ = _shard(comm, X)
    if comm.rank == 1:
        need = memplan.plan_resident(Xl.shape[0], D, K, torch.bfloat16, init="random").peak
        os.environ["MIKMEANS_HBM_BYTES"] = str(int(need * 0.9))
    try:
        km = mikmeans.KMeans(K, init="random", dtype="bfloat16", max_iter=8, seed=2, comm=comm,
                             device=DEV).fit(Xl)
    finally:
        os.environ.pop("MIKMEANS_HBM_BYTES", None)
    return {"C": km.cluster_centers_, "labels": km.labels_, "mode": km.memory_plan_["mode"]}


MB_B, MB_STEPS, MB_SEED = 1536, 6, 5


def case_minibatch_fit(comm):
    """MiniBatchKMeans.fit on a device-resident shard: every step's batch is drawn on the
    device (Philox keyed by (seed, rank, step), csrc/rows.hip) and read in place."""
    import mikmeans

    X = _data(torch.float32)
    Xl, _ = _shard(comm, X)
    km = mikmeans.MiniBatchKMeans(K, batch_size=MB_B, max_steps=MB_STEPS, init=X[:K].clone(), dtype="float32",
                                  seed=MB_SEED, comm=comm).fit(Xl)
    return {"C": km.cluster_centers_, "counts": km.counts_, "steps": km.n_steps_,
            "plan": km.memory_plan_["mode"]}


def case_fit_empty_shard(comm):
    import mikmeans

    X = _data(n=N_EMPTY)
    Xl, _ = _shard(comm, X)
    km = mikmeans.KMeans(K, init="random", dtype="bfloat16", max_iter=6, seed=2, comm=comm).fit(Xl)
    kp = mikmeans.KMeans(K, init="k-means++", dtype="bfloat16", max_iter=4, seed=3, comm=comm).fit(Xl)
    return {"C": km.cluster_centers_, "labels": km.labels_, "n": Xl.shape[0], "C_kpp": kp.cluster_centers_,
            "labels_kpp": kp.labels_}


def case_ckpt_save(comm, path):
    import mikmeans

    X = _data()
    Xl, _ = _shard(comm, X)
    mikmeans.KMeans(K, init="random", dtype="bfloat16", max_iter=3, tol=-1, seed=2, comm=comm,
                    checkpoint_every=1, checkpoint_dir=path).fit(Xl)
    return {}


def case_ckpt_resume(comm, path):
    import mikmeans

    X = _data()
    Xl, _ = _shard(comm, X)
    km = mikmeans.KMeans(K, init="random", dtype="bfloat16", max_iter=8, tol=-1, seed=2, comm=comm).fit(
        Xl, resume_from=path)
    return {"C": km.cluster_centers_, "labels": km.labels_}


CASES = {f.__name__[5:]: f for f in (case_lloyd_random_bf16, case_lloyd_random_f32, case_lloyd_kpp,
                                     case_kpp_greedy, case_fit_farthest, case_fit_weighted, case_fit_cosine,
                                     case_fit_graph, case_stream_agreement, case_minibatch_fit,
                                     case_fit_empty_shard, case_kpp_two_stage, case_kpar, case_fit_hamerly)}
CASES["fit_kpp_greedy_f32"] = _fit_kpp


def _suite(comm, names, extra):
    out = {n: CASES[n](comm) for n in names}
    if extra:
        fn, arg = extra
        out[fn] = {"ckpt_save": case_ckpt_save, "ckpt_resume": case_ckpt_resume}[fn](comm, arg)
    comm.barrier()
    return out


# ------------------------------------------------------------------ W = 1 references
def _local():
    from mikmeans.parallel import Comm

    return Comm.local(DEV)


@pytest.fixture(scope="module")
def refs(native):
    torch.cuda.set_device(DEV)
    return {n: f(_local()) for n, f in CASES.items() if n not in ("minibatch_fit", "stream_agreement")}


def _mb_reference(world):
    """The W-rank mini-batch fit as one rank: step s's batch is the ranks' draws in rank
    order (each rank's Philox rows offset by its shard start); the integer M-step makes the
    summed messages exact, so the centres must be bitwise the W-rank fit's."""
    from mikmeans.models.minibatch import MiniBatchEngine
    from mikmeans.ops import col_stats, native

    C = native.require()
    X = _data(torch.float32)
    # (a rank draws min(batch_size, its rows): W=8's short last shard draws 1248)
    bs = [min(MB_B, shard_range(N, r, world)[1] - shard_range(N, r, world)[0]) for r in range(world)]
    eng = MiniBatchEngine(K, D, sum(bs), dtype=torch.float32, device=DEV, comm=_local())
    eng.set_bound(col_stats(X, stats=False).absmax)
    eng.set_centers(X[:K].clone())
    for s in range(MB_STEPS):
        parts = []
        for r in range(world):
            r0, r1 = shard_range(N, r, world)
            rows = torch.empty(bs[r], dtype=torch.int64, device=DEV)
            C.sample_index(r1 - r0, bs[r], MB_SEED, r, s, rows)
            parts.append(rows + r0)
        eng.partial_fit_rows(X, torch.cat(parts))
    return eng.centers.clone().cpu(), eng.vcount.clone().cpu()


def _cat_labels(outs, key="labels"):
    return torch.cat([o[key].cpu() for o in outs])


def _check_lloyd(ref, outs):
    for o in outs:     # centres replicated bit-identically
        assert torch.equal(o["C"], outs[0]["C"])
    assert torch.equal(outs[0]["C0"], ref["C0"].cpu())
    assert torch.equal(outs[0]["C"], ref["C"].cpu())
    assert torch.equal(_cat_labels(outs), ref["labels"].cpu())
    assert torch.equal(outs[0]["counts"], ref["counts"].cpu())
    assert outs[0]["changed"] == ref["changed"]
    assert outs[0]["inertia"] == pytest.approx(ref["inertia"], rel=1e-9)


def _check_fit(ref, outs):
    for o in outs:
        assert torch.equal(o["C"], outs[0]["C"])
    assert torch.equal(outs[0]["C"], ref["C"].cpu())
    assert torch.equal(_cat_labels(outs), ref["labels"].cpu())
    assert outs[0]["n_iter"] == ref["n_iter"]
    assert outs[0]["inertia"] == pytest.approx(ref["inertia"], rel=1e-9)


def _check(name, ref, outs):
    if name.startswith("lloyd"):
        _check_lloyd(ref, outs)
    elif name in ("kpp_greedy", "kpar"):
        for o in outs:
            assert torch.equal(o["C"], ref["C"].cpu())
    elif name == "fit_kpp_greedy_f32":
        assert torch.equal(outs[0]["C"], ref["C"].cpu())
        assert torch.equal(_cat_labels(outs), ref["labels"].cpu())
    else:
        _check_fit(ref, outs)


W2_CASES = ["lloyd_random_bf16", "lloyd_random_f32", "lloyd_kpp", "kpp_greedy", "fit_farthest", "fit_weighted",
            "fit_cosine", "fit_graph", "fit_kpp_greedy_f32", "stream_agreement", "minibatch_fit",
            "kpp_two_stage", "kpar"]
W4_CASES = ["lloyd_random_bf16", "lloyd_kpp", "kpp_greedy", "fit_farthest", "fit_weighted", "minibatch_fit",
            "fit_empty_shard", "kpp_two_stage", "kpar"]
W8_CASES = ["lloyd_random_bf16", "lloyd_random_f32", "lloyd_kpp", "kpp_greedy", "fit_farthest", "fit_weighted",
            "fit_hamerly", "minibatch_fit", "fit_empty_shard", "kpp_two_stage", "kpar"]
_NOT_W1 = ("minibatch_fit", "stream_agreement", "fit_empty_shard", "kpp_two_stage")


@pytest.fixture(scope="module")
def w2(refs, tmp_path_factory):
    path = str(tmp_path_factory.mktemp("ck") / "run")
    outs = spawn_local(_suite, 2, W2_CASES, ("ckpt_save", path), device="cuda", timeout=600)
    return outs, path


@pytest.fixture(scope="module")
def w4(w2):
    _, path = w2
    return spawn_local(_suite, 4, W4_CASES, ("ckpt_resume", path), device="cuda", timeout=600)


@pytest.fixture(scope="module")
def w8(w4, tmp_path_factory):
    """Eight ranks on cuda:0 (the 8-GPU node's world size; 8 of the box's 16 GPU processes),
    saving a checkpoint after three iterations that a W = 2 spawn then resumes."""
    path = str(tmp_path_factory.mktemp("ck8") / "run")
    outs = spawn_local(_suite, 8, W8_CASES, ("ckpt_save", path), device="cuda", timeout=900)
    back = spawn_local(_suite, 2, [], ("ckpt_resume", path), device="cuda", timeout=600)
    return outs, back


@pytest.mark.parametrize("name", [n for n in W2_CASES if n not in _NOT_W1])
def test_w2_equals_w1(refs, w2, name):
    outs, _ = w2
    _check(name, refs[name], [o[name] for o in outs])


@pytest.mark.parametrize("name", [n for n in W4_CASES if n not in _NOT_W1])
def test_w4_equals_w1(refs, w4, name):
    _check(name, refs[name], [o[name] for o in w4])


@pytest.mark.parametrize("name", [n for n in W8_CASES if n not in _NOT_W1])
def test_w8_equals_w1(refs, w8, name):
    _check(name, refs[name], [o[name] for o in w8[0]])


def test_w8_grid_and_empty_tail_ranks(w8):
    """The W=8 shards: one 1536-row unit per rank (the last short) on the 12k set, and on the
    4k set only ranks 0-2 hold rows -- the empty tail ranks still join every collective."""
    outs, _ = w8
    assert [shard_range(N, r, 8)[1] - shard_range(N, r, 8)[0] for r in range(8)] == [1536] * 7 + [1248]
    assert [o["fit_empty_shard"]["n"] for o in outs] == [1536, 1536, 928, 0, 0, 0, 0, 0]


def test_checkpoint_w8_resumed_at_w2(w8):
    """Three iterations at W=8, checkpointed; resumed at W=2 to iteration 8: the W=1 run's
    eight-iteration centres and labels."""
    import mikmeans

    ref = mikmeans.KMeans(K, init="random", dtype="bfloat16", max_iter=8, tol=-1, seed=2, comm=_local()).fit(
        _data())
    res = [o["ckpt_resume"] for o in w8[1]]
    assert torch.equal(res[0]["C"], ref.cluster_centers_.cpu())
    assert torch.equal(_cat_labels(res), ref.labels_.cpu())


@pytest.mark.parametrize("world", [2, 4, 8])
def test_kpp_two_stage_replicas(refs, w2, w4, w8, world):
    """Two-stage k-means++ on real ranks: every rank holds the same centres, each one a data
    row, none drawn twice; at W = 1 it is the exact path (refs)."""
    from mikmeans.ops import pad_columns

    res = [o["kpp_two_stage"] for o in {2: w2[0], 4: w4, 8: w8[0]}[world]]
    X = pad_columns(_data()).float().cpu()[:, :D]
    for t in (1, 3):
        for r in res:
            assert torch.equal(r[f"C{t}"], res[0][f"C{t}"])
        C = res[0][f"C{t}"].cpu()
        assert bool((C[:, None, :] == X[None]).all(-1).any(1).all()) and torch.unique(C, dim=0).shape[0] == K
    assert torch.equal(refs["kpp_two_stage"]["C3"].cpu(), refs["kpp_greedy"]["C"].cpu())


def test_w2_stream_agreement(w2):
    """One rank over its budget: both ranks stream, and the model is the resident W=1 fit's."""
    import mikmeans

    outs, _ = w2
    res = [o["stream_agreement"] for o in outs]
    assert [r["mode"] for r in res] == ["streaming", "streaming"]
    ref = mikmeans.KMeans(K, init="random", dtype="bfloat16", max_iter=8, seed=2, comm=_local()).fit(_data())
    assert torch.equal(res[0]["C"], ref.cluster_centers_.cpu())
    assert torch.equal(_cat_labels(res), ref.labels_.cpu())


@pytest.mark.parametrize("world", [2, 4, 8])
def test_minibatch_device_sampler(w2, w4, w8, world):
    outs = {2: w2[0], 4: w4, 8: w8[0]}[world]
    res = [o["minibatch_fit"] for o in outs]
    C_ref, v_ref = _mb_reference(world)
    for r in res:
        assert r["plan"] == "minibatch-resident" and r["steps"] == MB_STEPS
        assert torch.equal(r["C"], res[0]["C"])
    assert torch.equal(res[0]["C"], C_ref)
    assert torch.equal(res[0]["counts"].double(), v_ref)


@pytest.mark.parametrize("world", [4, 8])
def test_empty_shard(refs, w4, w8, world):
    res = [o["fit_empty_shard"] for o in (w4 if world == 4 else w8[0])]
    ref = refs["fit_empty_shard"]
    assert [r["n"] for r in res][-1] == 0
    for key, lab in (("C", "labels"), ("C_kpp", "labels_kpp")):
        for r in res:
            assert torch.equal(r[key], ref[key].cpu())
        assert torch.equal(_cat_labels(res, lab), ref[lab].cpu())


def test_checkpoint_w2_resumed_at_w4(w4):
    """Three iterations at W=2, checkpointed; resumed at W=4 to iteration 8: the W=1 run's
    eight-iteration centres and labels."""
    import mikmeans

    ref = mikmeans.KMeans(K, init="random", dtype="bfloat16", max_iter=8, tol=-1, seed=2, comm=_local()).fit(
        _data())
    res = [o["ckpt_resume"] for o in w4]
    assert torch.equal(res[0]["C"], ref.cluster_centers_.cpu())
    assert torch.equal(_cat_labels(res), ref.labels_.cpu())
