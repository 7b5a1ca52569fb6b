"""Data-parallel correctness on CPU ranks (gloo): W ranks must reproduce the 1-rank result.

Same code paths as the RCCL/xGMI GPU job (packed f64 all-reduce per iteration,
k-means++ owner selection, checkpoint broadcast), only the backend differs.
"""
import numpy as np
import pytest
import torch

from mikmeans.parallel import shard_range
from mikmeans.parallel.launch import spawn_local

N, D, K = 6000, 8, 12


def _data():
    from mikmeans.data import blobs as B

    return B.make_blobs(N, D, K, seed=21)


def _lloyd(comm, init, iters):
    from mikmeans.models.init import resolve_init
    from mikmeans.models.lloyd import LloydEngine

    X = _data()
    s, e = shard_range(N, comm.rank, comm.world)
    Xl = X[s:e]
    C0 = resolve_init(init, Xl, D, K, N, s, comm, seed=3)
    eng = LloydEngine(Xl, K, comm=comm).set_centers(C0)
    eng.run(iters, tol=-1, check_every=1)
    st = eng.last_stats()
    return {"C0": C0, "C": eng.centers.clone(), "labels": eng.labels.clone(), "inertia": st.inertia,
            "changed": st.n_changed, "counts": eng.counts.clone()}


def _single(init, iters):
    from mikmeans.parallel import Comm

    return _lloyd(Comm.local(), init, iters)


@pytest.mark.parametrize("world,init", [(2, "random"), (2, "k-means++"), (3, "random"), (3, "k-means++"),
                                        (4, "k-means++"), (8, "random"), (8, "k-means++")])
def test_lloyd_dp_equals_single_rank(world, init):
    """W = 2/3/4/8 gloo ranks (the 1/2/4/8-GPU job's code path, backend aside)."""
    ref = _single(init, 6)
    outs = spawn_local(_lloyd, world, init, 6)
    for o in outs:  # centroids are replicated bit-identically on every rank
        assert torch.equal(o["C"], outs[0]["C"])
        assert torch.equal(o["C0"], ref["C0"])
    torch.testing.assert_close(outs[0]["C"], ref["C"], rtol=1e-5, atol=1e-5)
    assert torch.equal(torch.cat([o["labels"] for o in outs]), ref["labels"])
    assert outs[0]["inertia"] == pytest.approx(ref["inertia"], rel=1e-9)
    assert outs[0]["changed"] == ref["changed"]
    assert torch.equal(outs[0]["counts"], ref["counts"])


def _fit_api(comm):
    import mikmeans

    X = _data()
    s, e = shard_range(N, comm.rank, comm.world)
    km = mikmeans.KMeans(K, comm=comm, device="cpu", seed=1, max_iter=50).fit(X[s:e])
    return {"C": km.cluster_centers_, "inertia": km.inertia_, "n_iter": km.n_iter_, "labels": km.labels_}


def test_kmeans_api_distributed():
    from mikmeans.parallel import Comm
    import mikmeans

    X = _data()
    ref = mikmeans.KMeans(K, comm=Comm.local(), device="cpu", seed=1, max_iter=50).fit(X)
    outs = spawn_local(_fit_api, 2)
    torch.testing.assert_close(outs[0]["C"], ref.cluster_centers_, rtol=1e-5, atol=1e-5)
    assert outs[0]["inertia"] == pytest.approx(ref.inertia_, rel=1e-7)
    assert outs[0]["n_iter"] == ref.n_iter_
    assert torch.equal(torch.cat([o["labels"] for o in outs]), ref.labels_)


def _minibatch(comm, steps):
    from mikmeans.data.blobs import BlobStream
    from mikmeans.models.minibatch import MiniBatchEngine

    b = 256 // comm.world
    stream = BlobStream(10**6, D, K, b, seed=4, rank=comm.rank, world=comm.world)
    eng = MiniBatchEngine(K, D, b, comm=comm)
    from mikmeans.data.blobs import blob_centers

    eng.set_centers(blob_centers(K, D, 10.0, 4) + 0.5)
    for _ in range(steps):
        eng.partial_fit(next(stream))
    return {"C": eng.centers.clone(), "v": eng.vcount.clone()}


def test_minibatch_dp_equals_single_rank():
    from mikmeans.parallel import Comm

    ref = _minibatch(Comm.local(), 10)
    outs = spawn_local(_minibatch, 2, 10)
    torch.testing.assert_close(outs[0]["C"], ref["C"], rtol=1e-5, atol=1e-5)
    assert torch.equal(outs[0]["v"], ref["v"])


def _ckpt(comm, path):
    from mikmeans.utils.checkpoint import load_checkpoint, save_checkpoint

    C = torch.arange(12, dtype=torch.float32).reshape(3, 4) * (1 + comm.rank)  # only rank 0's is saved
    save_checkpoint(path, C, 7, {"n_clusters": 3}, comm=comm)
    st = load_checkpoint(path, comm=comm)
    return {"C": st["centers"], "it": st["iteration"], "world": st["world_size"]}


def test_checkpoint_broadcast(tmp_path):
    outs = spawn_local(_ckpt, 2, str(tmp_path / "ck"))
    for o in outs:
        assert torch.equal(o["C"], torch.arange(12, dtype=torch.float32).reshape(3, 4))
        assert o["it"] == 7 and o["world"] == 2


def _collectives(comm):
    t = torch.tensor([float(comm.rank + 1)], dtype=torch.float64)
    comm.allreduce_(t)
    m = torch.tensor([float(comm.rank)])
    comm.allreduce_max_(m)
    g = comm.all_gather(torch.tensor([comm.rank, 10 * comm.rank]))
    o = comm.all_gather_object({"r": comm.rank})
    b = comm.broadcast_object("hello" if comm.rank == 0 else None)
    comm.barrier()
    return {"sum": t.item(), "max": m.item(), "g": g, "o": [x["r"] for x in o], "b": b}


def test_comm_collectives_world4():
    outs = spawn_local(_collectives, 4)
    for o in outs:
        assert o["sum"] == 10 and o["max"] == 3 and o["b"] == "hello"
        assert o["g"].tolist() == [[0, 0], [1, 10], [2, 20], [3, 30]] and o["o"] == [0, 1, 2, 3]


def _minibatch_fit_uneven(comm):
    import mikmeans

    n = 1025
    X = _data()[:n]
    s, e = shard_range(n, comm.rank, comm.world, align=1)   # shards of 342 / 342 / 341 rows
    km = mikmeans.MiniBatchKMeans(4, batch_size=64, max_iter=1, seed=2, comm=comm).fit(X[s:e])
    return {"C": km.cluster_centers_.clone(), "steps": km.n_steps_}


def test_minibatch_fit_uneven_shards_same_step_count():
    """Ranks with different shard sizes must issue the same number of step collectives
    (steps came from the rank-local n and could deadlock)."""
    outs = spawn_local(_minibatch_fit_uneven, 3)
    assert len({o["steps"] for o in outs}) == 1
    for o in outs:
        assert torch.equal(o["C"], outs[0]["C"])


def _minibatch_tol(comm, tol):
    import mikmeans

    n = 1025
    X = _data()[:n]
    s, e = shard_range(n, comm.rank, comm.world, align=1)
    km = mikmeans.MiniBatchKMeans(4, batch_size=64, max_iter=3, seed=2, comm=comm, tol=tol).fit(X[s:e])
    return {"C": km.cluster_centers_.clone(), "steps": km.n_steps_}


@pytest.mark.parametrize("world", [2, 3])
def test_minibatch_tol_stops_every_rank_together(world):
    """The mini-batch tolerance check reads the replicated centre shift, so every rank stops
    at the same step (the first check, with a huge tol) and keeps the same centres; tol=0
    runs all max_iter epochs."""
    stop = spawn_local(_minibatch_tol, world, 1e30)
    full = spawn_local(_minibatch_tol, world, 0.0)
    assert {o["steps"] for o in stop} == {10}
    assert len({o["steps"] for o in full}) == 1 and full[0]["steps"] > 10
    for o in stop:
        assert torch.equal(o["C"], stop[0]["C"])


def _kpp(comm, trials):
    from mikmeans.models.init import init_kmeanspp

    X = _data()
    s, e = shard_range(N, comm.rank, comm.world)
    return init_kmeanspp(X[s:e], D, K, N, s, comm, seed=9, n_local_trials=trials)


@pytest.mark.parametrize("trials", [1, 3])
def test_kmeanspp_world_size_invariant(trials):
    """k-means++ (plain and greedy, one all-gather + one all-reduce of all L candidate rows
    per step) gives the 1-rank centres bit for bit on W = 2/4/8 gloo ranks, empty shards
    included (N=6000 covers 4 units of the 1536-row grid)."""
    from mikmeans.parallel import Comm

    ref = _kpp(Comm.local(), trials)
    for world in (2, 4, 8):
        outs = spawn_local(_kpp, world, trials)
        for o in outs:
            assert torch.equal(o, ref), (world, trials)


def _kpp2(comm, trials):
    from mikmeans.models.init import init_kmeanspp

    X = _data()
    s, e = shard_range(N, comm.rank, comm.world)
    return init_kmeanspp(X[s:e], D, K, N, s, comm, seed=9, n_local_trials=trials, sampling="two-stage")


@pytest.mark.parametrize("trials", [1, 3])
def test_kmeanspp_two_stage(trials):
    """sampling='two-stage' (one all-gather per centre): every rank holds the same centres,
    each a data row, no row drawn twice; W = 1 gives the exact path's centres; empty
    shards (W = 8 over 6000 rows) never win a draw."""
    from mikmeans.parallel import Comm

    X = _data()
    ref = _kpp(Comm.local(), trials)
    assert torch.equal(_kpp2(Comm.local(), trials), ref)
    for world in (2, 8):
        outs = spawn_local(_kpp2, world, trials)
        for o in outs:
            assert torch.equal(o, outs[0]), (world, trials)
        C = outs[0]
        hit = (C[:, None, :] == X.float()[None, :, :C.shape[1]]).all(-1).any(1)
        assert bool(hit.all()) and torch.unique(C, dim=0).shape[0] == K


def _kpar(comm):
    from mikmeans.models.init import init_kmeans_parallel

    X = _data()
    s, e = shard_range(N, comm.rank, comm.world)
    return init_kmeans_parallel(X[s:e], D, K, N, s, comm, seed=4)


def test_kmeans_parallel_world_size_invariant():
    """k-means||: candidates keyed by the global row, gathered in row order, integer weights
    -> the same centres on W = 1 / 2 / 3 gloo ranks (empty-ish shards included)."""
    from mikmeans.parallel import Comm

    ref = _kpar(Comm.local())
    assert ref.shape == (K, D)
    for world in (2, 3):
        outs = spawn_local(_kpar, world)
        for o in outs:
            assert torch.equal(o, ref), world


def test_pick_rank_is_proportional():
    """pick_rank(totals, v) selects rank r with probability totals[r] / sum (inverse CDF),
    never an empty rank, and the rounding edge (v -> 1) lands on the last non-empty rank."""
    from mikmeans.models.init import pick_rank

    tots = torch.tensor([3.0, 0.0, 1.0, 4.0, 0.0], dtype=torch.float64)
    v = (torch.arange(80_000, dtype=torch.float64) + 0.5) / 80_000
    got = torch.bincount(torch.stack([pick_rank(tots, x) for x in v[::8]]), minlength=5).double()
    freq = got / got.sum()
    assert torch.allclose(freq, tots / tots.sum(), atol=2e-3) and got[1] == 0 and got[4] == 0
    assert int(pick_rank(tots, torch.tensor(1.0, dtype=torch.float64))) == 3
    assert int(pick_rank(tots, torch.tensor(0.0, dtype=torch.float64))) == 0


def test_two_stage_draw_distribution():
    """The two-stage draw is the D^2 distribution: with 2 shards and a fixed first centre,
    the second centre's frequency over many seeds matches d2_i / sum d2 (chi-square-ish)."""
    from mikmeans.models.init import _draw, pick_rank

    g = torch.Generator().manual_seed(0)
    X = torch.randn(12, 2, generator=g)
    d2 = ((X - X[0]) ** 2).sum(1).double()
    shards = [(0, 5), (5, 12)]
    cs = [torch.cumsum(d2[a:b], 0) for a, b in shards]
    tots = torch.stack([c[-1] for c in cs])
    rng = torch.Generator().manual_seed(1)
    trials = 60_000
    u = torch.rand(trials, generator=rng, dtype=torch.float64)
    v = torch.rand(trials, generator=rng, dtype=torch.float64)
    hits = torch.zeros(12, dtype=torch.float64)
    for j in range(trials):
        r = int(pick_rank(tots, v[j]))
        a, b = shards[r]
        hits[a + _draw(cs[r], d2[a:b], float(u[j]) * float(cs[r][-1]))] += 1
    p = d2 / d2.sum()
    assert hits[0] == 0
    assert torch.allclose(hits / trials, p, atol=0.006)
