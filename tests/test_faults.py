"""Failure injection + elastic resume: kill a rank mid-fit, resume
from the last checkpoint with a different world size, get the no-fault result."""
import pytest
import torch

from mikmeans.parallel import shard_range
from mikmeans.parallel.launch import spawn_local

N, D, K, ITERS = 5000, 6, 10, 8


def _fit(comm, ckdir, resume):
    from mikmeans import KMeans
    from mikmeans.data.blobs import make_blobs

    X = make_blobs(N, D, K, std=4.0, seed=11)
    s, e = shard_range(N, comm.rank, comm.world)
    km = KMeans(K, init="k-means++", seed=2, max_iter=ITERS, tol=-1.0, device="cpu", comm=comm,
                checkpoint_every=2, checkpoint_dir=ckdir)
    km.fit(X[s:e], resume_from=ckdir if resume else None)
    return {"C": km.cluster_centers_, "n_iter": km.n_iter_, "inertia": km.inertia_}


def test_rank_failure_then_resume_with_other_world(tmp_path, monkeypatch):
    from mikmeans.parallel import Comm

    ref = _fit(Comm.local(), str(tmp_path / "ref"), False)
    ck = str(tmp_path / "ck")
    monkeypatch.setenv("MIKMEANS_FAULT", "1:5")
    with pytest.raises(Exception):
        spawn_local(_fit, 2, ck, False)
    monkeypatch.delenv("MIKMEANS_FAULT")
    from mikmeans.utils.checkpoint import load_checkpoint

    assert load_checkpoint(ck)["iteration"] == 4          # last checkpoint before the fault
    res = spawn_local(_fit, 3, ck, True)
    # the reference must run every iteration (labels still changing), so the resumed runs
    # are compared over the same trajectory
    assert ref["n_iter"] == ITERS
    for r in res:
        assert r["n_iter"] == ITERS
        assert torch.equal(r["C"], ref["C"])           # exact: integer-sum M-step, any world size
        assert r["inertia"] == pytest.approx(ref["inertia"], rel=1e-12)


def _mb_stream(comm, ckdir, resume, batch_global, steps):
    from mikmeans import MiniBatchKMeans
    from mikmeans.data.blobs import BlobStream

    b = batch_global // comm.world
    st = BlobStream(10**6, 8, 6, b, std=2.0, seed=3, rank=comm.rank, world=comm.world)
    km = MiniBatchKMeans(6, batch_size=b, seed=1, comm=comm, init="random", device="cpu")
    km.fit_stream(st, steps, resume_from=ckdir if resume else None, checkpoint_every=2, checkpoint_dir=ckdir)
    return {"C": km.cluster_centers_, "steps": km.n_steps_, "counts": km.counts_}


def test_minibatch_stream_failure_then_resume_with_other_world(tmp_path, monkeypatch):
    """Kill a rank mid-stream (W=2), resume from the last checkpoint on W=4 with the same
    global batch: the stream replays the same rows per step, the centres match the
    uninterrupted single-rank run bit for bit."""
    from mikmeans.parallel import Comm
    from mikmeans.utils.checkpoint import load_checkpoint

    ref = _mb_stream(Comm.local(), str(tmp_path / "ref"), False, 1024, 10)
    ck = str(tmp_path / "ck")
    monkeypatch.setenv("MIKMEANS_FAULT", "1:5")
    with pytest.raises(Exception):
        spawn_local(_mb_stream, 2, ck, False, 1024, 10)
    monkeypatch.delenv("MIKMEANS_FAULT")
    st = load_checkpoint(ck)
    assert st["iteration"] == 4 and st["kind"] == "minibatch" and st["stream_pos"] == 5 * 1024
    res = spawn_local(_mb_stream, 4, ck, True, 1024, 10)
    for r in res:
        assert r["steps"] == 10
        assert torch.equal(r["C"], ref["C"])
        assert torch.equal(r["counts"], ref["counts"])


def test_minibatch_save_load_roundtrip(tmp_path):
    import mikmeans
    from mikmeans.data.blobs import make_blobs

    X = make_blobs(4096, 5, 4, seed=2)
    km = mikmeans.MiniBatchKMeans(4, batch_size=512, seed=0, device="cpu").fit(X)
    km.save(tmp_path / "mb")
    km2 = mikmeans.MiniBatchKMeans.load(tmp_path / "mb", device="cpu")
    assert torch.equal(km2.cluster_centers_, km.cluster_centers_)
    assert torch.equal(km2.counts_, km.counts_) and km2.n_steps_ == km.n_steps_
    km.partial_fit(X[:512])
    km2.partial_fit(X[:512])
    assert torch.equal(km2.cluster_centers_, km.cluster_centers_)


def _mb_fit(comm, ckdir, resume):
    from mikmeans import MiniBatchKMeans
    from mikmeans.data.blobs import make_blobs

    X = make_blobs(6000, 5, 6, std=2.0, seed=4)
    s, e = shard_range(6000, comm.rank, comm.world)
    km = MiniBatchKMeans(6, batch_size=256, max_steps=12, seed=5, comm=comm, init="random", device="cpu")
    km.fit(X[s:e], resume_from=ckdir if resume else None, checkpoint_every=3, checkpoint_dir=ckdir)
    return {"C": km.cluster_centers_, "steps": km.n_steps_, "counts": km.counts_}


def test_minibatch_fit_failure_then_resume(tmp_path, monkeypatch):
    """MiniBatchKMeans.fit on tensors: batch rows are drawn from a generator keyed by
    (seed, rank, step), so the checkpointed step is the whole sampler state and a job
    killed mid-fit resumes to the uninterrupted fit's centres bit for bit."""
    from mikmeans.utils.checkpoint import load_checkpoint

    ref = spawn_local(_mb_fit, 2, str(tmp_path / "ref"), False)
    ck = str(tmp_path / "ck")
    monkeypatch.setenv("MIKMEANS_FAULT", "0:7")
    with pytest.raises(Exception):
        spawn_local(_mb_fit, 2, ck, False)
    monkeypatch.delenv("MIKMEANS_FAULT")
    st = load_checkpoint(ck)
    assert st["iteration"] == 6 and st["rng"]["step"] == 6 and st["rng"]["seed"] == 5
    res = spawn_local(_mb_fit, 2, ck, True)
    for r in res:
        assert r["steps"] == 12
        assert torch.equal(r["C"], ref[0]["C"])
        assert torch.equal(r["counts"], ref[0]["counts"])


def test_minibatch_refit_runs_all_steps():
    import mikmeans
    from mikmeans.data.blobs import make_blobs

    X = make_blobs(3000, 4, 3, seed=9)
    km = mikmeans.MiniBatchKMeans(3, batch_size=128, max_steps=5, seed=1, device="cpu")
    a = km.fit(X).cluster_centers_.clone()
    assert km.n_steps_ == 5
    assert torch.equal(km.fit(X).cluster_centers_, a) and km.n_steps_ == 5
