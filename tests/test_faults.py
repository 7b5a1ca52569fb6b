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
    if ref["n_iter"] == ITERS:
        for r in res:
            assert r["n_iter"] == ITERS
            assert torch.equal(r["C"], ref["C"])           # exact: integer-sum M-step, any world size
            assert r["inertia"] == pytest.approx(ref["inertia"], rel=1e-12)
