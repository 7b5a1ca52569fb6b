"""Mini-batch k-means on the device: the Philox row sampler (csrc/rows.hip) against its NumPy
mirror, device-resident vs host-resident shards (same rows, same model), host syncs per
step, and the helper kernels of the cosine / weighted paths."""
import numpy as np
import pytest
import torch

import mikmeans
from mikmeans.data import blobs as B
from mikmeans.data.sampler import sample_indices

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("dtype,D", [(torch.bfloat16, 256), (torch.float32, 20), (torch.bfloat16, 40)])
def test_sample_rows_matches_numpy_mirror(native, dtype, D):
    from mikmeans.ops import pad_columns

    n, b = 123_457, 50_001
    X = pad_columns(B.make_blobs(n, D, 16, seed=3, dtype=dtype, device=DEV))
    out = torch.empty((b, X.shape[1]), dtype=dtype, device=DEV)
    xn = torch.empty(b, dtype=torch.float32, device=DEV)
    idx = torch.empty(b, dtype=torch.int64, device=DEV)
    for step, rank in ((0, 0), (7, 3), (2**31 + 5, 1)):
        native.sample_rows(X, out, b, 99, rank, step, xn, idx)
        exp = torch.from_numpy(sample_indices(n, b, 99, rank, step))
        assert torch.equal(idx.cpu(), exp)
        assert torch.equal(out, X[exp.to(DEV)])
        torch.testing.assert_close(xn, X[exp.to(DEV)].float().pow(2).sum(1), rtol=1e-5, atol=1e-4)
    # uniform draws: every row about b/n times over many steps
    cnt = np.bincount(np.concatenate([sample_indices(1000, 10_000, 5, 0, s) for s in range(20)]), minlength=1000)
    assert cnt.min() > 120 and cnt.max() < 290


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_row_normalize_and_wdot(native, dtype):
    from mikmeans.ops import pad_columns

    X = pad_columns((torch.randn(5000, 40, device=DEV) * 3).to(dtype))
    X[7] = 0
    ref = X.float() / X.float().norm(dim=1, keepdim=True).clamp_min(1e-30)
    Y = X.clone()
    xn = torch.empty(5000, device=DEV)
    native.row_normalize(Y, xn)
    tol = 1e-6 if dtype == torch.float32 else 2 ** -8
    torch.testing.assert_close(Y.float(), ref, rtol=tol, atol=tol)
    assert torch.equal(Y[7], X[7])
    torch.testing.assert_close(xn, Y.float().pow(2).sum(1), rtol=1e-5, atol=1e-6)
    a, w = torch.rand(100_001, device=DEV), torch.rand(100_001, device=DEV)
    out = torch.zeros(1, dtype=torch.float64, device=DEV)
    scratch = torch.empty(native.WDOT_SCRATCH, dtype=torch.float64, device=DEV)
    native.wdot(a, w, out, scratch)
    assert float(out) == pytest.approx(float((a.double() * w.double()).sum()), rel=1e-12)
    again = torch.zeros(1, dtype=torch.float64, device=DEV)
    native.wdot(a, w, again, scratch)
    assert float(again) == float(out)                  # fixed summation order


def test_minibatch_fit_device_vs_host_shard(native, monkeypatch):
    """The same Philox rows on both placements: a device-resident shard (batches drawn by
    the gather kernel) and a host shard over the HBM budget (rows gathered on the host)
    give the same centres bit for bit; the CPU fit draws the same rows too."""
    n, D, K = 200_000, 32, 16
    X = B.make_blobs(n, D, K, seed=8, dtype=torch.float32, device="cpu")
    kw = dict(batch_size=4096, max_steps=25, init="random", seed=3, dtype="bfloat16", device=DEV)
    a = mikmeans.MiniBatchKMeans(K, **kw).fit(X)
    assert a.memory_plan_["mode"] == "minibatch-resident"
    from tests.test_gpu_memplan import host_budget

    monkeypatch.setenv("MIKMEANS_HBM_BYTES", str(host_budget(n, D, K, 4096)))
    b = mikmeans.MiniBatchKMeans(K, **kw).fit(X)
    assert b.memory_plan_["mode"] == "minibatch-host"
    assert torch.equal(a.cluster_centers_, b.cluster_centers_)
    assert torch.equal(a.counts_, b.counts_)
    monkeypatch.delenv("MIKMEANS_HBM_BYTES")
    c = mikmeans.MiniBatchKMeans(K, **dict(kw, dtype="float32")).fit(X.to(DEV))
    d = mikmeans.MiniBatchKMeans(K, **dict(kw, dtype="float32", device="cpu")).fit(X)
    torch.testing.assert_close(c.cluster_centers_.cpu(), d.cluster_centers_, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(c.counts_.cpu(), d.counts_)


def test_minibatch_fit_resume_widens_a_smaller_checkpoint_bound(native, tmp_path):
    """A mini-batch checkpoint whose col_bound is below the shard's maximum (fit_stream's,
    or a first-batch bound) resumed by fit(): the scales are widened to the shard's, so the
    unclamped M-step never saturates -- the centres equal an uninterrupted fit that started
    from the checkpoint's state with the shard's own bound (api.py:676)."""
    from mikmeans.utils.checkpoint import load_checkpoint

    n, D, K = 60_000, 32, 12
    X = B.make_blobs(n, D, K, seed=5, dtype=torch.float32, device=DEV)
    X[123, 7] = 900.0                   # one large value: far above any small-batch bound
    kw = dict(batch_size=2048, init="random", seed=3, dtype="float32", device=DEV)
    a = mikmeans.MiniBatchKMeans(K, max_steps=3, **kw).fit(X)
    ck = tmp_path / "mb"
    a.save(str(ck))
    st = load_checkpoint(str(ck))
    small = st["tensors"]["col_bound"].clone()
    small[:] = 1.0                      # a bound the shard's column 7 (900) exceeds
    from mikmeans.utils.checkpoint import save_checkpoint

    ck2 = tmp_path / "mb_small"
    save_checkpoint(str(ck2), st["centers"], st["iteration"], st["config"],
                    extra={"kind": "minibatch", "rescales": 0},
                    tensors={"vcount": st["tensors"]["vcount"], "col_bound": small})
    b = mikmeans.MiniBatchKMeans(K, max_steps=10, **kw).fit(X, resume_from=str(ck2))
    assert bool((b._eng.bound[:D].cpu() >= X.abs().amax(0).double().cpu()).all())
    c = mikmeans.MiniBatchKMeans(K, max_steps=10, **kw).fit(X, resume_from=str(ck))
    assert torch.equal(b.cluster_centers_, c.cluster_centers_)
    assert torch.equal(b.counts_, c.counts_)
    assert torch.isfinite(b.cluster_centers_).all()


def test_minibatch_fit_steps_do_not_sync(native):
    """Bounded scales from the whole shard: no step reads back to the host (one tol check
    per 10 steps at most) -- counted with a hooked .item()/.tolist() on device tensors."""
    n, D, K = 100_000, 64, 32
    X = B.make_blobs(n, D, K, seed=2, dtype=torch.bfloat16, device=DEV)
    km = mikmeans.MiniBatchKMeans(K, batch_size=2048, max_steps=40, init="random", seed=1,
                                  dtype="bfloat16", device=DEV, tol=1e-12)
    calls = {"n": 0}
    orig_item, orig_float = torch.Tensor.item, torch.Tensor.__float__

    def item(t):
        if t.is_cuda:
            calls["n"] += 1
        return orig_item(t)

    def flt(t):
        if t.is_cuda:
            calls["n"] += 1
        return orig_float(t)
    km._engine(D, torch.device(DEV))
    torch.Tensor.item, torch.Tensor.__float__ = item, flt
    try:
        eng = km._eng
        before = calls["n"]
        km.fit(X)
        per_step = (calls["n"] - before) / 40
    finally:
        torch.Tensor.item, torch.Tensor.__float__ = orig_item, orig_float
    assert eng.rescales == 0 and km.n_steps_ == 40
    # setup (bound, shard sizes, init) costs a few reads; the loop at most 1 per 10 steps
    assert per_step <= 0.1 + 12 / 40, per_step


@pytest.mark.parametrize("D,K,dtype,force_ks", [(256, 512, torch.bfloat16, None), (128, 1024, torch.bfloat16, None),
                                                (64, 4096, torch.bfloat16, None), (128, 256, torch.float32, None),
                                                (40, 20000, torch.float32, None), (256, 512, torch.bfloat16, "1"),
                                                (256, 600, torch.bfloat16, None)])
def test_gathered_rows_step_equals_materialised_batch(native, kvariant, D, K, dtype, force_ks):
    """partial_fit_rows (assign + M-step reading X[rows] through the index list: slice,
    K-split and global-atomic M-step kernels; force_ks: the K-split kernel where the slice
    kernel is the default; K=600 at D=256: the slice kernel without its LDS index staging,
    which no longer fits beside the cells) equals partial_fit on the gathered copy."""
    from mikmeans.models.minibatch import MiniBatchEngine
    from mikmeans.ops import col_stats, pad_columns

    if force_ks is not None:
        kvariant("update_ks", force_ks)

    n, b = 600_000, 270_000     # b > SPLIT_MAX_ROWS: both paths take the one-pass assign grid
    X = pad_columns(B.make_blobs(n, D, 64, seed=D, dtype=dtype, device=DEV))
    rows = torch.empty(b, dtype=torch.int64, device=DEV)
    bound = col_stats(X, stats=False).absmax
    ea = MiniBatchEngine(K, D, b, dtype=dtype, device=DEV).set_bound(bound)
    eb = MiniBatchEngine(K, D, b, dtype=dtype, device=DEV).set_bound(bound)
    C0 = X[torch.randperm(n, generator=torch.Generator().manual_seed(0))[:K].to(DEV), :D].float()
    ea.set_centers(C0)
    eb.set_centers(C0)
    for s in range(3):
        native.sample_index(n, b, 7, 0, s, rows)
        ea.partial_fit_rows(X, rows)
        eb.partial_fit(X[rows])
        torch.cuda.synchronize()
        assert torch.equal(ea.labels[:b], eb.labels[:b]), s
        assert torch.equal(ea.C, eb.C) and torch.equal(ea.vcount, eb.vcount), s
    assert ea.last_batch_inertia() == pytest.approx(eb.last_batch_inertia(), rel=1e-9)
