"""HBM memory planner (parallel/memplan.py): the Python mirror of csrc/plan.h against the
native launch planning, the allocation inventory for fixed shapes, and the plan choice."""
import itertools

import pytest
import torch

from mikmeans.parallel import memplan as M


def _native():
    from mikmeans.ops import native

    if not native.available():
        pytest.skip("native extension not built")
    return native.require()


def test_plan_h_mirror_matches_native():
    C = _native()
    for dt, K, D, N, w in itertools.product((0, 1), (1, 3, 64, 256, 512, 1024, 3500, 4096, 9000, 20000),
                                            (2, 8, 16, 32, 64, 96, 128, 256),
                                            (1, 1000, 1 << 20, 100_000_000), (False, True)):
        es = 2 if dt == 1 else 4
        if (D * es) % 16:
            continue
        assert M.choose_sw(es, K, D, w)[0] == C.update_slice_width(dt, K, D, w), (dt, K, D, w)
        assert M.update_n_chunks(es, K, D, N, w) == C.update_n_chunks(dt, K, D, N, w), (dt, K, D, N, w)
    for dt, dpad, K in itertools.product((0, 1), (16, 32, 64, 128, 256), (1, 7, 256, 1000, 1024, 4096, 5000)):
        es = 2 if dt == 1 else 4
        assert M.assign_kpad(es, dpad, K) == C.assign_kpad(dt, dpad, K), (dt, dpad, K)
    for kp in (16, 256, 1024, 4352):
        assert M.assign_cn_len(kp) == C.assign_cn_len(kp)
    assert (M.NSLOT, M.SLOT_STRIDE) == (C.NSLOT, C.SLOT_STRIDE)
    for dt, n, dp in itertools.product((0, 1), (1, 17, 1000, 40_000, 1 << 20, 100_000_000), (16, 64, 128, 256, 1024)):
        es = 2 if dt == 1 else 4
        assert M.colstat_rows(es, n, dp) == C.colstat_rows(dt, n, dp), (dt, n, dp)
    assert M.WDOT_SCRATCH == C.WDOT_SCRATCH


def test_resident_inventory_fixed_shapes():
    """Byte-for-byte inventory of three shapes (hand-derived from LloydEngine._init_gpu)."""
    # headline shard: N=1e8 D=128 K=1024 bf16, incremental, k-means++ (1 trial)
    p = M.plan_resident(100_000_000, 128, 1024, "bfloat16", incremental=True)
    assert p.Dp == 128
    assert p.persistent["X"] == 25_600_000_000
    assert p.persistent["labels"] == p.persistent["xn"] == 400_000_000
    nch = M.update_n_chunks(2, 1024, 128, 100_000_000, True)
    assert nch == 64                       # weighted-count LDS: 4 slices of 32 columns -> 64 chunks
    assert p.persistent["slab"] == 64 * 1024 * 128 * 8
    assert p.persistent["cnt_slab"] == 64 * 1024 * 8
    assert p.persistent["packed"] == M._r((1024 * 128 + 1024 + 2) * 8) == 1_057_280
    assert p.persistent["pack"] == 1024 * 128 * 2 and p.persistent["cn"] == 1024 * 4
    assert p.persistent["delta_prev"] == 400_000_000
    assert p.persistent["delta_list"] == 100_000_256          # 12.5M x (row, label), 512-B rounded
    assert p.persistent["delta_tot"] == (1024 * 128 + 1024) * 8
    assert "split_keys" not in p.persistent
    assert p.transient["final_assign"] == {"labels_out": 400_000_000, "mind_out": 400_000_000}
    assert p.transient["init"]["kpp_d2"] == 400_000_000 and p.transient["init"]["kpp_owner"] == 400_000_000
    # cfg2: N=1e6 D=128 K=256 f32, full M-step, weighted, random init
    q = M.plan_resident(1_000_000, 128, 256, "float32", weighted=True, incremental=False, init="random")
    assert q.persistent["X"] == 512_000_000 and q.persistent["weights"] == q.persistent["mind"] == 4_000_256
    assert q.persistent["slab"] == M.update_n_chunks(4, 256, 128, 1_000_000, True) * 256 * 128 * 8
    assert "delta_prev" not in q.persistent
    assert q.transient["init"] == {"init_rows": M._r(256 * 128 * 8)}
    # small ragged shard: N=70_000 D=30 (padded to 32 bf16) K=9: split keys, 512-B rounding
    r = M.plan_resident(70_000, 30, 9, "bfloat16", incremental=False)
    assert r.Dp == 32 and r.persistent["X"] == 70_000 * 32 * 2
    assert r.persistent["split_keys"] == 560_128 and r.persistent["labels"] == 280_064
    assert r.persistent["C"] == M._r(9 * 32 * 4) == 1536
    assert r.persistent["pack"] == M.assign_kpad(2, 32, 9) * 32 * 2


def test_plan_fit_choice():
    # the headline shard fits one GPU; a 1e9 x 256 bf16 shard (512 GB) does not, but streams
    p = M.plan_fit(100_000_000, 128, 1024, budget=280 * 10**9, x_on_device=False)
    assert p.mode == "resident" and p.fits
    q = M.plan_fit(1_000_000_000, 256, 512, budget=280 * 10**9, x_on_device=False)
    assert q.mode == "streaming" and q.fits and q.chunk_rows % M.ROW_ALIGN == 0 and q.chunk_rows <= 1 << 24
    assert q.peak <= 280 * 10**9
    # at W=8 the 125M-row shard (64 GB) is resident
    assert M.plan_fit(125_000_000, 256, 512, budget=280 * 10**9, x_on_device=False).mode == "resident"
    # per-row state alone over budget: a clear error, not an OOM
    with pytest.raises(M.HBMCapacityError):
        M.plan_fit(10**10, 256, 512, budget=40 * 10**9, x_on_device=False)
    with pytest.raises(M.HBMCapacityError):
        M.plan_fit(10**9, 256, 512, budget=280 * 10**9, x_on_device=True)
    # smaller budgets pick smaller chunks, all on the 1536-row grid
    a = M.plan_fit(10**8, 128, 1024, budget=20 * 10**9, x_on_device=False)
    b = M.plan_fit(10**8, 128, 1024, budget=4 * 10**9, x_on_device=False)
    assert a.mode == b.mode == "streaming" and a.chunk_rows > b.chunk_rows and b.peak <= 4 * 10**9


def test_minibatch_plan():
    p = M.plan_minibatch(125_000_000, 256, 512, "bfloat16", batch_rows=1 << 24)
    assert p.persistent["X"] == 64_000_000_000
    # a resident shard is read in place through the step's int64 row list: no batch copy
    assert p.persistent["rows"] == (1 << 24) * 8 and "batch" not in p.persistent
    h = M.plan_minibatch(10**9, 256, 512, "bfloat16", batch_rows=1 << 24, resident=False)
    assert "X" not in h.persistent and h.mode == "minibatch-host"
    assert h.persistent["batch"] == (1 << 24) * 256 * 2 and "rows" not in h.persistent


def test_budget_env_override(monkeypatch):
    monkeypatch.setenv("MIKMEANS_HBM_BYTES", "12345678")
    assert M.hbm_budget() == 12_345_678
