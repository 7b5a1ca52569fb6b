"""The one-ring-per-CU assign (csrc/assign_ring.hip, switch ``assign_ring``): labels and
distances bitwise the production kernel's, its spins never give up, on ragged N, outlier rows
(per-point-offset groups), several K and tiny grids (waves without blocks)."""
import pytest
import torch

from mikmeans import ops
from mikmeans.data import blobs as B
from mikmeans.ops.native import slot_totals

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("n,k,outlier", [(300_007, 1024, False), (1_000_003, 1024, True), (70_001, 256, False),
                                         (200_003, 2048, True), (5_000, 1024, False), (256, 64, False),
                                         (4_000_000, 1024, False)])
def test_ring_assign_bitwise_production(native, kvariant, n, k, outlier):
    d = 128
    X = ops.pad_columns(B.make_blobs(n, d, 64, seed=n % 97, dtype=torch.bfloat16, device=DEV))
    if outlier:
        X[n // 3] *= 40.0
    C = X[torch.randperm(n, generator=torch.Generator().manual_seed(k))[:k].to(DEV), :d].float() + 0.125
    pk = ops.pack_centers(C, X.shape[1], torch.bfloat16, DEV)
    xn = ops.row_sqnorm(X)
    out = {}
    for arm in (0, 1):
        kvariant("assign_ring", arm)
        lab = torch.full((n,), 5, dtype=torch.int32, device=DEV)
        mind = torch.empty(n, device=DEV)
        slots = torch.zeros(native.NSLOT * native.SLOT_STRIDE, dtype=torch.float64, device=DEV)
        pk.assign(X, xn, lab, mind, slots, True)
        torch.cuda.synchronize()
        out[arm] = (lab, mind, slot_totals(slots))
    assert native.assign_ring_fault() == 0
    assert torch.equal(out[0][0], out[1][0])
    assert torch.equal(out[0][1], out[1][1])
    assert out[0][2][1] == out[1][2][1] == int((out[0][0] != 5).sum())
    assert out[1][2][0] == pytest.approx(out[0][2][0], rel=1e-9)
