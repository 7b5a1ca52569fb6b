"""The RCCL path on hardware: a real one-rank ``nccl`` (RCCL) process group on the GPU box.

Every collective the multi-GPU job issues (packed f64 all-reduce, all-gather,
broadcast, barrier, hipGraph capture of the all-reduce, k-means++ owner selection)
runs here through RCCL and must give bitwise the results of the no-group path.
This is the one-GPU rehearsal of the reference's mesh + full-state sync
(app.mjs:70-118); the 8-GPU run is the driver's.
"""
import os

import pytest
import torch
import torch.distributed as dist

from mikmeans.data import blobs as B
from mikmeans.parallel import Comm
from mikmeans.parallel.launch import free_port

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


@pytest.fixture(scope="module")
def rccl(native):
    assert not dist.is_initialized()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()))
    torch.cuda.set_device(DEV)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=DEV)
    comm = Comm(rank=0, world=1, local_rank=0, backend=dist.get_backend(), device=DEV, owns_group=True)
    assert comm.grouped and comm.backend == "nccl"
    yield comm
    comm.close()
    assert not dist.is_initialized()


def test_rccl_collectives(rccl):
    t = torch.arange(1 << 17, dtype=torch.float64, device=DEV)
    ref = t.clone()
    rccl.allreduce_(t)
    assert torch.equal(t, ref)
    m = torch.tensor([3.5], dtype=torch.float64, device=DEV)
    rccl.allreduce_max_(m)
    assert float(m) == 3.5
    g = rccl.all_gather(torch.arange(12, dtype=torch.float32, device=DEV).view(3, 4))
    assert g.shape == (1, 3, 4) and torch.equal(g[0].flatten().cpu(), torch.arange(12, dtype=torch.float32))
    b = torch.full((7,), 2.0, device=DEV)
    rccl.broadcast_(b)
    assert torch.equal(b, torch.full((7,), 2.0, device=DEV))
    rccl.barrier()
    torch.cuda.synchronize()


def test_rccl_lloyd_bitwise_equal_to_local(rccl):
    from mikmeans.models.lloyd import LloydEngine

    X = B.make_blobs(60_000, 128, 64, seed=3, dtype=torch.bfloat16, device=DEV)
    C0 = X[:64].float()
    ea = LloydEngine(X, 64, comm=Comm.local(DEV)).set_centers(C0)
    eb = LloydEngine(X, 64, comm=rccl).set_centers(C0)
    for _ in range(4):
        ea.step()
        eb.step()
    torch.cuda.synchronize()
    assert torch.equal(ea.centers, eb.centers)
    sa, sb = ea.last_stats(), eb.last_stats()
    assert sa.inertia == sb.inertia and sa.n_changed == sb.n_changed


@pytest.mark.parametrize("incremental", [False, True])
def test_rccl_graph_capture_of_allreduce(rccl, incremental):
    """hipGraph capture with the RCCL all-reduce inside replays bitwise like eager steps."""
    from mikmeans.models.lloyd import LloydEngine

    X = B.make_blobs(50_000, 64, 40, seed=9, dtype=torch.bfloat16, device=DEV)
    C0 = X[:40].float()
    ea = LloydEngine(X, 40, comm=Comm.local(DEV), incremental=incremental).set_centers(C0)
    eb = LloydEngine(X, 40, comm=rccl, incremental=incremental).set_centers(C0).capture()
    assert eb._graphs is not None
    for _ in range(5):
        ea.step()
        eb.step()
        torch.cuda.synchronize()
        assert torch.equal(ea.centers, eb.centers)
    assert ea.last_stats().inertia == eb.last_stats().inertia


@pytest.mark.parametrize("trials", [1, 3])
def test_rccl_kmeanspp_multi_rank_path(rccl, trials):
    """With a group, k-means++ takes the owner-selection path (all-gather of potentials,
    owner kernel, all-reduce of the drawn row) and must pick the same centres."""
    from mikmeans.models.init import init_kmeanspp

    n, d, k = 40_000, 64, 48
    X = B.make_blobs(n, d, 30, seed=2, dtype=torch.bfloat16, device=DEV)
    a = init_kmeanspp(X, d, k, n, 0, Comm.local(DEV), seed=5, n_local_trials=trials)
    b = init_kmeanspp(X, d, k, n, 0, rccl, seed=5, n_local_trials=trials, owner_path=True)
    # the owner path draws with target - 0 on the only rank: same row every step
    assert torch.equal(a, b)


def test_rccl_minibatch_and_api(rccl):
    import mikmeans
    from mikmeans.models.minibatch import MiniBatchEngine

    X = B.make_blobs(16_384, 32, 10, seed=3, device=DEV)
    C0 = X[:10].clone()
    ea = MiniBatchEngine(10, 32, 2048, device=DEV, comm=Comm.local(DEV))
    eb = MiniBatchEngine(10, 32, 2048, device=DEV, comm=rccl)
    ea.set_centers(C0)
    eb.set_centers(C0)
    for s in range(8):
        xb = X[s * 2048 : (s + 1) * 2048]
        ea.partial_fit(xb)
        eb.partial_fit(xb)
    assert torch.equal(ea.centers, eb.centers)
    km_a = mikmeans.KMeans(10, seed=1, max_iter=20, comm=Comm.local(DEV)).fit(X)
    km_b = mikmeans.KMeans(10, seed=1, max_iter=20, comm=rccl).fit(X)
    assert torch.equal(km_a.cluster_centers_, km_b.cluster_centers_)
