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
    """hipGraph replay around the (eager) RCCL all-reduce is bitwise the eager steps."""
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


def _graph_case(opt):
    """(X, C0, engine kwargs) of one engine option set for the capture tests."""
    n, d, k = 50_000, 64, 40
    dtype = torch.float32 if opt == "f32" else torch.bfloat16
    X = B.make_blobs(n, d, 30, seed=9, dtype=dtype, device=DEV)
    C0 = X[:k].float().clone()
    kw = {}
    if opt == "weighted":
        kw["sample_weight"] = (torch.rand(n, generator=torch.Generator().manual_seed(3)) + 0.5).to(DEV)
    elif opt == "spherical":
        from mikmeans.ops import native as nat

        nat.require().row_normalize(X)
        C0 = X[:k].float().clone()
        kw["spherical"] = True
    elif opt == "incremental":
        kw["incremental"] = True
    elif opt == "wide_column":
        X[777, 3] = 3.0e5
    elif opt == "segments":
        kw["segments"] = 4
    elif opt == "farthest":
        C0[5:9] = 1.0e4                        # far-away centres: empty -> relocated between graphs
        kw["empty_policy"] = "farthest"
    return X, C0, k, kw


@pytest.mark.parametrize("opt", ["plain", "f32", "weighted", "spherical", "incremental", "wide_column",
                                 "segments", "farthest"])
def test_rccl_graph_every_option_set(rccl, opt):
    """Every engine option set captures (no RCCL call is recorded: the collective and the
    'farthest' relocation run between the graphs) and replays bitwise like eager steps."""
    from mikmeans.models.lloyd import LloydEngine

    X, C0, k, kw = _graph_case(opt)
    ea = LloydEngine(X, k, comm=Comm.local(DEV), **kw).set_centers(C0)
    eb = LloydEngine(X, k, comm=rccl, **kw).set_centers(C0).capture()
    assert eb._graphs is not None, eb.capture_error
    if opt == "wide_column":
        assert eb.scales.nw == 1
    for _ in range(5):
        ea.step()
        eb.step()
        torch.cuda.synchronize()
        assert torch.equal(ea.centers, eb.centers), opt
        assert torch.equal(ea.labels, eb.labels), opt
    sa, sb = ea.last_stats(), eb.last_stats()
    assert sa.n_changed == sb.n_changed and sa.inertia == pytest.approx(sb.inertia, rel=1e-12)


def test_rccl_graph_capture_failure_falls_back_eager(rccl):
    """A capture-illegal call during capture: the capture is torn down, the engine keeps
    stepping eagerly with the eager result, and the RCCL group stays healthy."""
    from mikmeans.models.lloyd import LloydEngine

    X, C0, k, kw = _graph_case("plain")
    ea = LloydEngine(X, k, comm=Comm.local(DEV)).set_centers(C0)
    eb = LloydEngine(X, k, comm=rccl).set_centers(C0)
    eb._inject_capture_fault = True
    eb.capture()
    assert eb._graphs is None and eb.capture_error
    for _ in range(4):
        ea.step()
        eb.step()
    torch.cuda.synchronize()
    assert torch.equal(ea.centers, eb.centers)
    t = torch.ones(4, dtype=torch.float64, device=DEV)
    rccl.allreduce_(t)
    rccl.barrier()
    assert float(t.sum()) == 4.0


_FAULT_SCRIPT = r"""
import os, sys, time, torch, torch.distributed as dist
sys.path.insert(0, os.getcwd())
from mikmeans.data import blobs as B
from mikmeans.models.lloyd import LloydEngine
from mikmeans.parallel import Comm
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
comm = Comm(rank=0, world=1, local_rank=0, backend="nccl", device=dev, owns_group=True)
X = B.make_blobs(40_000, 64, 30, seed=9, dtype=torch.bfloat16, device=dev)
C0 = X[:40].float().clone()
ea = LloydEngine(X, 40, comm=Comm.local(dev)).set_centers(C0)
eb = LloydEngine(X, 40, comm=comm).set_centers(C0)
for _ in range(2):          # collectives in flight for the watchdog before the capture
    eb.step()
    ea.step()
eb._inject_capture_fault = True
eb.capture()
assert eb._graphs is None and eb.capture_error, "capture should have failed"
for _ in range(6):
    ea.step(); eb.step()
torch.cuda.synchronize()
time.sleep(3)               # the RCCL watchdog polls its work queue meanwhile
assert torch.equal(ea.centers, eb.centers)
comm.close()
print("FALLBACK-OK", eb.capture_error)
"""


def test_graph_capture_failure_no_abort_subprocess():
    """The same injected failure in a fresh process with RCCL work in flight: exit code 0,
    the eager result, no watchdog abort / core (round-3 verdict: a failed capture had
    ended in 'operation not permitted on an event last recorded in a capturing stream')."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()))
    r = subprocess.run([sys.executable, "-c", _FAULT_SCRIPT], cwd=root, env=env, capture_output=True, text=True,
                       timeout=180)
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    assert "FALLBACK-OK" in r.stdout


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
    # two-stage (one all-gather per centre): on one rank the in-rank draw is the exact one
    c = init_kmeanspp(X, d, k, n, 0, rccl, seed=5, n_local_trials=trials, owner_path=True, sampling="two-stage")
    assert torch.equal(a, c)


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
