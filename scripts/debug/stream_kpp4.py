"""Debug: is the streamed k-means++ fit nondeterministic?  Repeats the streamed fits
(k-means++ sample init, and from explicit centres) and prints each run's n_changed
trajectory next to the resident fit's; then steps a streamed and a resident engine in
lockstep from the same centres and reports the first label difference."""
import os, sys, gc
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import mikmeans
from mikmeans.data import blobs as B
from mikmeans.models.init import resolve_init
from mikmeans.parallel import Comm

DEV = "cuda"


def prev(dtype):
    X = B.make_blobs(50_000, 60, 32, seed=21, dtype=torch.float32, device=DEV)
    C0 = X[:32].cpu()
    mikmeans.KMeans(32, init=C0, dtype=dtype, max_iter=6, tol=0, device=DEV).fit(X)
    mikmeans.KMeans(32, init=C0, dtype=dtype, max_iter=6, tol=0, device=DEV, chunk_rows=6_000).fit(X.cpu())


X = B.make_blobs(40_000, 32, 16, seed=5, dtype=torch.bfloat16, device="cpu")
idx = torch.randperm(40_000, generator=torch.Generator().manual_seed(0))[:4096].sort().values
C0 = resolve_init("k-means++", X[idx].to(DEV), 32, 16, 4096, 0, Comm.local(torch.device(DEV)), 0)
ref = mikmeans.KMeans(16, init=C0.cpu(), dtype="bfloat16", max_iter=20, device=DEV).fit(X.to(DEV))
traj = lambda km: [h["n_changed"] for h in km.history_]
print("ref", ref.n_iter_, traj(ref), flush=True)
prev("bfloat16")
prev("float32")
for t in range(6):
    km = mikmeans.KMeans(16, dtype="bfloat16", max_iter=20, device=DEV, chunk_rows=1 << 13, init_size=4096).fit(X)
    st = mikmeans.KMeans(16, init=C0.cpu(), dtype="bfloat16", max_iter=20, device=DEV, chunk_rows=1 << 13).fit(X)
    print(t, "km", km.n_iter_, torch.equal(km.cluster_centers_, ref.cluster_centers_), traj(km),
          "| st", st.n_iter_, torch.equal(st.cluster_centers_, ref.cluster_centers_), traj(st), flush=True)

# lockstep: streamed vs resident engine from the same centres, labels compared every step
from mikmeans.models.lloyd import LloydEngine
from mikmeans.models.streaming import StreamingLloydEngine

for rep in range(4):
    es = StreamingLloydEngine(X, 16, chunk_rows=1 << 13, device=DEV, dtype=torch.bfloat16)
    er = LloydEngine(X.to(DEV), 16)
    es.set_centers(C0[:, :32])
    er.set_centers(C0[:, :32])
    for it in range(14):
        es.step()
        er.step()
        torch.cuda.synchronize()
        d = (es.labels != er.labels).nonzero().flatten()
        if d.numel() or not torch.equal(es.centers, er.centers):
            print("rep", rep, "iter", it + 1, "label diffs", d.numel(), d[:8].tolist(),
                  "centres equal", torch.equal(es.centers, er.centers), flush=True)
            if d.numel():
                i = d[:4]
                print("   es", es.labels[i].tolist(), "er", er.labels[i].tolist(), flush=True)
            break
    else:
        print("rep", rep, "lockstep equal for 14 steps", flush=True)
    del es, er
    gc.collect()
