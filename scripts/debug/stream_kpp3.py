"""Debug: the streaming tests in sequence in one process, with diagnostics."""
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
    ref = mikmeans.KMeans(32, init=C0, dtype=dtype, max_iter=6, tol=0, device=DEV).fit(X)
    st = mikmeans.KMeans(32, init=C0, dtype=dtype, max_iter=6, tol=0, device=DEV, chunk_rows=6_000).fit(X.cpu())
    print("prev", dtype, torch.equal(st.cluster_centers_, ref.cluster_centers_), flush=True)


def kpp(tag):
    X = B.make_blobs(40_000, 32, 16, seed=5, dtype=torch.bfloat16, device="cpu")
    km = mikmeans.KMeans(16, dtype="bfloat16", max_iter=20, device=DEV, chunk_rows=1 << 13, init_size=4096).fit(X)
    idx = torch.randperm(40_000, generator=torch.Generator().manual_seed(0))[:4096].sort().values
    C0 = resolve_init("k-means++", X[idx].to(DEV), 32, 16, 4096, 0, Comm.local(torch.device(DEV)), 0)
    ref = mikmeans.KMeans(16, init=C0.cpu(), dtype="bfloat16", max_iter=20, device=DEV).fit(X.to(DEV))
    st = mikmeans.KMeans(16, init=C0.cpu(), dtype="bfloat16", max_iter=20, device=DEV, chunk_rows=1 << 13).fit(X)
    Xs = km._engine.sample_rows(4096, 0)
    C1 = resolve_init("k-means++", Xs, 32, 16, 4096, 0, Comm.local(torch.device(DEV)), 0)
    print(tag, "km==ref", torch.equal(km.cluster_centers_, ref.cluster_centers_), "st==ref",
          torch.equal(st.cluster_centers_, ref.cluster_centers_), "sample==X[idx]", torch.equal(Xs.cpu(), X[idx]),
          "C1==C0", torch.equal(C1, C0), "n_iter", km.n_iter_, ref.n_iter_, st.n_iter_, flush=True)
    print("  ", [(h["iter"], round(h["shift"], 6), h["n_changed"]) for h in km.history_][:3],
          [(h["iter"], round(h["shift"], 6), h["n_changed"]) for h in ref.history_][:3], flush=True)


kpp("first")
prev("bfloat16")
prev("float32")
kpp("after-prev")
gc.collect()
kpp("after-gc")
