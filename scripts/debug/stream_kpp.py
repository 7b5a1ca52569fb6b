"""Debug: streamed (k-means++ sample init) vs resident fit from the same seeding."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import mikmeans
from mikmeans.data import blobs as B
from mikmeans.models.init import resolve_init
from mikmeans.parallel import Comm

DEV = "cuda"
X = B.make_blobs(40_000, 32, 16, seed=5, dtype=torch.bfloat16, device="cpu")
for tol in (1e-4, 0.0):
    km = mikmeans.KMeans(16, dtype="bfloat16", max_iter=20, device=DEV, chunk_rows=1 << 13, init_size=4096,
                         tol=tol, verbose=0).fit(X)
    idx = torch.randperm(40_000, generator=torch.Generator().manual_seed(0))[:4096].sort().values
    C0 = resolve_init("k-means++", X[idx].to(DEV), 32, 16, 4096, 0, Comm.local(torch.device(DEV)), 0)
    ref = mikmeans.KMeans(16, init=C0.cpu(), dtype="bfloat16", max_iter=20, device=DEV, tol=tol).fit(X.to(DEV))
    st = mikmeans.KMeans(16, init=C0.cpu(), dtype="bfloat16", max_iter=20, device=DEV, tol=tol,
                         chunk_rows=1 << 13).fit(X)
    h1 = [(h["iter"], h["shift"], h["n_changed"]) for h in km.history_]
    h2 = [(h["iter"], h["shift"], h["n_changed"]) for h in ref.history_]
    print("tol", tol, "n_iter km/ref/st", km.n_iter_, ref.n_iter_, st.n_iter_,
          "km==ref", torch.equal(km.cluster_centers_, ref.cluster_centers_),
          "st==ref", torch.equal(st.cluster_centers_, ref.cluster_centers_),
          "maxdiff", float((km.cluster_centers_ - ref.cluster_centers_).abs().max()), flush=True)
    print(" km hist", h1[:4], h1[-2:], flush=True)
    print(" ref hist", h2[:4], h2[-2:], flush=True)
    C0s = km._engine  # streaming engine
