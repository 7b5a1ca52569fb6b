"""Debug: does the streamed k-means++-sample fit read uninitialised device memory?"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import mikmeans
from mikmeans.data import blobs as B
from mikmeans.models.init import resolve_init
from mikmeans.parallel import Comm

DEV = "cuda"


def once(tag):
    X = B.make_blobs(40_000, 32, 16, seed=5, dtype=torch.bfloat16, device="cpu")
    km = mikmeans.KMeans(16, dtype="bfloat16", max_iter=20, device=DEV, chunk_rows=1 << 13, init_size=4096).fit(X)
    idx = torch.randperm(40_000, generator=torch.Generator().manual_seed(0))[:4096].sort().values
    C0 = resolve_init("k-means++", X[idx].to(DEV), 32, 16, 4096, 0, Comm.local(torch.device(DEV)), 0)
    ref = mikmeans.KMeans(16, init=C0.cpu(), dtype="bfloat16", max_iter=20, device=DEV).fit(X.to(DEV))
    st = mikmeans.KMeans(16, init=C0.cpu(), dtype="bfloat16", max_iter=20, device=DEV, chunk_rows=1 << 13).fit(X)
    # the sample init on its own
    Xs = km._engine.sample_rows(4096, 0)
    C1 = resolve_init("k-means++", Xs, 32, 16, 4096, 0, Comm.local(torch.device(DEV)), 0)
    print(tag, "km==ref", torch.equal(km.cluster_centers_, ref.cluster_centers_), "st==ref",
          torch.equal(st.cluster_centers_, ref.cluster_centers_), "sample==X[idx]",
          torch.equal(Xs.cpu(), X[idx]), "C1==C0", torch.equal(C1, C0), "n_iter", km.n_iter_, ref.n_iter_,
          st.n_iter_, flush=True)


once("fresh")
junk = torch.full((1 << 29,), float("nan"), device=DEV)   # 2 GB of NaN, then freed
del junk
once("after-nan")
junk = torch.randint(-2**31, 2**31 - 1, (1 << 29,), device=DEV, dtype=torch.int32)
del junk
once("after-rand")
