"""Debug: native weighted k-means++ draws (csrc/kpp.hip wkpp) against a NumPy replay."""
import numpy as np
import torch

from mikmeans.ops import native

C_ = native.require()
g = torch.Generator().manual_seed(1)
M, D, K = 300, 8, 6
C = torch.randn(M, D, generator=g) * 3
w = torch.randint(1, 20, (M,), generator=g).double()
u = torch.rand(K, generator=g, dtype=torch.float64)
dev = "cuda"
Ct = C.t().contiguous().to(dev)
d2 = torch.full((M,), float("inf"), dtype=torch.float64, device=dev)
cum = torch.empty(M, dtype=torch.float64, device=dev)
part = torch.empty(-(-M // 256), dtype=torch.float64, device=dev)
state = torch.tensor([-1, 0], dtype=torch.int64, device=dev)
out = torch.zeros((K, D), dtype=torch.float32, device=dev)
for k in range(K):
    C_.wkpp(Ct, w.to(dev), d2, cum, part, u.to(dev), state, out, 1)
    torch.cuda.synchronize()
    print(k, "state", state.tolist(), "part", part.tolist()[:3], "cum[-1]", float(cum[M - 1]), "d2[:4]", d2[:4].tolist())
# numpy replay
Cd = C.double().numpy()
wd = w.numpy()
dd = np.full(M, np.inf)
picks = []
for k in range(K):
    if picks:
        dd = np.minimum(dd, ((Cd - Cd[picks[-1]]) ** 2).sum(1))
    cum_ = np.cumsum(wd * dd if picks else wd)
    j = min(int(np.searchsorted(cum_, u[k].item() * cum_[-1], side="right")), M - 1)
    picks.append(j)
got = [int(torch.cdist(out[i:i + 1].double().cpu(), C.double()).argmin()) for i in range(K)]
print("numpy picks ", picks)
print("native picks", got)
