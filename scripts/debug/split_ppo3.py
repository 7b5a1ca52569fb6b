"""Debug 3: nondeterminism of one-pass vs split assign (bf16 D=32 origin data, PPO workgroups)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import mikmeans  # noqa: F401
from mikmeans import ops
from mikmeans.ops import native

C_ = native.require()
DEV = "cuda"
n, d, k = 70000, 32, 300
g = torch.Generator().manual_seed(n + k)
X = torch.randn(n, d, generator=g).to(torch.bfloat16)
C = torch.randn(k, d, generator=torch.Generator().manual_seed(k + 11))
Xp = ops.pad_columns(X.to(DEV))
xn = ops.row_sqnorm(Xp)
for trial in range(3):
    pk = ops.pack_centers(C.to(DEV), Xp.shape[1], Xp.dtype, DEV)
    ref = None
    for mode in ("one", "split", "one", "split", "split_noxn", "one_noxn"):
        res = []
        for rep in range(10):
            lab = torch.full((n,), 7, dtype=torch.int32, device=DEV)
            use_xn = not mode.endswith("noxn")
            mind = torch.empty(n, dtype=torch.float32, device=DEV) if use_xn else None
            if mode.startswith("split"):
                pk.assign(Xp, xn if use_xn else None, lab, mind, None, True)
            else:
                C_.assign(Xp, pk.pack, pk.cn, xn if use_xn else None, lab, mind, None, pk.Kpad, pk.dpad, True, None)
            res.append(lab.cpu())
        if ref is None:
            ref = res[0]
        print(trial, mode, [int((r != ref).sum()) for r in res], flush=True)
    del pk
