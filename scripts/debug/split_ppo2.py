"""Debug 2: split-mode wrong labels -- determinism, xn / no xn, per-WG pattern."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import mikmeans  # noqa: F401
from mikmeans import ops
from mikmeans.ops import native

C_ = native.require()
DEV = "cuda"


def run(X, C, split, with_xn=True, reps=1):
    n = X.shape[0]
    Xp = ops.pad_columns(X.to(DEV))
    pk = ops.pack_centers(C.to(DEV), Xp.shape[1], Xp.dtype, DEV)
    xn = ops.row_sqnorm(Xp) if with_xn else None
    outs = []
    for _ in range(reps):
        lab = torch.full((n,), 7, dtype=torch.int32, device=DEV)
        mind = torch.empty(n, dtype=torch.float32, device=DEV) if with_xn else None
        if split:
            pk.assign(Xp, xn, lab, mind, None, True)
        else:
            C_.assign(Xp, pk.pack, pk.cn, xn, lab, mind, None, pk.Kpad, pk.dpad, True, None)
        torch.cuda.synchronize()
        outs.append(lab.cpu())
    return outs


for d, k, n, shift in ((32, 300, 70000, 0.0), (32, 300, 70000, 2.0), (64, 300, 70000, 0.0), (128, 300, 70000, 0.0),
                       (32, 600, 70000, 0.0), (32, 300, 7000, 0.0)):
    g = torch.Generator().manual_seed(n + k)
    X = (torch.randn(n, d, generator=g) + shift).to(torch.bfloat16)
    C = torch.randn(k, d, generator=torch.Generator().manual_seed(k + 11)) + shift
    one = run(X, C, False)[0]
    sp = run(X, C, True, reps=4)
    spn = run(X, C, True, with_xn=False, reps=2)
    onen = run(X, C, False, with_xn=False)[0]
    diffs = [int((s != one).sum()) for s in sp]
    diffn = [int((s != onen).sum()) for s in spn]
    bad = (sp[0] != one).nonzero().flatten()
    wgs = sorted(set((bad // 256).tolist()))
    pos = sorted(set((bad % 256).tolist()))[:20]
    print(f"d={d} k={k} n={n} shift={shift}: split-vs-one diffs {diffs} (no xn: {diffn}); "
          f"bad WGs {wgs[:10]} positions {pos} labels {sp[0][bad[:8]].tolist()}", flush=True)
