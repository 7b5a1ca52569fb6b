"""Debug: split vs one-pass assign label differences (bf16, D=32, K=300, n=70000)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import mikmeans  # noqa: F401
from mikmeans import ops
from mikmeans.ops import cpu as ref
from mikmeans.ops import native

C_ = native.require()
DEV = "cuda"
for shift in (0.0, 50.0):
    for d, k, n in ((32, 300, 70000), (128, 1024, 1000), (64, 4096, 16384)):
        g = torch.Generator().manual_seed(n + k)
        X = (torch.randn(n, d, generator=g) + shift).to(torch.bfloat16)
        C = torch.randn(k, d, generator=torch.Generator().manual_seed(k + 11)) + shift
        Xp = ops.pad_columns(X.to(DEV))
        pk = ops.pack_centers(C.to(DEV), Xp.shape[1], Xp.dtype, DEV)
        xn = ops.row_sqnorm(Xp)
        out = []
        for split in (False, True):
            lab = torch.full((n,), 7, dtype=torch.int32, device=DEV)
            mind = torch.empty(n, dtype=torch.float32, device=DEV)
            if split:
                pk.assign(Xp, xn, lab, mind, None, True)
            else:
                C_.assign(Xp, pk.pack, pk.cn, xn, lab, mind, None, pk.Kpad, pk.dpad, True, None)
            out.append((lab.cpu(), mind.cpu()))
        diff = (out[0][0] != out[1][0]).nonzero().flatten()
        sc = ref.scores(X.double(), ref.quantize_centers(C, torch.bfloat16).double())
        xx = (X.double() ** 2).sum(1)
        msg = f"shift={shift} d={d} k={k} n={n}: {diff.numel()} label diffs"
        if diff.numel():
            i = diff[:5]
            a, b = out[0][0][i].long(), out[1][0][i].long()
            msg += f" rows {i.tolist()} one-pass {a.tolist()} split {b.tolist()} " \
                   f"d(one)-d(split) {(sc[i, a] - sc[i, b]).tolist()} |x|^2 {xx[i].tolist()}"
            wg = (i // 256).tolist()
            msg += f" wg {wg}"
        print(msg, flush=True)
