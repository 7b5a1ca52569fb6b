"""Centre-stationary assign vs the streaming kernel with 64-row seed offsets: where they differ."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import torch

import mikmeans
from mikmeans import ops
from mikmeans.ops import native as nat, pad_columns
from mikmeans.ops import cpu as ref

DEV = "cuda"
C_ = nat.require()
for (n, d, k) in [(20000, 128, 256), (3000, 256, 512)]:
    g = torch.Generator().manual_seed(n + d + k)
    X = torch.randn(n, d, generator=g)
    Xb = pad_columns(X.to(torch.bfloat16).to(DEV))
    C = torch.randn(k, d, generator=g) * 0.8
    pk = ops.pack_centers(C.to(DEV), Xb.shape[1], torch.bfloat16, DEV)
    xn = ops.row_sqnorm(Xb)
    nat.set_variant("assign_cs", 1)
    lab = torch.full((n,), 5, dtype=torch.int32, device=DEV)
    mind = torch.empty(n, device=DEV)
    pk.assign(Xb, xn, lab, mind)
    oseed = pk.seed_offsets(xn)
    nat.set_variant("assign_cs", 0)
    lab_g = torch.empty(n, dtype=torch.int32, device=DEV)
    mind_g = torch.empty(n, device=DEV)
    pk.assign(Xb, xn, lab_g, mind_g, rows=torch.arange(n, device=DEV), oseed=oseed)
    lab_p = torch.empty(n, dtype=torch.int32, device=DEV)
    mind_p = torch.empty(n, device=DEV)
    pk.assign(Xb, xn, lab_p, mind_p)
    torch.cuda.synchronize()
    # expected 64-row offsets
    xx = xn.cpu()
    pad = (-n) % 64
    xw = torch.cat([xx, xx[-1:].expand(pad)]).view(-1, 64)
    m, mn = xw.max(1).values, xw.min(1).values
    ppo = m > 4 * mn
    off = torch.where(ppo[:, None], xw * (1 + 2**-12), (m * (1 + 2**-12))[:, None].expand(-1, 64)).reshape(-1)[:n]
    print(f"n={n} d={d} k={k}: ppo blocks {int(ppo.sum())}/{len(ppo)}; oseed vs torch max rel "
          f"{float(((oseed.cpu() - off).abs() / off).max()):.3e}")
    dl = (lab != lab_g).cpu()
    dm = (mind != mind_g).cpu()
    print(f"  labels differ {int(dl.sum())}, mind differ {int(dm.sum())}; vs plain: labels {int((lab != lab_p).sum())}"
          f" mind {int((mind != mind_p).sum())}; gathered vs plain labels {int((lab_g != lab_p).sum())}")
    idx = torch.nonzero(dm)[:, 0]
    if len(idx):
        print("  first rows", idx[:20].tolist())
        print("  row%64 hist", torch.bincount(idx % 64, minlength=64).tolist())
        print("  mind cs", mind.cpu()[idx[:8]].tolist())
        print("  mind g ", mind_g.cpu()[idx[:8]].tolist())
        print("  mind p ", mind_p.cpu()[idx[:8]].tolist())
        sc = ref.scores(X.to(torch.bfloat16)[idx[:8]], C)
        print("  exact  ", (sc.min(1).values + (X.to(torch.bfloat16)[idx[:8]].float() ** 2).sum(1)).tolist())
        print("  lab cs/g", lab.cpu()[idx[:8]].tolist(), lab_g.cpu()[idx[:8]].tolist())
