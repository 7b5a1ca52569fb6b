"""Repro of test_assign_value_argmin_d64[300000-False-32-1024]: packed-key path (VARG=0) and
value-only path against the f64 argmin over many launches in one process, with other kernels
run in between (LDS left dirty by them): which rows differ (workgroup, wave, point block,
per-point-offset workgroup or not), which labels they got, and how often."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

from mikmeans.ops import native

from mikmeans import ops
from mikmeans.ops import cpu as ref

DEV = "cuda"
NL = int(os.environ.get("REPRO_LAUNCHES", "12"))


def case(n, d, k, shift, seed):
    g = torch.Generator().manual_seed(seed)
    X = torch.randn(n, d, generator=g) + shift
    C = torch.randn(k, d, generator=g) * 0.8 + shift
    Xb = X.to(torch.bfloat16)
    Cq = ref.quantize_centers(C, torch.bfloat16).double()
    Xd = Xb.double()
    xx = (Xd * Xd).sum(1)
    dist = xx[:, None] - 2 * Xd @ Cq.T + (Cq * Cq).sum(1)[None]
    m = dist.min(1, keepdim=True).values
    idx = torch.arange(k).expand_as(dist)
    exp = torch.where(dist == m, idx, k).min(1).values
    srt = dist.sort(1).values
    return Xb, C, exp, srt[:, 1] - srt[:, 0], xx


def dirty(i):
    """Other kernels between the launches (they leave their own data in LDS)."""
    if i % 3 == 0:
        Y = torch.randn(300_000, 256, device=DEV, dtype=torch.bfloat16) * 100
        ops.assign(Y, torch.randn(512, 256, device=DEV) * 50, with_dist=True)
    elif i % 3 == 1:
        Y = torch.randn(200_000, 64, device=DEV, dtype=torch.bfloat16) * 1e4
        ops.assign(Y, -torch.rand(4096, 64, device=DEV) * 1e4, with_dist=False)
    else:
        torch.cuda.synchronize()


def main():
    wg = 256
    for (n, d, k, shift, seed) in [(300_000, 32, 1024, 0.0, 11 + 300_000 + 32), (300_000, 32, 1024, 3.0, 5),
                                   (300_000, 64, 1024, 0.0, 7)]:
        Xb, C, exp, gap, xx = case(n, d, k, shift, seed)
        wgp = 256 if d == 32 else 512
        xg = torch.cat([xx, xx[-1:].expand((-n) % wgp)]).view(-1, wgp)
        ppo = xg.max(1).values > 4 * xg.min(1).values
        print(f"== n={n} d={d} k={k} shift={shift}: {xg.shape[0]} workgroups, {int(ppo.sum())} per-point-offset",
              flush=True)
        Xd, Cd = Xb.to(DEV), C.to(DEV)
        for pm in ("0", "1"):
            native.set_variant("assign_pmaj", int(pm))
            for env in ("0", "1"):
                native.set_variant("assign_varg", int(env))
                nbad_launches, tot = 0, 0
                for r in range(NL):
                    dirty(r)
                    lab, _ = ops.assign(Xd, Cd, with_dist=False)
                    lab = lab.cpu().long()
                    bad = ((lab != exp) & (gap > 1e-3)).nonzero().flatten()
                    if len(bad):
                        nbad_launches += 1
                        tot += len(bad)
                        w = bad // wgp
                        off = bad % wgp
                        ws = sorted(set(w.tolist()))
                        print(f"  PMAJ={pm} VARG={env} launch {r}: {len(bad)} wrong rows in workgroups {ws[:6]} "
                              f"(ppo {[bool(ppo[x]) for x in ws[:6]]}); waves {sorted(set((off // (wgp // 4)).tolist()))} "
                              f"blocks {sorted(set(((off % (wgp // 4)) // 16).tolist()))} labels {sorted(set(lab[bad].tolist()))[:8]}",
                              flush=True)
                print(f"  PMAJ={pm} VARG={env}: {nbad_launches}/{NL} launches wrong, {tot} rows", flush=True)
    native.set_variant("assign_varg", -1)
    native.set_variant("assign_pmaj", -1)


if __name__ == "__main__":
    main()
