"""K-split M-step row groups in flight (MIKMEANS_UPDATE_KS_GM) at the cfg4 and headline shapes,
one process, interleaved: median ms of one full pass on Lloyd labels, sums checked equal."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from mikmeans.data.blobs import blob_centers, make_blobs
from mikmeans.models.init import init_random
from mikmeans.models.lloyd import LloydEngine
from mikmeans.ops import native
from mikmeans.parallel import Comm


def main():
    C = native.require()
    dev = torch.device("cuda")
    comm = Comm.local(dev)
    for n, d, k in ((10_000_000, 64, 4096), (20_000_000, 128, 1024)):
        X = make_blobs(n, d, k, seed=0, dtype=torch.bfloat16, device=dev, centers=blob_centers(k, d, 10.0, 0, device=dev))
        eng = LloydEngine(X, k, comm=comm).set_centers(init_random(X, d, k, n, 0, comm, 0))
        for _ in range(3):
            eng.step()
        nch = C.update_n_chunks(native.dtype_code(torch.bfloat16), k, eng.Dp, n, False)
        slab = torch.empty(nch * k * eng.Dp, dtype=torch.int64, device=dev)
        cnt = torch.empty(nch * k, dtype=torch.int64, device=dev)
        arms = ["2", "3", "6"]
        t = {g: [] for g in arms}
        sums = {}
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        for rd in range(5):
            for g in (arms if rd % 2 == 0 else arms[::-1]):
                native.set_variant("update_ks_gm", int(g))
                C.update(eng.X, eng.labels, k, slab, cnt, nch, None, eng.col_exp, eng.cnt_exp, False)
                ev[0].record()
                for _ in range(5):
                    C.update(eng.X, eng.labels, k, slab, cnt, nch, None, eng.col_exp, eng.cnt_exp, False)
                ev[1].record()
                torch.cuda.synchronize()
                t[g].append(ev[0].elapsed_time(ev[1]) / 5)
                sums[g] = slab.view(nch, -1).sum(0)
        native.set_variant("update_ks_gm", -1)
        print(json.dumps({"n": n, "d": d, "k": k, **{g: round(statistics.median(v), 4) for g, v in t.items()},
                          "sums_equal": all(torch.equal(sums[g], sums["2"]) for g in arms)}), flush=True)
        del eng, X


if __name__ == "__main__":
    main()
