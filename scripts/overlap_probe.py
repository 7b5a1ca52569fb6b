"""Can the blob generator share the chip with the mini-batch M-step or the assign?

cfg5 shapes (16.8M x 256 bf16 batch, K=512): times the update kernel, the generator and
the assign alone, then update+generator and assign+generator launched together on two
streams (events on both).  If a pair costs about the sum of its parts, the kernels do
not co-reside (profiles/r1_18_blobstream_prefetch_ab.json found that for the assign).

run (GPU): python scripts/overlap_probe.py
"""
import json
import sys

import torch

sys.path.insert(0, ".")
from mikmeans.data.blobs import BlobStream, make_blobs  # noqa: E402
from mikmeans.models.minibatch import MiniBatchEngine  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    b, D, K = 1 << 24, 256, 512
    st = BlobStream(10**9, D, K, b, seed=0, dtype=torch.bfloat16, device=dev, with_norms=True)
    X0 = next(st).clone()
    n0 = st.last_norms.clone()
    X1 = torch.empty_like(X0)
    n1 = torch.empty_like(n0)
    eng = MiniBatchEngine(K, D, b, dtype=torch.bfloat16, device=dev, value_bound=st.value_bound)
    eng.set_centers(X0[:K].float())
    eng.partial_fit(X0, n0)   # scales, kernel attributes
    C = eng._C
    lab = eng.labels

    def upd():
        C.update(X0, lab, K, eng.slab, eng.cnt_slab, eng.n_chunks, None, eng.col_exp, 0, False,
                 clamp_count=None)

    def gen():
        make_blobs(b, D, 0, seed=1, i0=b, dtype=torch.bfloat16, device=dev, centers=st.centers,
                   out=X1, norms=n1)

    def asg():
        eng.pk.assign(X0, n0, lab, None, eng.slots, False)

    side = torch.cuda.Stream(device=dev)
    main_s = torch.cuda.current_stream(dev)

    def timed(fn_main, fn_side=None, reps=10):
        ts = []
        for _ in range(reps):
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(main_s)
            if fn_side is not None:
                side.wait_event(e0)
                with torch.cuda.stream(side):
                    fn_side()
            fn_main()
            if fn_side is not None:
                main_s.wait_stream(side)
            e1.record(main_s)
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        ts.sort()
        return round(ts[len(ts) // 2], 4)

    out = {}
    for _ in range(2):
        out["update"] = timed(upd)
        out["gen"] = timed(gen)
        out["assign"] = timed(asg)
        out["update+gen"] = timed(upd, gen)
        out["assign+gen"] = timed(asg, gen)
        out["update_then_gen_serial"] = timed(lambda: (upd(), gen()))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
