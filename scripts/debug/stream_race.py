"""Debug: the chunk-copy / buffer zero-fill race of the streaming engine.  Builds the engine
behind a busy caller stream with the copy stream's wait disabled (the pre-fix behaviour)
and enabled, and reports whether chunk 0's row norms came out right."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from mikmeans.data import blobs as B
from mikmeans.models.streaming import StreamingLloydEngine

X = B.make_blobs(40_000, 32, 16, seed=5, dtype=torch.bfloat16, device="cpu")
ref = X.to("cuda").float().pow(2).sum(1)
orig = torch.cuda.Stream.wait_stream
for label, patch in (("no wait (old)", True), ("wait (fixed)", False)):
    if patch:
        torch.cuda.Stream.wait_stream = lambda self, other: None
    torch.cuda._sleep(200_000_000)
    eng = StreamingLloydEngine(X, 16, chunk_rows=1 << 13, device="cuda", dtype=torch.bfloat16)
    torch.cuda.Stream.wait_stream = orig
    bad = int((~torch.isclose(eng.xn, ref, rtol=1e-5, atol=1e-4)).sum())
    print(label, "rows with wrong norms:", bad, "first chunk rows:", eng.ranges[0], flush=True)
    eng.close()
