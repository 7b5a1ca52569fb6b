"""A/B the blob generator's lanes-per-row cap (MIKMEANS_BLOBS_TPR) at the cfg5 batch shape.
Each variant runs in a child process (the cap is read once per process); the batch bytes
are hashed to show every variant generates identical data."""
import json, os, subprocess, sys

CHILD = r'''
import hashlib, torch, mikmeans
from mikmeans.data.blobs import blob_centers, make_blobs
D, K, b = 256, 512, 1 << 24
C = blob_centers(K, D, 10.0, 0, device="cuda")
X = torch.empty((b, D), dtype=torch.bfloat16, device="cuda"); nrm = torch.empty(b, device="cuda")
for _ in range(3): make_blobs(b, D, K, seed=0, i0=123, dtype=torch.bfloat16, device="cuda", centers=C, out=X, norms=nrm)
torch.cuda.synchronize()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
ts = []
for _ in range(10):
    ev[0].record(); make_blobs(b, D, K, seed=0, i0=123, dtype=torch.bfloat16, device="cuda", centers=C, out=X, norms=nrm); ev[1].record()
    torch.cuda.synchronize(); ts.append(ev[0].elapsed_time(ev[1]))
h = hashlib.sha1(X[:65536].view(torch.int16).cpu().numpy().tobytes()).hexdigest()[:12] + "/" + hashlib.sha1(nrm[:65536].cpu().numpy().tobytes()).hexdigest()[:6]
print(sorted(ts)[len(ts)//2], h)
'''
res = {}
for rnd in range(1):
    for tpr in (16, 8, 4):
        env = dict(os.environ, MIKMEANS_BLOBS_TPR=str(tpr))
        out = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=120)
        line = [l for l in out.stdout.splitlines() if l.strip()][-1]
        ms, h = line.split()
        res.setdefault(str(tpr), []).append({"ms": round(float(ms), 4), "hash": h})
        print(tpr, ms, h, flush=True)
json.dump({"shape": "16.8M x 256 bf16, K=512", "median_ms_and_hash_by_tpr_cap": res},
          open("gpurun_out/blobs_tpr_ab.json", "w"), indent=1)
