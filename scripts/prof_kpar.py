#!/usr/bin/env python3
"""k-means|| seeding at the cfg4 shape (N=1e7, D=64, K=4096, bf16) for rocprofv3: one warm-up
seeding, then one timed; prints the timed seconds.  The recluster runs on csrc/kpp.hip wkpp.

usage: rocprofv3 --kernel-trace --stats -d <dir> -- python3 scripts/prof_kpar.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from mikmeans.data.blobs import blob_centers, make_blobs  # noqa: E402
from mikmeans.models.init import init_kmeans_parallel  # noqa: E402
from mikmeans.parallel import Comm  # noqa: E402

N, D, K = 10_000_000, 64, 4096
dev = torch.device("cuda")
comm = Comm.local(dev)
X = make_blobs(N, D, K, seed=0, dtype=torch.bfloat16, device=dev, centers=blob_centers(K, D, 10.0, 0, device=dev))
for rep in range(int(os.environ.get("KPAR_REPS", "2"))):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    C = init_kmeans_parallel(X, D, K, N, 0, comm, seed=0)
    torch.cuda.synchronize()
    print(f"init_kmeans_parallel rep {rep}: {time.perf_counter() - t0:.3f} s", flush=True)
