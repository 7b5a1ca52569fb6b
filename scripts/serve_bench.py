#!/usr/bin/env python3
"""Serving throughput of a fitted model on one MI355X: the in-process ``predict`` on
device-resident and host rows, and the HTTP service (``mikmeans.serve``, uvicorn on
127.0.0.1) answering ``POST /api/predict.npy`` batches and small ``POST /api/predict``
JSON requests.  K=1024 centres of D=128 features fitted on synthetic blobs (a short fit:
the centres' quality does not change the work of a predict).

usage: serve_bench.py [--k 1024] [--d 128] [--dtype bfloat16|float32]
Prints one JSON line per measurement and a summary line."""
import argparse
import io
import json
import os
import socket
import statistics
import sys
import threading
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from mikmeans import KMeans  # noqa: E402
from mikmeans.data.blobs import blob_centers, make_blobs  # noqa: E402


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _timed(fn, reps: int, sync: bool = True) -> float:
    sync = sync and torch.cuda.is_available()
    fn()
    if sync:
        torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        if sync:
            torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=1024)
    ap.add_argument("--d", type=int, default=128)
    ap.add_argument("--dtype", default="bfloat16")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--device", default="cuda", help="cpu: a dry run of the script on the torch path")
    ap.add_argument("--sizes", default="1000,100000,10000000", help="device-resident predict batch sizes")
    ap.add_argument("--fit-rows", type=int, default=500_000)
    a = ap.parse_args()
    dev = torch.device(a.device)
    tdt = torch.bfloat16 if a.dtype == "bfloat16" else torch.float32
    C = blob_centers(a.k, a.d, 10.0, 0, device=dev)
    Xfit = make_blobs(a.fit_rows, a.d, a.k, seed=1, dtype=tdt, device=dev, centers=C)
    km = KMeans(a.k, init="random", max_iter=3, dtype=a.dtype, algorithm="lloyd").fit(Xfit)
    out = {"k": a.k, "d": a.d, "dtype": a.dtype}

    def put(name, rows, sec, **kw):
        rec = {"rows": rows, "ms": round(sec * 1e3, 3), "rows_per_s": round(rows / sec, 1), **kw}
        out[name] = rec
        print(json.dumps({name: rec}), flush=True)

    # in-process predict, rows already on the device (the kernel and its launch)
    for n in [int(v) for v in a.sizes.split(",")]:
        X = make_blobs(n, a.d, a.k, seed=2, dtype=tdt, device=dev, centers=C)
        put(f"predict_device_{n}", n, _timed(lambda X=X: km.predict(X), a.reps))
        del X
    # host float32 rows (copied to the device in ~256 MB blocks, converted there)
    nh = 1_000_000 if dev.type == "cuda" else 20_000
    Xh = make_blobs(nh, a.d, a.k, seed=3, dtype=torch.float32, device=dev, centers=C).cpu().numpy()
    put(f"predict_host_f32_{nh}", Xh.shape[0], _timed(lambda: km.predict(Xh), a.reps))

    # the HTTP service
    import httpx
    import uvicorn

    from mikmeans import serve

    app = serve.create_app(model=km, max_body_bytes=1 << 30, max_rows=1 << 22)
    port = _free_port()
    server = uvicorn.Server(uvicorn.Config(app, host="127.0.0.1", port=port, log_level="warning"))
    th = threading.Thread(target=server.run, daemon=True)
    th.start()
    deadline = time.time() + 60
    while not server.started and time.time() < deadline:
        time.sleep(0.05)
    if not server.started:
        raise SystemExit("uvicorn did not start")
    url = f"http://127.0.0.1:{port}"
    try:
        with httpx.Client(timeout=120.0) as cl:
            for n in ((4_096, 65_536, 262_144) if dev.type == "cuda" else (1_024, 4_096)):
                buf = io.BytesIO()
                np.save(buf, Xh[:n], allow_pickle=False)
                body = buf.getvalue()

                def call(body=body, n=n):
                    r = cl.post(url + "/api/predict.npy", content=body,
                                headers={"Content-Type": "application/octet-stream"})
                    r.raise_for_status()
                    lab = np.load(io.BytesIO(r.content), allow_pickle=False)
                    assert lab.shape == (n,)
                put(f"http_npy_{n}", n, _timed(call, a.reps, sync=False), body_MB=round(len(body) / 1e6, 2))
            pts = Xh[:64].tolist()

            def small():
                r = cl.post(url + "/api/predict", json={"points": pts})
                r.raise_for_status()
            put("http_json_64", 64, _timed(small, 4 * a.reps, sync=False))
            # the served labels are the in-process ones
            buf = io.BytesIO()
            np.save(buf, Xh[:4096], allow_pickle=False)
            r = cl.post(url + "/api/predict.npy", content=buf.getvalue())
            served = np.load(io.BytesIO(r.content), allow_pickle=False)
            out["http_labels_equal_predict"] = bool((served == km.predict(Xh[:4096]).astype(np.int32)).all())
    finally:
        server.should_exit = True
        th.join(timeout=10)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
