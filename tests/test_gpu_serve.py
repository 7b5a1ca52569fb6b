"""Model serving over HTTP on the GPU: /api/predict and /api/transform run the MFMA assign /
transform kernels on the fitted model's serving pack (mikmeans/serve.py)."""
import numpy as np
import pytest
import torch

pytest.importorskip("fastapi")
pytest.importorskip("httpx")

pytestmark = pytest.mark.gpu


def test_gpu_model_serving(native):
    from fastapi.testclient import TestClient

    import mikmeans
    from mikmeans.data import blobs as B
    from mikmeans.serve import create_app

    X = B.make_blobs(50_000, 96, 20, seed=3, device="cuda")
    km = mikmeans.KMeans(20, dtype="bfloat16", device="cuda", max_iter=10, seed=1).fit(X)
    c = TestClient(create_app(None, km))
    q = X[:2000].cpu()
    r = c.post("/api/predict", json={"points": q.tolist(), "distances": True}).json()
    assert r["labels"] == km.predict(q.cuda()).cpu().tolist()
    t = np.asarray(c.post("/api/transform", json={"points": q[:10].tolist()}).json()["distances"])
    assert np.allclose(t, km.transform(q[:10].cuda()).cpu().numpy(), rtol=1e-5, atol=1e-4)
    assert int(np.argmin(t, 1)[0]) == r["labels"][0] or np.isclose(np.sort(t[0])[0], np.sort(t[0])[1])
