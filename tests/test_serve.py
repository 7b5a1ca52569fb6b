"""The HTTP service (mikmeans/serve.py): the reference's page and security headers, the
room API against the Room model, and model serving against KMeans.predict (CPU)."""
import json

import numpy as np
import pytest
import torch

pytest.importorskip("fastapi")
pytest.importorskip("httpx")

from fastapi.testclient import TestClient  # noqa: E402

import mikmeans  # noqa: E402
from mikmeans.models.room import Room  # noqa: E402
from mikmeans.serve import SECURITY_HEADERS, create_app  # noqa: E402


def _client(room=None, model=None):
    return TestClient(create_app(room, model))


def test_page_and_security_headers():
    """The page and its script come from this origin; every response carries the
    reference's `_headers` policy (no CDNs / trackers left to allow)."""
    c = _client(Room(seed=1))
    r = c.get("/")
    assert r.status_code == 200 and "<script src=\"/app.js\"></script>" in r.text
    js = c.get("/app.js")
    assert js.status_code == 200 and js.headers["content-type"].startswith("text/javascript")
    for resp in (r, js, c.get("/api/dashboard")):
        for k, v in SECURITY_HEADERS.items():
            assert resp.headers[k] == v
    assert "default-src 'none'" in SECURITY_HEADERS["Content-Security-Policy"]
    assert "frame-ancestors 'none'" in SECURITY_HEADERS["Content-Security-Policy"]


def test_room_api_matches_room_model():
    """The JSON API drives the same Room operations as the reference's handlers: at most 3
    centroids, locks respected, export byte-exact, import round trip."""
    room = Room(seed=3, clock=lambda: 1_700_000_000_000)
    c = _client(room)
    a = c.post("/api/centroids", json={"name": "Sweet"}).json()
    c.post("/api/centroids", json={"name": "Sour"})
    c.post("/api/centroids", json={})
    assert c.post("/api/centroids", json={"name": "Fourth"}).status_code == 409
    card = c.post("/api/cards", json={"title": "Mango", "traits": ["Fruity", "Sweet"]}).json()
    assert c.post("/api/cards", json={"title": "  "}).status_code == 400
    assert c.post("/api/assign", json={"card": card["id"], "centroid": a["id"]}).json() == {"ok": True}
    assert room.cards[-1]["assignedTo"] == a["id"]
    assert c.post(f"/api/centroids/{a['id']}/lock").json() == {"locked": True}
    other = c.post("/api/cards", json={"title": "Lime", "traits": ["Sour"]}).json()
    assert c.post("/api/assign", json={"card": other["id"], "centroid": a["id"]}).status_code == 409
    exp = c.get("/api/room")
    assert exp.text == room.export_json()
    assert exp.headers["content-disposition"].endswith(f'"{room.export_filename}"')
    st = c.get("/api/state").json()
    assert st["room"] == room.room and len(st["cards"]) == len(room.cards)
    from mikmeans.serve import _jsonable

    assert c.get("/api/dashboard").json() == _jsonable(room.dashboard())
    r2 = Room(seed=4)
    c2 = _client(r2)
    assert c2.post("/api/room/import", json=json.loads(exp.text)).json()["centroids"] == 3
    assert [x["id"] for x in r2.cards] == [x["id"] for x in room.cards]
    assert c.post("/api/auto", json={"seed": 0}).status_code == 200


def test_model_serving_matches_predict():
    """/api/predict and /api/transform give KMeans.predict / transform's answers; bad shapes
    are refused; without a model the endpoints say so."""
    X = torch.as_tensor(np.random.default_rng(0).normal(size=(500, 5)), dtype=torch.float32)
    km = mikmeans.KMeans(4, device="cpu", seed=1).fit(X)
    c = _client(Room(seed=0), km)
    info = c.get("/api/model").json()
    assert info["n_clusters"] == 4 and len(info["centroids"]) == 20
    r = c.post("/api/predict", json={"points": X[:50].tolist(), "distances": True}).json()
    assert r["labels"] == km.predict(X[:50]).tolist()
    assert len(r["distances"]) == 50
    t = c.post("/api/transform", json={"points": X[:3].tolist()}).json()["distances"]
    assert np.allclose(np.asarray(t), km.transform(X[:3]).numpy(), rtol=1e-5, atol=1e-5)
    assert c.post("/api/predict", json={"points": [[1.0, 2.0]]}).status_code == 400
    import io

    buf = io.BytesIO()
    np.save(buf, X[:200].numpy())
    rb = c.post("/api/predict.npy", content=buf.getvalue(), headers={"Content-Type": "application/octet-stream"})
    assert rb.status_code == 200
    lab = np.load(io.BytesIO(rb.content), allow_pickle=False)
    assert lab.dtype == np.int32 and lab.tolist() == km.predict(X[:200]).tolist()
    assert c.post("/api/predict.npy", content=b"not npy").status_code == 400
    assert _client(Room(seed=0)).post("/api/predict", json={"points": [[0.0] * 5]}).status_code == 404


def test_cli_serve_process(tmp_path):
    """`python -m mikmeans serve` binds 127.0.0.1, serves the page and a room loaded from an
    export file, and stops cleanly."""
    import os
    import subprocess
    import sys
    import time
    import urllib.request

    from mikmeans.parallel.launch import free_port

    room = Room(seed=5)
    room.add_centroid("Sweet")
    (tmp_path / "r.json").write_text(room.export_json())
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    port = free_port()
    p = subprocess.Popen([sys.executable, "-m", "mikmeans", "serve", "--port", str(port), "--room",
                          str(tmp_path / "r.json")], cwd=root, stdout=subprocess.PIPE, stderr=subprocess.PIPE)
    try:
        body = None
        for _ in range(100):
            try:
                with urllib.request.urlopen(f"http://127.0.0.1:{port}/api/room", timeout=2) as r:
                    body = r.read().decode()
                    hdr = r.headers
                break
            except OSError:
                time.sleep(0.2)
        assert body is not None, p.stderr.read1(4000) if p.poll() is not None else "server did not come up"
        assert json.loads(body)["centroids"][0]["name"] == "Sweet"
        assert hdr["X-Content-Type-Options"] == "nosniff"
    finally:
        p.terminate()
        p.wait(timeout=20)


def test_concurrent_room_edits_are_serialised():
    """Many clients adding cards at once: every edit lands exactly once (one lock around the
    room, as the reference's single-threaded page has no concurrent handlers)."""
    from concurrent.futures import ThreadPoolExecutor

    room = Room(seed=6)
    c = _client(room)
    n0 = len(room.cards)

    def add(i):
        return c.post("/api/cards", json={"title": f"card {i}", "traits": ["T"]}).status_code

    with ThreadPoolExecutor(8) as ex:
        codes = list(ex.map(add, range(64)))
    assert codes == [200] * 64
    titles = sorted(x["title"] for x in room.cards[n0:])
    assert titles == sorted(f"card {i}" for i in range(64))
    assert len({x["id"] for x in room.cards}) == len(room.cards)
