"""HTTP service: the room board (the reference's page, ``index.html`` + ``app.mjs``) and
model serving (nearest-centre labels on the MFMA assign kernel) behind one FastAPI app.

The reference is a static page whose state lives in the browser and travels between peers
(``app.mjs:39-118``); here the room lives in this process (:class:`~mikmeans.models.room.Room`,
every mutation under one lock) and the page talks to it over a small JSON API.  The
reference's ``_headers`` policy is kept, minus the CDNs and WebRTC trackers the page no
longer needs: ``default-src 'none'``, scripts and fetches from this origin only, no
framing, no referrer, no camera / microphone / geolocation / payment, ``nosniff``
(``_headers:1-22``).

Endpoints (JSON in and out):

* ``GET /`` the board page, ``GET /app.js`` its script;
* ``GET /api/room`` the export JSON, byte-exact ``JSON.stringify(state, null, 2)``
  (``app.mjs:263-267``); ``POST /api/room/import`` replaces cards / centroids, merges meta
  (``app.mjs:268-282``);
* ``POST /api/cards`` {title, traits}; ``POST /api/centroids`` {name} (at most 3,
  ``app.mjs:126-129``); ``POST /api/assign`` {card, centroid|null} (the drop / select
  paths, locks respected); ``POST /api/centroids/{id}/lock``, ``DELETE /api/centroids/{id}``;
* ``POST /api/auto`` numeric k-means over the cards' trait vectors; ``GET /api/dashboard``;
* ``GET /api/model`` the served model's centroids as flat floats; ``POST /api/predict``
  {points[, distances]} -> labels (and squared distances), ``POST /api/predict.npy`` (a
  ``.npy`` body in, ``.npy`` labels out), ``POST /api/transform``.

``mikmeans serve [--room FILE] [--model DIR] [--host 127.0.0.1] [--port 8000]``.
"""
from __future__ import annotations

import threading

import numpy as np
import torch
from fastapi import Body, FastAPI, HTTPException, Request
from fastapi.responses import HTMLResponse, Response

from .models.room import Room

SECURITY_HEADERS = {
    "Content-Security-Policy": ("default-src 'none'; script-src 'self'; script-src-elem 'self'; "
                                "script-src-attr 'none'; style-src 'self' 'unsafe-inline'; img-src 'self' data:; "
                                "connect-src 'self'; base-uri 'none'; frame-ancestors 'none'"),
    "Referrer-Policy": "no-referrer",
    "Permissions-Policy": "camera=(), microphone=(), geolocation=(), payment=()",
    "X-Content-Type-Options": "nosniff",
}

PAGE = """<!doctype html>
<html lang="en"><head><meta charset="utf-8"><title>k-means room</title>
<style>
body{font-family:system-ui,sans-serif;margin:1rem;background:#fafafa}
.zones{display:flex;gap:1rem;flex-wrap:wrap}
.zone{border:2px solid #ccc;border-radius:8px;padding:.5rem;min-width:14rem;background:#fff}
.card{border:1px solid #ddd;border-radius:6px;padding:.25rem .5rem;margin:.25rem 0}
.traits{color:#666;font-size:.85em}
#dash{white-space:pre-wrap;font-family:monospace;font-size:.85em}
</style></head>
<body>
<h1>k-means room <span id="room"></span></h1>
<p><input id="title" placeholder="card title"> <input id="traits" placeholder="traits, comma separated">
<button id="addCard">Add card</button>
<input id="cname" placeholder="centroid name"> <button id="addCentroid">Add centroid</button>
<button id="auto">Auto-assign (k-means)</button> <a href="/api/room" download>Export JSON</a></p>
<div class="zones" id="zones"></div>
<h2>Dashboard</h2><div id="dash"></div>
<script src="/app.js"></script>
</body></html>
"""

APP_JS = """'use strict';
async function api(path, method, body) {
  const r = await fetch(path, {method: method || 'GET', headers: {'Content-Type': 'application/json'},
                               body: body ? JSON.stringify(body) : undefined});
  if (!r.ok) throw new Error(await r.text());
  return r.json();
}
function el(tag, cls, text) { const e = document.createElement(tag); if (cls) e.className = cls;
  if (text !== undefined) e.textContent = text; return e; }
function cardEl(card, centroids) {
  const d = el('div', 'card');
  d.appendChild(el('div', '', card.title));
  d.appendChild(el('div', 'traits', (card.traits || []).join(', ')));
  const s = el('select');
  s.appendChild(new Option('unassigned', ''));
  for (const c of centroids) s.appendChild(new Option(c.name, c.id));
  s.value = card.assignedTo || '';
  s.addEventListener('change', () => api('/api/assign', 'POST', {card: card.id, centroid: s.value || null}).then(render));
  d.appendChild(s);
  return d;
}
async function render() {
  const st = await api('/api/state');
  document.getElementById('room').textContent = st.room;
  const zones = document.getElementById('zones');
  zones.replaceChildren();
  const groups = [{id: null, name: 'Unassigned', color: '#999'}].concat(st.centroids);
  for (const g of groups) {
    const z = el('div', 'zone');
    z.style.borderColor = g.color || '#ccc';
    z.appendChild(el('h3', '', g.name + (g.locked ? ' (locked)' : '')));
    for (const card of st.cards.filter(c => (c.assignedTo || null) === g.id)) z.appendChild(cardEl(card, st.centroids));
    zones.appendChild(z);
  }
  document.getElementById('dash').textContent = JSON.stringify(st.dashboard, null, 2);
}
document.getElementById('addCard').addEventListener('click', () => {
  const t = document.getElementById('title').value.trim();
  const tr = document.getElementById('traits').value.split(',').map(s => s.trim()).filter(Boolean);
  if (t) api('/api/cards', 'POST', {title: t, traits: tr}).then(render);
});
document.getElementById('addCentroid').addEventListener('click', () => {
  api('/api/centroids', 'POST', {name: document.getElementById('cname').value.trim() || null}).then(render);
});
document.getElementById('auto').addEventListener('click', () => api('/api/auto', 'POST', {}).then(render));
render();
"""


def _jsonable(obj):
    """Non-finite floats as JSON null (what the reference's JSON.stringify writes for
    Infinity / NaN, e.g. the dashboard's unbounded balance ratio)."""
    import math

    if isinstance(obj, float):
        return obj if math.isfinite(obj) else None
    if isinstance(obj, dict):
        return {k: _jsonable(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return [_jsonable(v) for v in obj]
    return obj


def create_app(room: Room | None = None, model=None, *, device=None):
    """The FastAPI app serving ``room`` (a new one when None) and, when given, a fitted
    ``model`` (:class:`~mikmeans.KMeans` / :class:`~mikmeans.MiniBatchKMeans`)."""
    app = FastAPI(title="mikmeans", docs_url=None, redoc_url=None, openapi_url=None)
    state = {"room": room if room is not None else Room(seed=0)}
    lock = threading.Lock()

    @app.middleware("http")
    async def _headers(request, call_next):
        resp = await call_next(request)
        for k, v in SECURITY_HEADERS.items():
            resp.headers[k] = v
        return resp

    def _room() -> Room:
        return state["room"]

    @app.get("/", response_class=HTMLResponse)
    def page():
        return HTMLResponse(PAGE)

    @app.get("/app.js")
    def app_js():
        return Response(APP_JS, media_type="text/javascript")

    @app.get("/api/room")
    def export_room():
        with lock:
            txt = _room().export_json()
            name = _room().export_filename
        return Response(txt, media_type="application/json",
                        headers={"Content-Disposition": f'attachment; filename="{name}"'})

    @app.get("/api/state")
    def room_state():
        with lock:
            r = _room()
            return _jsonable({"room": r.room, "cards": r.cards, "centroids": r.centroids,
                              "dashboard": r.dashboard()})

    @app.post("/api/room/import")
    def import_room(body: dict = Body(...)):
        import json

        with lock:
            _room().import_json(json.dumps(body))
            return {"cards": len(_room().cards), "centroids": len(_room().centroids)}

    @app.post("/api/cards")
    def add_card(body: dict = Body(...)):
        title = str(body.get("title", "")).strip()
        if not title:
            raise HTTPException(400, "title required")
        traits = body.get("traits", [])
        with lock:
            return _room().add_card(title, traits)

    @app.post("/api/centroids")
    def add_centroid(body: dict = Body(default={})):
        with lock:
            c = _room().add_centroid(body.get("name") or None)
        if c is None:
            raise HTTPException(409, "at most %d centroids" % _room().max_centroids)
        return c

    @app.post("/api/centroids/{cid}/lock")
    def toggle_lock(cid: str):
        with lock:
            _room().toggle_lock(cid)
            return {"locked": bool((_room()._centroid(cid) or {}).get("locked"))}

    @app.delete("/api/centroids/{cid}")
    def remove_centroid(cid: str):
        with lock:
            _room().remove_centroid(cid)
            return {"centroids": len(_room().centroids)}

    @app.post("/api/assign")
    def assign(body: dict = Body(...)):
        with lock:
            ok = _room().update_card_assign(body.get("card"), body.get("centroid") or None)
        if not ok:
            raise HTTPException(409, "not assigned (unknown card or locked centroid)")
        return {"ok": True}

    @app.post("/api/auto")
    def auto(body: dict = Body(default={})):
        with lock:
            return _jsonable(_room().auto_assign(seed=int(body.get("seed", 0))))

    @app.get("/api/dashboard")
    def dashboard():
        with lock:
            return _jsonable(_room().dashboard())

    # ------------------------------------------------------------------- model serving
    def _model():
        if model is None:
            raise HTTPException(404, "no model loaded (mikmeans serve --model DIR)")
        return model

    @app.get("/api/model")
    def model_info():
        m = _model()
        C = m.cluster_centers_.float().cpu()
        return {"n_clusters": int(C.shape[0]), "n_features": int(C.shape[1]),
                "centroids": [float(v) for v in C.reshape(-1).tolist()]}

    def _points(body: dict) -> torch.Tensor:
        pts = body.get("points")
        if not isinstance(pts, list) or not pts:
            raise HTTPException(400, "points: a non-empty list of rows")
        X = torch.as_tensor(np.asarray(pts, dtype=np.float32))
        m = _model()
        if X.dim() != 2 or X.shape[1] != m.cluster_centers_.shape[1]:
            raise HTTPException(400, f"points must be [n, {m.cluster_centers_.shape[1]}]")
        return X.to(m.cluster_centers_.device)

    @app.post("/api/predict")
    def predict(body: dict = Body(...)):
        m = _model()
        X = _points(body)
        with lock:   # (one batch at a time on the device: the serving pack is shared)
            labels, mind, _ = m._assign_rows(X, bool(body.get("distances", False)))
        out = {"labels": labels.cpu().tolist()}
        if mind is not None:
            out["distances"] = mind.cpu().tolist()
        return out

    @app.post("/api/predict.npy")
    async def predict_npy(request: Request):
        """Binary serving: the body is a ``.npy`` array [n, D] (``numpy.save``; loaded with
        ``allow_pickle=False``), the answer the int32 labels as ``.npy`` -- no JSON
        parsing of large batches."""
        import io

        m = _model()
        raw = await request.body()
        try:
            arr = np.load(io.BytesIO(raw), allow_pickle=False)
        except Exception as e:  # noqa: BLE001 -- any malformed payload is the client's error
            raise HTTPException(400, f"body must be a .npy array: {e}") from None
        if arr.ndim != 2 or arr.shape[1] != m.cluster_centers_.shape[1]:
            raise HTTPException(400, f"array must be [n, {m.cluster_centers_.shape[1]}]")
        X = torch.as_tensor(np.ascontiguousarray(arr, dtype=np.float32)).to(m.cluster_centers_.device)
        with lock:
            labels, _, _ = m._assign_rows(X, False)
        buf = io.BytesIO()
        np.save(buf, labels.cpu().numpy().astype(np.int32), allow_pickle=False)
        return Response(buf.getvalue(), media_type="application/octet-stream")

    @app.post("/api/transform")
    def transform(body: dict = Body(...)):
        m = _model()
        X = _points(body)
        with lock:
            d = m.transform(X)
        return {"distances": d.cpu().tolist()}

    return app


def serve(room_path=None, model_path=None, host: str = "127.0.0.1", port: int = 8000, device=None):
    """Run the app with uvicorn (blocking)."""
    import uvicorn

    room = None
    if room_path:
        with open(room_path) as f:
            room = Room.from_json(f.read())
    model = None
    if model_path:
        from .api import KMeans

        model = KMeans.load(model_path, device=device)
    uvicorn.run(create_app(room, model), host=host, port=port, log_level="warning")
