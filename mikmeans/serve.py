"""HTTP service: the room board (the reference's page, ``index.html`` + ``app.mjs``) and
model serving (nearest-centre labels on the MFMA assign kernel) behind one FastAPI app.

The reference is a static page whose state lives in the browser and travels between peers
(``app.mjs:39-118``); every replicated change re-renders every peer (``ydoc.on("update")``
broadcast, ``app.mjs:121``, then ``observeDeep`` -> ``renderAll``, ``app.mjs:579-580``).  Here
the room lives in this process (:class:`~mikmeans.models.room.Room`, every mutation under one
lock) and bumps a change counter; every open page long-polls ``/api/changes`` and re-renders
on any edit, its own or another browser's.  The reference's ``_headers`` policy is kept,
minus the CDNs and WebRTC trackers the page no longer needs: ``default-src 'none'``, scripts
and fetches from this origin only, no framing, no referrer, no camera / microphone /
geolocation / payment, ``nosniff`` (``_headers:1-22``).

Endpoints (JSON in and out) -- the reference's controls (``index.html:76-131``,
``app.mjs:240-288, 571-573``):

* ``GET /`` the board page, ``GET /app.js`` its script;
* ``GET /api/state`` cards, centroids, meta, card positions, dashboard, presence and the
  change ``version``; ``GET /api/changes?since=V&wait=S&user=NAME`` (async) answers as soon as
  the version passes ``V`` (or after ``S`` <= 25 seconds) -- the live-update channel, whose
  polling names are the presence list (the reference's Peers chip and avatars, app.mjs:51-65);
* ``GET /api/room`` the export JSON, byte-exact ``JSON.stringify(state, null, 2)``
  (``app.mjs:263-267``); ``POST /api/room/import`` replaces cards / centroids, merges meta
  (``app.mjs:268-282``);
* cards: ``POST /api/cards`` {title, traits[, user]}, ``DELETE /api/cards/{id}``,
  ``POST /api/assign`` {card, centroid|null} (the ``<select>`` path, app.mjs:398-402),
  ``POST /api/drop`` {card, centroid|null, x, y} (drag-and-drop: the clamped ``pos:<id>`` with
  the assignment, locks respected, app.mjs:356-372; null = onto Unassigned, app.mjs:421-433),
  ``POST /api/populate`` (test data), ``POST /api/shuffle_unassigned``, ``POST /api/restart``
  (unassign all), ``POST /api/reset`` {mode?} (hard reset);
* centroids (at most 3, ``app.mjs:126-129``): ``POST /api/centroids`` {name},
  ``POST /api/centroids/{id}/rename`` {name}, ``POST /api/centroids/{id}/apply_suggestion``,
  ``POST /api/centroids/{id}/lock``, ``DELETE /api/centroids/{id}``;
* meta: ``POST /api/mode`` {mode}, ``POST /api/iteration`` {value}; tools: ``GET /api/coin``,
  ``GET /api/d12``, ``GET /api/shuffle_names``, ``GET /api/link?base=URL``;
* ``POST /api/auto`` numeric k-means over the cards' trait vectors; ``GET /api/dashboard``;
* ``GET /api/model`` the served model's shape and centroids, ``GET /api/model/centroids.json``
  the flat-float centroid array byte-identical to a saved ``centroids.json``
  (:func:`~mikmeans.utils.jsjson.centroids_to_json`); ``POST /api/predict``
  {points[, distances]} -> labels (and squared distances), ``POST /api/predict.npy`` (a
  ``.npy`` body in, ``.npy`` labels out), ``POST /api/transform``.

Request bodies over ``max_body_bytes`` get 413 -- declared or counted as they stream in (chunked) --
as do batches over ``max_rows`` rows (and
transforms over ``max_transform_values`` output values); malformed input gets 400.

Session mode (``--found [ROOM]`` / ``--join``, ``--store-host/--store-port``): the served
room is one member of a live replicated session (:class:`~mikmeans.parallel.elastic.
ElasticRoomReplica`, the reference's peer mesh, ``app.mjs:70-118``): edits are queued (202)
and every member applies them in the same order at the next round, so boards served by
different processes -- and scripted ``mikmeans session`` members -- stay byte-identical.

``mikmeans serve [--room FILE] [--model DIR] [--host 127.0.0.1] [--port 8000] [--found|--join]``.
"""
from __future__ import annotations

import asyncio
import threading
import time

import numpy as np
import torch
from fastapi import Body, FastAPI, HTTPException, Request
from fastapi.responses import HTMLResponse, JSONResponse, Response

from .models.room import Room

SECURITY_HEADERS = {
    "Content-Security-Policy": ("default-src 'none'; script-src 'self'; script-src-elem 'self'; "
                                "script-src-attr 'none'; style-src 'self' 'unsafe-inline'; img-src 'self' data:; "
                                "connect-src 'self'; base-uri 'none'; frame-ancestors 'none'"),
    "Referrer-Policy": "no-referrer",
    "Permissions-Policy": "camera=(), microphone=(), geolocation=(), payment=()",
    "X-Content-Type-Options": "nosniff",
}

MAX_BODY_BYTES = 64 << 20          # request bodies (a .npy batch of 1M x 16 f32 rows fits)
MAX_ROWS = 1 << 20                 # rows per predict / transform batch
MAX_TRANSFORM_VALUES = 1 << 24     # n x K distances per transform answer
LONG_POLL_S = 25.0

PAGE = """<!doctype html>
<html lang="en"><head><meta charset="utf-8"><title>k-means room</title>
<style>
body{font-family:system-ui,sans-serif;margin:1rem;background:#fafafa;color:#222}
.row{display:flex;gap:.5rem;flex-wrap:wrap;align-items:center;margin:.35rem 0}
.board{display:grid;grid-template-columns:1fr 18rem;gap:1rem}
.zones{display:grid;grid-template-columns:repeat(auto-fit,minmax(15rem,1fr));gap:1rem}
.zone{position:relative;border:2px solid #ccc;border-radius:8px;padding:.5rem;background:#fff;min-height:16rem}
.zone.over{background:#eef4ff}
.zone .head{display:flex;gap:.3rem;flex-wrap:wrap;align-items:center;margin-bottom:.3rem}
.swatch{width:.9rem;height:.9rem;border-radius:3px;display:inline-block}
.card{border:1px solid #ddd;border-radius:6px;padding:.25rem .5rem;margin:.25rem 0;background:#fff;cursor:grab}
.card.float{position:absolute;width:11rem;margin:0;box-shadow:0 2px 6px rgba(0,0,0,.15)}
.card.dragging{opacity:.5}
.traits{color:#666;font-size:.85em}
#unassigned{border:2px dashed #bbb;border-radius:8px;padding:.5rem;min-height:16rem;background:#fff}
#unassigned.over{background:#eef4ff}
.chip{border:1px solid #ccc;border-radius:99px;padding:.1rem .6rem;font-size:.85em;display:inline-block}
.chip.ok{background:#e8f7ec;border-color:#8fcf9f}.chip.warn{background:#fdf5e0;border-color:#e0c070}
.avatar{width:1.7rem;height:1.7rem;border-radius:50%;border:1px solid #bbb;display:inline-grid;place-items:center;font-size:.7em;font-weight:700;background:#eee}
.kmrow{display:flex;gap:.5rem;align-items:center;margin:.3rem 0;white-space:nowrap}
.bar{flex:1;min-width:6rem;height:.5rem;border:1px solid #ccc;border-radius:99px;overflow:hidden;background:#f3f3f3}
.fill{height:100%}
.delta{font-size:.8em;color:#2b6be0}.delta.bad{color:#c0392b}
.top{font-size:.8em;color:#555;overflow:hidden;text-overflow:ellipsis}
</style></head>
<body>
<h1>k-means room <span id="room" class="chip"></span> <span id="status" class="chip"></span>
<span id="presence"></span> <span id="version" class="chip"></span></h1>
<div class="row"><button id="copy">Copy link</button> <button id="populate">Populate test data</button>
<label>Your name <input id="name" placeholder="e.g., Alex"></label> <button id="saveName">Save</button></div>
<div class="row"><input id="cname" placeholder="centroid name"> <button id="addCentroid">Add centroid (max 3)</button>
<button id="coin">Coin flip</button> <button id="d12">d12</button> <button id="shuffle">Shuffle names</button>
<button id="shuffleUnassigned">Randomize Unassigned</button> <button id="restartAll">Restart (Unassign All)</button>
<span id="tool" class="chip"></span></div>
<div class="row"><input id="title" placeholder="Customer name"> <input id="traitA" placeholder="Trait One">
<input id="traitB" placeholder="Trait Two"> <button id="addCard">Add</button>
<select id="mode"><option value="learn">learn</option><option value="playtest">playtest</option>
<option value="custom">custom</option></select>
<input id="iter" type="number" min="0" step="1" value="0" style="width:6rem">
<a href="/api/room" download>Export JSON</a> <input id="import" type="file" accept="application/json">
<button id="reset">Reset</button> <button id="auto">Auto-assign (k-means)</button></div>
<h2>Dashboard</h2><div id="kmeans"></div>
<div class="board"><div class="zones" id="canvas"></div>
<div><h3>Unassigned</h3><div id="unassigned"></div></div></div>
<script src="/app.js"></script>
</body></html>
"""

APP_JS = """'use strict';
let version = -1;
let user = localStorage.getItem('mkUser') || '';
let drag = {id: null, dx: 90, dy: 24};        // the card in flight and where it was grabbed
async function api(path, method, body) {
  const r = await fetch(path, {method: method || 'GET', headers: {'Content-Type': 'application/json'},
                               body: body ? JSON.stringify(body) : undefined});
  if (!r.ok) throw new Error(await r.text());
  return r.json();
}
function $(id) { return document.getElementById(id); }
function el(tag, cls, text) { const e = document.createElement(tag); if (cls) e.className = cls;
  if (text !== undefined) e.textContent = text; return e; }
function btn(text, fn) { const b = el('button', '', text); b.addEventListener('click', fn); return b; }
function initials(n) { return (n || '??').trim().split(/\\s+/).slice(0, 2).map(s => (s[0] || '').toUpperCase()).join('') || '??'; }
function cardEl(card, centroids, pos) {
  const d = el('div', 'card' + (pos ? ' float' : ''));
  d.draggable = true;
  if (pos) { d.style.left = (pos.x * 100).toFixed(4) + '%'; d.style.top = (pos.y * 100).toFixed(4) + '%'; }
  d.appendChild(el('div', '', card.title));
  d.appendChild(el('div', 'traits', (card.traits || []).join(' \\u2022 ')));
  const s = el('select');
  s.appendChild(new Option('Unassigned', ''));
  for (const c of centroids) s.appendChild(new Option(c.name, c.id));
  s.value = card.assignedTo || '';
  s.addEventListener('change', () => api('/api/assign', 'POST', {card: card.id, centroid: s.value || null}));
  d.appendChild(s);
  d.appendChild(btn('Delete', () => { if (confirm('Delete "' + card.title + '"?'))
    api('/api/cards/' + encodeURIComponent(card.id), 'DELETE'); }));
  d.addEventListener('dragstart', ev => {
    ev.dataTransfer.setData('text/plain', card.id);
    const r = d.getBoundingClientRect();
    drag = {id: card.id, dx: ev.clientX - r.left, dy: ev.clientY - r.top};
    d.classList.add('dragging');
  });
  d.addEventListener('dragend', () => d.classList.remove('dragging'));
  return d;
}
function dropTarget(node, onDrop) {
  node.addEventListener('dragover', ev => { ev.preventDefault(); node.classList.add('over'); });
  node.addEventListener('dragleave', () => node.classList.remove('over'));
  node.addEventListener('drop', ev => {
    ev.preventDefault(); node.classList.remove('over');
    const id = ev.dataTransfer.getData('text/plain') || drag.id;
    if (id) onDrop(id, ev);
  });
}
function zoneHead(g, row) {
  const h = el('div', 'head');
  const sw = el('span', 'swatch'); sw.style.background = g.color; h.appendChild(sw);
  const inp = el('input'); inp.value = g.name; inp.size = 12;
  inp.addEventListener('change', () => api('/api/centroids/' + encodeURIComponent(g.id) + '/rename', 'POST',
                                           {name: inp.value.trim() || g.name}));
  h.appendChild(inp);
  const id = encodeURIComponent(g.id);
  h.appendChild(btn(g.locked ? 'Unlock' : 'Lock', () => api('/api/centroids/' + id + '/lock', 'POST')));
  h.appendChild(btn('Remove', () => { if (confirm('Remove centroid "' + g.name + '"?')) api('/api/centroids/' + id, 'DELETE'); }));
  return h;
}
function renderCanvas(st) {
  const wrap = $('canvas');
  wrap.replaceChildren();
  if (!st.centroids.length) {
    wrap.appendChild(el('div', 'traits', 'Add up to 3 centroids. Each appears here as a section where you can drop cards.'));
    return;
  }
  const minH = Math.max(260, 64 + st.cards.length * 120);
  for (const g of st.centroids) {
    const z = el('div', 'zone');
    z.style.borderColor = g.color || '#ccc';
    z.style.minHeight = minH + 'px';
    z.appendChild(zoneHead(g));
    z.appendChild(el('div', 'traits', g.locked ? 'Locked: drops are refused' : 'Drop cards here'));
    dropTarget(z, (id, ev) => {
      if (g.locked) return;
      const r = z.getBoundingClientRect();
      api('/api/drop', 'POST', {card: id, centroid: g.id, x: (ev.clientX - r.left - drag.dx) / r.width,
                                y: (ev.clientY - r.top - drag.dy) / r.height});
    });
    for (const card of st.cards.filter(c => c.assignedTo === g.id))
      z.appendChild(cardEl(card, st.centroids, st.positions[card.id] || {x: 0.05, y: 0.18}));
    wrap.appendChild(z);
  }
}
function renderUnassigned(st) {
  const u = $('unassigned');
  u.replaceChildren();
  const cards = st.cards.filter(c => !c.assignedTo);
  if (!cards.length) u.appendChild(el('div', 'traits', 'No unassigned cards.'));
  for (const card of cards) u.appendChild(cardEl(card, st.centroids, null));
}
function deltaSpan(text) {
  const good = text.indexOf('\\u2191') >= 0 || text.indexOf('+') >= 0 || text.indexOf('\\u00b1') >= 0;
  return el('span', 'delta' + (good ? '' : ' bad'), text);
}
function renderDashboard(d) {
  const root = $('kmeans');
  root.replaceChildren();
  const m = el('div', 'row');
  for (const c of d.chips) m.appendChild(el('span', 'chip', c));
  for (const t of d.deltas) m.appendChild(deltaSpan(t));
  root.appendChild(m);
  for (const r of d.rows) {
    const row = el('div', 'kmrow');
    row.appendChild(el('span', 'chip', r.name));
    const bar = el('div', 'bar'), fill = el('div', 'fill');
    fill.style.width = r.bar_pct + '%'; fill.style.background = r.color || '#888';
    bar.appendChild(fill); row.appendChild(bar);
    const coh = el('span', 'chip', r.cohesion);
    if (r.cohesion_delta) coh.appendChild(deltaSpan(r.cohesion_delta));
    row.appendChild(coh);
    row.appendChild(el('span', 'top', r.top));
    const sg = el('span', 'top', r.suggested);
    if (r.suggestion) sg.appendChild(btn('Use', () => api('/api/centroids/' + encodeURIComponent(r.id) + '/apply_suggestion', 'POST')));
    row.appendChild(sg);
    root.appendChild(row);
  }
}
function renderPresence(st) {
  const p = st.presence || {};
  const s = $('status');
  s.textContent = 'Peers: ' + (p.peers || 0) + ' | ' + (p.link || 'local');
  s.className = 'chip ' + ((p.peers || 0) > 0 ? 'ok' : 'warn');
  const box = $('presence');
  box.replaceChildren();
  const me = user || ('Guest ' + st.room);
  const names = [me].concat((p.names || []).filter(n => n !== me)).slice(0, 6);
  for (const n of names) { const a = el('span', 'avatar', initials(n)); a.title = n; box.appendChild(a); }
}
async function render() {
  const st = await api('/api/state');
  version = st.version;
  $('room').textContent = 'Room: ' + st.room;
  $('version').textContent = 'v' + st.version;
  if (document.activeElement !== $('mode')) $('mode').value = st.meta.mode || 'learn';
  if (document.activeElement !== $('iter')) $('iter').value = st.meta.iteration || 0;
  renderPresence(st);
  renderCanvas(st);
  renderUnassigned(st);
  renderDashboard(st.dashboard);
}
async function follow() {          // live updates: re-render whenever the room or the presence changes
  for (;;) {
    try {
      const c = await api('/api/changes?since=' + version + '&wait=20&user=' + encodeURIComponent(user || ''));
      if (c.version !== version) await render();
    } catch (e) { await new Promise(r => setTimeout(r, 2000)); }
  }
}
dropTarget($('unassigned'), id => api('/api/drop', 'POST', {card: id, centroid: null}));
$('name').value = user;
$('saveName').addEventListener('click', () => { user = $('name').value.trim(); localStorage.setItem('mkUser', user); render(); });
$('copy').addEventListener('click', async () => {
  const r = await api('/api/link?base=' + encodeURIComponent(location.origin + location.pathname));
  if (navigator.clipboard) navigator.clipboard.writeText(r.link); $('tool').textContent = r.link; });
$('populate').addEventListener('click', () => api('/api/populate', 'POST', {}));
$('addCentroid').addEventListener('click', () => api('/api/centroids', 'POST', {name: $('cname').value.trim() || null}));
$('coin').addEventListener('click', async () => { $('tool').textContent = (await api('/api/coin')).result; });
$('d12').addEventListener('click', async () => { $('tool').textContent = 'd12: ' + (await api('/api/d12')).result; });
$('shuffle').addEventListener('click', async () => { $('tool').textContent = (await api('/api/shuffle_names')).names.join(', '); });
$('shuffleUnassigned').addEventListener('click', () => api('/api/shuffle_unassigned', 'POST', {}));
$('restartAll').addEventListener('click', () => { if (confirm('Unassign every card?')) api('/api/restart', 'POST', {}); });
$('addCard').addEventListener('click', () => {
  const t = $('title').value.trim();
  const tr = [$('traitA').value.trim(), $('traitB').value.trim()].filter(Boolean);
  if (t) api('/api/cards', 'POST', {title: t, traits: tr, user: user || null});
});
$('mode').addEventListener('change', () => api('/api/mode', 'POST', {mode: $('mode').value}));
$('iter').addEventListener('change', () => api('/api/iteration', 'POST', {value: $('iter').value}));
$('import').addEventListener('change', async () => {
  const f = $('import').files[0]; if (!f) return;
  try { await api('/api/room/import', 'POST', JSON.parse(await f.text())); } catch (e) { alert('Import failed: ' + e); }
});
$('reset').addEventListener('click', () => { if (confirm('Clear the board?')) api('/api/reset', 'POST', {mode: $('mode').value}); });
$('auto').addEventListener('click', () => api('/api/auto', 'POST', {}));
render().then(follow);
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


PRESENCE_TTL_S = 60.0
PRESENCE_MAX = 1024      # names tracked at once (a client cannot grow the list without bound)


class _Board:
    """The served room plus its change counter: every mutation runs under the lock, bumps
    the version and wakes the long-polls.  Long-polls wait on asyncio events set from
    whichever thread bumped the version, so an open page holds no worker thread.  The names
    the open pages poll with are the presence list (the reference's HELLO / ROSTER names,
    app.mjs:59-67), expiring PRESENCE_TTL_S after a page's last poll."""

    queued = False    # (mutations apply at once)

    def __init__(self, room: Room):
        self.room = room
        self.version = 0
        self.cond = threading.Condition()
        self._init_waiters()

    def _init_waiters(self):
        self._waiters: set = set()          # (loop, asyncio.Event) of the open long-polls
        self._seen: dict[str, float] = {}   # presence: name -> monotonic time of its last poll

    def read(self, fn):
        with self.cond:
            return fn(self.room)

    def mutate(self, fn):
        with self.cond:
            out = fn(self.room)
            self._bump()
            return out

    def _bump(self):
        """(under the lock) a new version: wake every long-poll."""
        self.version += 1
        self.cond.notify_all()
        for loop, ev in list(self._waiters):
            try:
                loop.call_soon_threadsafe(ev.set)
            except RuntimeError:   # (its loop has closed)
                self._waiters.discard((loop, ev))

    def wait_past(self, since: int, timeout: float) -> int:
        with self.cond:
            self.cond.wait_for(lambda: self.version != since, timeout=max(0.0, timeout))
            return self.version

    async def wait_past_async(self, since: int, timeout: float) -> int:
        ev = asyncio.Event()
        w = (asyncio.get_running_loop(), ev)
        with self.cond:
            if self.version != since:
                return self.version
            self._waiters.add(w)
        try:
            await asyncio.wait_for(ev.wait(), max(0.0, timeout))
        except asyncio.TimeoutError:
            pass
        finally:
            with self.cond:
                self._waiters.discard(w)
        with self.cond:
            return self.version

    def seen(self, name: str):
        """A page polled as ``name``: a new name (or one back after expiring) is a change."""
        name = name.strip()[:64]
        if not name:
            return
        now = time.monotonic()
        with self.cond:
            fresh = name not in self._seen or now - self._seen[name] > PRESENCE_TTL_S
            if fresh and len(self._seen) >= PRESENCE_MAX:   # (expired names go first; then refuse)
                self._seen = {n: t for n, t in self._seen.items() if now - t <= PRESENCE_TTL_S}
                if len(self._seen) >= PRESENCE_MAX:
                    return
            self._seen[name] = now
            if fresh:
                self._bump()

    def presence_names(self) -> list[str]:
        now = time.monotonic()
        with self.cond:
            return sorted(n for n, t in self._seen.items() if now - t <= PRESENCE_TTL_S)


class _QueuedRoom:
    """What the route handlers see in session mode: the replica's room for reads, and every
    replicated Room operation (parallel/replica.py OPS) queued for the next round instead of
    applied (the reference broadcasts each transaction, app.mjs:121; here every member
    applies the same ops in the same order)."""

    def __init__(self, replica):
        self._rep = replica

    def __getattr__(self, name):
        from .parallel.replica import OPS

        if name in OPS:
            op = getattr(self._rep, name)

            def queue(*args, **kw):
                kw.pop("created_by", None)     # (the member's own name is the author)
                if name == "import_json":
                    kw.pop("compat", None)
                out = op(*args, **kw)
                return out if out is not None else True
            return queue
        return getattr(self._rep.room, name)


class _ReplicaBoard(_Board):
    """The served room as one member of a live replicated session
    (:class:`~mikmeans.parallel.elastic.ElasticRoomReplica`): edits are queued and applied by
    every member at the next round; a background thread runs the rounds and bumps the version
    whenever one applied an op or changed the roster, so every browser on every member's
    server re-renders."""

    queued = True

    def __init__(self, replica, interval: float = 0.2):
        self.replica = replica
        self.version = 0
        self.cond = threading.Condition()
        self._init_waiters()
        self.interval = float(interval)
        self.error = None
        self._stop = threading.Event()
        self._thread = threading.Thread(target=self._rounds, name="mikmeans-session", daemon=True)
        self._thread.start()

    @property
    def room(self):
        return self.replica.room

    def read(self, fn):
        with self.cond:
            return fn(self.replica.room)

    def mutate(self, fn):
        with self.cond:
            return fn(_QueuedRoom(self.replica))

    def _rounds(self):
        """The session's rounds.  Only the round's local steps hold the board's lock -- taking
        the queued ops, then applying the gathered ones; the collectives (the all-gather, and an
        epoch change's group formation and full-state broadcast) run without it, so a slow or
        dead peer stalls this thread, not the handlers."""
        rep = self.replica
        roster = None
        while not self._stop.is_set() and not rep.left:
            try:
                with self.cond:
                    msg = rep.round_begin()
                parts = rep.round_exchange(msg)
                with self.cond:      # (the ops change the room the handlers read)
                    applied, change = rep.round_apply(parts)
                    if applied or rep.roster != roster or change is not None:
                        roster = list(rep.roster)
                        self._bump()
                if change is not None and rep.round_transition(change):
                    with self.cond:
                        self._bump()
            except Exception as e:  # noqa: BLE001 -- a dead session: keep serving the last state
                self.error = f"{type(e).__name__}: {e}"
                with self.cond:
                    self._bump()
                return
            self._stop.wait(self.interval)

    def close(self, leave: bool = True):
        if leave and not self.replica.left:
            with self.cond:
                self.replica.leave()
        deadline = 50
        while leave and not self.replica.left and self._thread.is_alive() and deadline:
            self._stop.wait(self.interval)
            deadline -= 1
        self._stop.set()
        self._thread.join(timeout=5)


class _BodyCap:
    """ASGI middleware: 413 for a request whose body passes ``limit`` bytes, by its declared
    Content-Length or -- chunked transfers declare none -- by the bytes actually received:
    past the cap the body the handler reads ends there, and whatever the handler answers to
    that truncated body is replaced by the 413."""

    def __init__(self, app, limit: int):
        self.app, self.limit = app, int(limit)

    async def __call__(self, scope, receive, send):
        if scope["type"] != "http":
            return await self.app(scope, receive, send)
        limit = self.limit
        for k, v in scope.get("headers", []):
            if k == b"content-length":
                try:
                    declared = int(v)
                except ValueError:
                    declared = 0
                if declared > limit:
                    resp = JSONResponse({"detail": f"request body over {limit} bytes"}, status_code=413,
                                        headers=SECURITY_HEADERS)
                    return await resp(scope, receive, send)
        got, over, replaced = 0, False, False

        async def capped():
            # past the cap the body ends here (the handler then fails on what it got) and the
            # answer is replaced by the 413 below
            nonlocal got, over
            if over:
                return {"type": "http.request", "body": b"", "more_body": False}
            msg = await receive()
            if msg["type"] == "http.request":
                got += len(msg.get("body", b""))
                if got > limit:
                    over = True
                    return {"type": "http.request", "body": b"", "more_body": False}
            return msg

        async def send_checked(msg):
            nonlocal replaced
            if over and not replaced and msg["type"] == "http.response.start":
                replaced = True
                resp = JSONResponse({"detail": f"request body over {limit} bytes"}, status_code=413,
                                    headers=SECURITY_HEADERS)
                return await resp(scope, capped, send)
            if replaced:
                return None       # (the handler's own answer to the truncated body)
            return await send(msg)
        return await self.app(scope, capped, send_checked)


def _npy_view(buf: memoryview) -> np.ndarray:
    """A ``.npy`` payload as an array viewing ``buf`` (no copy): the header parsed by numpy's
    own reader, object dtypes refused (nothing is unpickled)."""
    import io

    f = io.BytesIO(bytes(buf[:65536]))   # (the header: at most a few KiB)
    major, _ = np.lib.format.read_magic(f)
    if major == 1:
        shape, fortran, dtype = np.lib.format.read_array_header_1_0(f)
    else:
        shape, fortran, dtype = np.lib.format.read_array_header_2_0(f)
    if dtype.hasobject:
        raise ValueError("object arrays are not accepted")
    count = int(np.prod(shape)) if shape else 1
    arr = np.frombuffer(buf, dtype=dtype, count=count, offset=f.tell())
    return arr.reshape(shape[::-1]).T if fortran else arr.reshape(shape)


def create_app(room: Room | None = None, model=None, *, device=None, max_body_bytes: int = MAX_BODY_BYTES,
               max_rows: int = MAX_ROWS, max_transform_values: int = MAX_TRANSFORM_VALUES, replica=None,
               session_interval: float = 0.2):
    """The FastAPI app serving ``room`` (a new one when None) and, when given, a fitted
    ``model`` (:class:`~mikmeans.KMeans` / :class:`~mikmeans.MiniBatchKMeans`).  ``replica``
    (an :class:`~mikmeans.parallel.elastic.ElasticRoomReplica`): serve that member's room of a
    live session instead -- edits are queued (HTTP 202) and appear on every member's board
    after the next round."""
    app = FastAPI(title="mikmeans", docs_url=None, redoc_url=None, openapi_url=None)
    if replica is not None:
        board = _ReplicaBoard(replica, session_interval)
    else:
        board = _Board(room if room is not None else Room(seed=0))
    model_lock = threading.Lock()   # (one batch at a time on the device: the serving pack is shared)

    @app.middleware("http")
    async def _headers(request, call_next):
        resp = await call_next(request)
        # session mode: a room edit is queued for the next round, not applied yet
        if (board.queued and resp.status_code == 200 and request.method in ("POST", "DELETE")
                and request.url.path.startswith("/api/") and request.url.path not in _READ_POSTS):
            resp.status_code = 202
        for k, v in SECURITY_HEADERS.items():
            resp.headers[k] = v
        return resp

    app.add_middleware(_BodyCap, limit=max_body_bytes)

    @app.get("/", response_class=HTMLResponse)
    def page():
        return HTMLResponse(PAGE)

    @app.get("/app.js")
    def app_js():
        return Response(APP_JS, media_type="text/javascript")

    # ------------------------------------------------------------------- room state
    @app.get("/api/room")
    def export_room():
        txt, name = board.read(lambda r: (r.export_json(), r.export_filename))
        return Response(txt, media_type="application/json",
                        headers={"Content-Disposition": f'attachment; filename="{name}"'})

    @app.get("/api/state")
    def room_state():
        def snap(r):
            pos = {k[4:]: v for k, v in r.meta.to_dict().items() if k.startswith("pos:")}
            out = {"room": r.room, "version": board.version, "cards": r.cards, "centroids": r.centroids,
                   "meta": {"mode": r.meta.get("mode"), "iteration": r.meta.get("iteration")},
                   "positions": pos, "dashboard": r.dashboard()}
            names = board.presence_names()
            if board.queued:    # the session's presence (the reference's roster, app.mjs:66-67, :94-95)
                rep = board.replica
                out["session"] = {"round": rep.round, "epoch": rep.epoch, "peers": rep.peers,
                                  "roster": rep.roster, "error": board.error}
                out["presence"] = {"peers": rep.peers, "names": sorted(set(names) | set(rep.roster)),
                                   "link": f"round {rep.round}" if board.error is None else "session lost"}
            else:   # (the browsers on this board: the pages polling it, by their names)
                out["presence"] = {"peers": max(0, len(names) - 1), "names": names, "link": "local"}
            return _jsonable(out)
        return board.read(snap)

    @app.get("/api/changes")
    async def changes(since: int = -1, wait: float = 0.0, user: str = ""):
        """Long-poll: the current version as soon as it differs from ``since`` (an async wait:
        open pages hold no worker thread).  ``user``: the polling page's name (presence)."""
        board.seen(user)
        v = await board.wait_past_async(int(since), min(float(wait), LONG_POLL_S))
        return {"version": v, "changed": v != since}

    @app.post("/api/room/import")
    def import_room(body: dict = Body(...)):
        import json

        try:                     # (validated before it reaches the room -- or a session's queue)
            Room.from_json(json.dumps(body))
        except (ValueError, TypeError, KeyError, AttributeError) as e:
            raise HTTPException(400, f"not a room export: {e}") from None

        def imp(r):
            r.import_json(json.dumps(body))
            return {"cards": len(r.cards), "centroids": len(r.centroids)}
        try:
            return board.mutate(imp)
        except (ValueError, TypeError, KeyError, AttributeError) as e:
            raise HTTPException(400, f"not a room export: {e}") from None

    # ------------------------------------------------------------------- cards
    @app.post("/api/cards")
    def add_card(body: dict = Body(...)):
        title = str(body.get("title", "")).strip()
        if not title:
            raise HTTPException(400, "title required")
        traits = body.get("traits", [])
        if not isinstance(traits, list) or not all(isinstance(t, str) for t in traits):
            raise HTTPException(400, "traits: a list of strings")
        user = body.get("user") or None
        return board.mutate(lambda r: r.add_card(title, traits, created_by=str(user) if user else None))

    @app.delete("/api/cards/{card_id}")
    def delete_card(card_id: str):
        def rm(r):
            if r._card_index(card_id) < 0:
                return None
            r.delete_card(card_id)
            return {"cards": len(r.cards)}
        out = board.mutate(rm)
        if out is None:
            raise HTTPException(404, "no such card")
        return out

    @app.post("/api/assign")
    def assign(body: dict = Body(...)):
        ok = board.mutate(lambda r: r.update_card_assign(body.get("card"), body.get("centroid") or None))
        if not ok:
            raise HTTPException(409, "not assigned (unknown card or locked centroid)")
        return {"ok": True}

    @app.post("/api/drop")
    def drop(body: dict = Body(...)):
        """Drag-and-drop: a card dropped on a centroid zone at the normalised position (x, y)
        (clamped, refused on a locked centroid, the assignment and ``pos:<id>`` in one
        transaction, app.mjs:356-372), or on Unassigned (``centroid`` null: unassigned and its
        ``pos:`` deleted, app.mjs:421-433)."""
        import math

        card, cid = body.get("card"), body.get("centroid") or None
        if not isinstance(card, str):
            raise HTTPException(400, "card: a card id")
        if cid is None:
            ok = board.mutate(lambda r: r.update_card_assign(card, None))
        else:
            try:
                x, y = float(body.get("x", 0.05)), float(body.get("y", 0.18))
            except (TypeError, ValueError):
                raise HTTPException(400, "x, y: numbers") from None
            if not (math.isfinite(x) and math.isfinite(y)):
                raise HTTPException(400, "x, y: finite numbers")
            ok = board.mutate(lambda r: r.drop_card(card, str(cid), x, y))
        if not ok:
            raise HTTPException(409, "not dropped (unknown card or centroid, or a locked centroid)")
        return {"ok": True}

    @app.post("/api/populate")
    def populate(body: dict = Body(default={})):
        return board.mutate(lambda r: (r.populate_test_data(), {"cards": len(r.cards)})[1])

    @app.post("/api/shuffle_unassigned")
    def shuffle_unassigned(body: dict = Body(default={})):
        return board.mutate(lambda r: (r.shuffle_unassigned(), {"cards": [c["id"] for c in r.cards]})[1])

    @app.post("/api/restart")
    def restart(body: dict = Body(default={})):
        return board.mutate(lambda r: (r.restart_all(), {"ok": True})[1])

    @app.post("/api/reset")
    def reset(body: dict = Body(default={})):
        mode = body.get("mode")
        if mode is not None and not isinstance(mode, str):
            raise HTTPException(400, "mode: a string")
        return board.mutate(lambda r: (r.hard_reset(mode), {"cards": len(r.cards), "centroids": 0})[1])

    # ------------------------------------------------------------------- centroids
    @app.post("/api/centroids")
    def add_centroid(body: dict = Body(default={})):
        c = board.mutate(lambda r: r.add_centroid(body.get("name") or None))
        if c is None:
            raise HTTPException(409, "at most %d centroids" % board.room.max_centroids)
        return c

    def _known(r, cid):
        if r.centroid(cid) is None:
            raise HTTPException(404, "no such centroid")

    @app.post("/api/centroids/{cid}/rename")
    def rename_centroid(cid: str, body: dict = Body(...)):
        name = body.get("name")
        if not isinstance(name, str):
            raise HTTPException(400, "name: a string")

        def ren(r):
            _known(r, cid)
            r.rename_centroid(cid, name)
            return r.centroid(cid)
        return board.mutate(ren)

    @app.post("/api/centroids/{cid}/apply_suggestion")
    def apply_suggestion(cid: str):
        """The dashboard's "Suggested:" name for this centroid (app.mjs:571-573)."""
        def app_(r):
            _known(r, cid)
            sug = next((row["suggestion"] for row in r.dashboard()["rows"] if row["id"] == cid), None)
            if not sug:
                raise HTTPException(409, "no suggestion for this centroid")
            r.apply_suggested_name(cid, sug)
            return r.centroid(cid)
        return board.mutate(app_)

    @app.post("/api/centroids/{cid}/lock")
    def toggle_lock(cid: str):
        def tog(r):
            _known(r, cid)
            r.toggle_lock(cid)
            return {"locked": bool(r.centroid(cid).get("locked"))}
        return board.mutate(tog)

    @app.delete("/api/centroids/{cid}")
    def remove_centroid(cid: str):
        return board.mutate(lambda r: (r.remove_centroid(cid), {"centroids": len(r.centroids)})[1])

    # ------------------------------------------------------------------- meta / tools
    @app.post("/api/mode")
    def set_mode(body: dict = Body(...)):
        mode = body.get("mode")
        if not isinstance(mode, str):
            raise HTTPException(400, "mode: a string")
        return board.mutate(lambda r: (r.set_mode(mode), {"mode": r.meta.get("mode")})[1])

    @app.post("/api/iteration")
    def set_iteration(body: dict = Body(...)):
        return board.mutate(lambda r: (r.set_iteration(body.get("value")), {"iteration": r.meta.get("iteration")})[1])

    @app.get("/api/coin")
    def coin():
        return {"result": board.read(lambda r: r.coin())}

    @app.get("/api/d12")
    def d12():
        return {"result": board.read(lambda r: r.d12())}

    @app.get("/api/shuffle_names")
    def shuffle_names():
        return {"names": board.read(lambda r: r.shuffled_titles())}

    @app.get("/api/link")
    def link(base: str = ""):
        return {"link": board.read(lambda r: r.share_link(base))}

    @app.post("/api/auto")
    def auto(body: dict = Body(default={})):
        return _jsonable(board.mutate(lambda r: r.auto_assign(seed=int(body.get("seed", 0)))))

    @app.get("/api/dashboard")
    def dashboard():
        return board.read(lambda r: _jsonable(r.dashboard()))

    # ------------------------------------------------------------------- model serving
    def _model():
        if model is None:
            raise HTTPException(404, "no model loaded (mikmeans serve --model DIR)")
        return model

    def _centroid_text() -> str:
        from .utils.jsjson import centroids_to_json

        return centroids_to_json(_model().cluster_centers_)

    @app.get("/api/model")
    def model_info():
        C = _model().cluster_centers_
        # the centroids as the flat-float array of centroids.json, spliced in verbatim
        body = (f'{{"n_clusters":{int(C.shape[0])},"n_features":{int(C.shape[1])},'
                f'"centroids":{_centroid_text()}}}')
        return Response(body, media_type="application/json")

    @app.get("/api/model/centroids.json")
    def model_centroids():
        return Response(_centroid_text(), media_type="application/json")

    def _check_rows(n: int):
        if n > max_rows:
            raise HTTPException(413, f"at most {max_rows} rows per batch")

    def _points(body: dict) -> torch.Tensor:
        pts = body.get("points")
        if not isinstance(pts, list) or not pts:
            raise HTTPException(400, "points: a non-empty list of rows")
        _check_rows(len(pts))
        try:
            arr = np.asarray(pts, dtype=np.float32)
        except (ValueError, TypeError) as e:
            raise HTTPException(400, f"points: a rectangular array of numbers ({e})") from None
        X = torch.as_tensor(arr)
        m = _model()
        if X.dim() != 2 or X.shape[1] != m.cluster_centers_.shape[1]:
            raise HTTPException(400, f"points must be [n, {m.cluster_centers_.shape[1]}]")
        return X.to(m.cluster_centers_.device)

    @app.post("/api/predict")
    def predict(body: dict = Body(...)):
        m = _model()
        X = _points(body)
        with model_lock:
            labels, mind, _ = m._assign_rows(X, bool(body.get("distances", False)))
        out = {"labels": labels.cpu().tolist()}
        if mind is not None:
            out["distances"] = mind.cpu().tolist()
        return out

    @app.post("/api/predict.npy")
    async def predict_npy(request: Request):
        """Binary serving: the body is a ``.npy`` array [n, D] (``numpy.save``; loaded with
        ``allow_pickle=False``), the answer the int32 labels as ``.npy`` -- no JSON
        parsing of large batches.  The body is read up to ``max_body_bytes`` (413 beyond,
        whatever the request declared)."""
        import io

        m = _model()
        try:
            declared = int(request.headers.get("content-length", "-1"))
        except ValueError:
            declared = -1
        if 0 <= declared <= max_body_bytes:
            # one buffer of the declared size, filled in place (joining ~2000 64-KiB chunks of
            # a 134 MB batch cost ~90 ms, np.load's copy ~50 ms more)
            body, size = bytearray(declared), 0
            async for part in request.stream():
                if size + len(part) > declared:
                    raise HTTPException(400, "request body longer than its Content-Length")
                body[size:size + len(part)] = part
                size += len(part)
            body = memoryview(body)[:size]
        else:
            chunks, size = [], 0
            async for part in request.stream():
                size += len(part)
                if size > max_body_bytes:
                    raise HTTPException(413, f"request body over {max_body_bytes} bytes")
                chunks.append(part)
            body = memoryview(bytearray(b"".join(chunks)))   # (writable: the rows become a tensor)
        try:
            arr = _npy_view(body)
        except Exception as e:  # noqa: BLE001 -- any malformed payload is the client's error
            raise HTTPException(400, f"body must be a .npy array: {e}") from None
        if arr.ndim != 2 or arr.shape[1] != m.cluster_centers_.shape[1]:
            raise HTTPException(400, f"array must be [n, {m.cluster_centers_.shape[1]}]")
        _check_rows(arr.shape[0])
        try:
            X = torch.as_tensor(np.ascontiguousarray(arr, dtype=np.float32)).to(m.cluster_centers_.device)
        except (ValueError, TypeError) as e:
            raise HTTPException(400, f"array must hold numbers ({e})") from None
        with model_lock:
            labels, _, _ = m._assign_rows(X, False)
        buf = io.BytesIO()
        np.save(buf, labels.cpu().numpy().astype(np.int32), allow_pickle=False)
        return Response(buf.getvalue(), media_type="application/octet-stream")

    @app.post("/api/transform")
    def transform(body: dict = Body(...)):
        m = _model()
        X = _points(body)
        if X.shape[0] * int(m.cluster_centers_.shape[0]) > max_transform_values:
            raise HTTPException(413, f"at most {max_transform_values} distances per answer")
        with model_lock:
            d = m.transform(X)
        return {"distances": d.cpu().tolist()}

    app.state.board = board
    if board.queued:
        app.router.on_shutdown.append(board.close)
    return app


# POST routes that change nothing in the room (model serving)
_READ_POSTS = ("/api/predict", "/api/predict.npy", "/api/transform")


def serve(room_path=None, model_path=None, host: str = "127.0.0.1", port: int = 8000, device=None,
          session: dict | None = None):
    """Run the app with uvicorn (blocking).  ``session``: serve a member of a live room
    session -- ``{"store_host", "store_port", "found": ROOM or None (join), "member", "user"}``
    (the founder hosts the rendezvous store; ``room_path`` seeds a founded room)."""
    import uvicorn

    room = None
    text = None
    if room_path:
        with open(room_path) as f:
            text = f.read()
        room = Room.from_json(text)
    model = None
    if model_path:
        from .api import KMeans

        model = KMeans.load(model_path, device=device)
    replica = None
    if session is not None:
        replica = open_session(text, **session)
    uvicorn.run(create_app(room, model, replica=replica), host=host, port=port, log_level="warning")


def open_session(state_json=None, *, store_host: str = "127.0.0.1", store_port: int, found=None,
                 member: str | None = None, user: str | None = None, timeout_s: float = 120.0, seed: int = 0):
    """Found (``found`` = room code, "" for a new one) or join a live room session over a
    TCPStore at ``store_host:store_port`` and return this member's ElasticRoomReplica."""
    import datetime
    import os
    import socket

    import torch.distributed as dist

    from .parallel.elastic import ElasticRoomReplica

    store = dist.TCPStore(store_host, int(store_port), is_master=found is not None, wait_for_workers=False,
                          timeout=datetime.timedelta(seconds=timeout_s))
    member = member or f"{socket.gethostname()}-{os.getpid()}-serve"
    kw = dict(user=user, seed=seed, timeout_s=timeout_s)
    if found is not None:
        rep = ElasticRoomReplica.found(store, member, found or None, state_json=state_json, **kw)
    else:
        rep = ElasticRoomReplica.join(store, member, **kw)
    rep._store_ref = store          # (the master store lives as long as the replica)
    return rep
