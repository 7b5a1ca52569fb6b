"""Trait-card "room": the reference's collaborative k-means board as a headless model.

The reference (``schusto/k-means-demo``) is a classroom game where people drag
"flavor cards" onto <=3 named centroids, with a live dashboard.  This module
re-creates its data model, mutations, seed data, metrics, dashboard text and
byte-exact export/import without a browser, and bridges it to the numeric engine
(:meth:`Room.auto_assign` runs real k-means on multi-hot trait vectors).

Parity map (reference file:line -> here):

* state ``cards`` / ``centroids`` / ``meta`` Yjs doc (app.mjs:30-33)      -> :class:`Room` (+ :class:`OrderedMeta`)
* nextColor / addCentroid / removeCentroid (app.mjs:125-142)              -> :meth:`next_color`, :meth:`add_centroid`, :meth:`remove_centroid`
* addCard / updateCardAssign / setCardPos / getCardPos (app.mjs:143-158)  -> same names, snake_case
* shuffleUnassigned / restartAll / deleteCard (app.mjs:159-185)
* JESSICA / ensureJessicaOnce / dedupeSeeds / populateTestData / hardReset (app.mjs:188-237)
* drop handler with lock + clamping (app.mjs:356-372)                     -> :meth:`drop_card`
* rename / lock toggle / applySuggestedName (app.mjs:325-346, :571-573)
* mode / iteration + prevSnapshot hook (app.mjs:285-288, :498-508)        -> :meth:`set_mode`, :meth:`set_iteration`
* snapshotMetrics / renderKMeans text (app.mjs:481-570)                   -> :meth:`snapshot_metrics`, :meth:`dashboard`
* Export / Import (app.mjs:263-282)                                       -> :meth:`export_json`, :meth:`import_json`
* room code (app.mjs:15-19)                                               -> :func:`room_code`

Known reference defects are NOT replicated by default:
the lock is enforced on every assignment path (#3), import keeps fields that are
absent from the file (#9) -- pass ``compat=True`` to :meth:`import_json` for the
reference's exact behaviour -- and duplicate ids never arise from our single
writer (#5).
"""
from __future__ import annotations

import random as _random
import time as _time

from ..data.cards import JESSICA, TEST_ITEMS
from ..utils import jsjson, metrics as mm, traits as tr

COLORS = ["#6EE7B7", "#93C5FD", "#FBCFE8", "#FDE68A", "#C7D2FE", "#FCA5A5"]
ROOM_ALPHABET = "ABCDEFGHJKLMNPQRSTUVWXYZ23456789"
MAX_CENTROIDS = 3
_DELETED = object()


def room_code(rng=None) -> str:
    rng = rng or _random.Random()
    return "".join(ROOM_ALPHABET[int(rng.random() * len(ROOM_ALPHABET))] for _ in range(4))


def js_base36_fraction(x: float, n: int = 5) -> str:
    """``Math.random().toString(36).slice(2, 2+n)`` for x in [0, 1)."""
    digits = "0123456789abcdefghijklmnopqrstuvwxyz"
    out = []
    for _ in range(n):
        x *= 36
        d = int(x)
        out.append(digits[d])
        x -= d
        if x == 0:
            break
    return "".join(out)


class OrderedMeta:
    """Y.Map-like key/value store: a deleted key keeps its slot, so re-setting it
    later does not move it to the end (Yjs keeps the map entry and flags it
    deleted); iteration skips deleted keys."""

    def __init__(self, items=None):
        self._d: dict = {}
        for k, v in (items or {}).items():
            self._d[k] = v

    def get(self, k, default=None):
        v = self._d.get(k, _DELETED)
        return default if v is _DELETED else v

    def set(self, k, v):
        self._d[k] = v

    def delete(self, k):
        if k in self._d:
            self._d[k] = _DELETED

    def __contains__(self, k):
        return self._d.get(k, _DELETED) is not _DELETED

    def keys(self):
        return [k for k, v in self._d.items() if v is not _DELETED]

    def items(self):
        return [(k, v) for k, v in self._d.items() if v is not _DELETED]

    def to_dict(self) -> dict:
        return dict(self.items())


def _js_strict_ne(a, b) -> bool:
    """JavaScript ``a !== b`` for JSON values: objects/arrays compare by identity, a
    boolean never equals a number, 3 === 3.0."""
    if isinstance(a, (dict, list)) or isinstance(b, (dict, list)):
        return a is not b
    if isinstance(a, bool) != isinstance(b, bool):
        return True
    return a != b


class Room:
    def __init__(self, room_id: str | None = None, *, user: str | None = None, seed: int | None = None,
                 clock=None, max_centroids: int = MAX_CENTROIDS, seed_jessica: bool = True):
        self.rng = _random.Random(seed)
        self.clock = clock or (lambda: int(_time.time() * 1000))
        self.room = room_id or room_code(self.rng)
        self.user = user or f"Guest {self.room}"
        self.max_centroids = max_centroids
        self.cards: list[dict] = []
        self.centroids: list[dict] = []
        self.meta = OrderedMeta()
        self._last_iter = None
        # the #mode <select>'s value: syncMeta (app.mjs:299) copies a truthy meta mode into
        # it; hardReset reads it back (app.mjs:231)
        self._mode_select = "learn"
        self.log: list[tuple] = []  # applied operations (for replication)
        if seed_jessica:
            self.ensure_jessica_once()
        self._last_iter = self.meta.get("iteration")

    # ------------------------------------------------------------ id helpers
    def _new_id(self, prefix: str) -> str:
        return f"{prefix}:{self.clock()}-{js_base36_fraction(self.rng.random())}"

    def _card_index(self, card_id):
        for i, c in enumerate(self.cards):
            if c.get("id") == card_id:
                return i
        return -1

    def _centroid(self, cid):
        for c in self.centroids:
            if c.get("id") == cid:
                return c
        return None

    def centroid(self, cid) -> dict | None:
        """The centroid record ``cid`` (None when absent)."""
        return self._centroid(cid)

    # -------------------------------------------------------------- centroids
    def next_color(self) -> str:
        used = {c.get("color") for c in self.centroids}
        for col in COLORS:
            if col not in used:
                return col
        return COLORS[int(self.rng.random() * len(COLORS))]

    def add_centroid(self, name: str | None = None, *, cid: str | None = None):
        """Add a centroid (at most ``max_centroids``); returns its record or None when full."""
        if len(self.centroids) >= self.max_centroids:
            return None
        c = {"id": cid or self._new_id("c"), "name": name or f"Centroid {len(self.centroids) + 1}",
             "color": self.next_color(), "locked": False}
        self.centroids.append(c)
        self.log.append(("add_centroid", c["name"], c["id"]))
        return c

    def remove_centroid(self, cid: str):
        for i, card in enumerate(self.cards):
            if card.get("assignedTo") == cid:
                self.cards[i] = {**card, "assignedTo": None}
                self.meta.delete(f"pos:{card['id']}")
        self.centroids = [c for c in self.centroids if c.get("id") != cid]
        self.log.append(("remove_centroid", cid))

    def _replace_centroid(self, cid, **upd):
        for i, c in enumerate(self.centroids):
            if c.get("id") == cid:
                self.centroids[i] = {**c, **upd}
                return self.centroids[i]
        return None

    def rename_centroid(self, cid: str, name: str):
        c = self._centroid(cid)
        if c is not None:
            self._replace_centroid(cid, name=tr.js_trim(name) or c["name"])
            self.log.append(("rename_centroid", cid, name))

    def toggle_lock(self, cid: str):
        c = self._centroid(cid)
        if c is not None:
            self._replace_centroid(cid, locked=not c.get("locked", False))
            self.log.append(("toggle_lock", cid))

    def apply_suggested_name(self, cid: str, name: str):
        if self._centroid(cid) is not None:
            self._replace_centroid(cid, name=name)
            self.log.append(("apply_suggested_name", cid, name))

    # ------------------------------------------------------------------ cards
    def add_card(self, title: str, traits, *, card_id: str | None = None, assigned_to=None,
                 created_by: str | None = None):
        card = {"id": card_id or self._new_id("card"), "title": title, "traits": list(traits),
                "assignedTo": assigned_to, "createdBy": created_by or self.user or "anon"}
        self.cards.append(card)
        self.log.append(("add_card", card))
        return card

    def update_card_assign(self, card_id: str, cid, *, respect_lock: bool = True) -> bool:
        """Assign a card (``cid=None`` unassigns).  Locked centroids refuse new cards
        on every path (the reference enforced it on drop only: defect #3)."""
        i = self._card_index(card_id)
        if i < 0:
            return False
        if cid is not None:
            c = self._centroid(cid)
            if c is None:
                return False
            if respect_lock and c.get("locked") and self.cards[i].get("assignedTo") != cid:
                return False
        self.cards[i] = {**self.cards[i], "assignedTo": cid}
        if not cid:
            self.meta.delete(f"pos:{card_id}")
        self.log.append(("update_card_assign", card_id, cid))
        return True

    def drop_card(self, card_id: str, cid: str, x: float, y: float) -> bool:
        """Drop onto a centroid zone: refused when locked; position clamped to
        x in [0.02, 0.92], y in [0.10, 0.92] (app.mjs:358-371)."""
        c = self._centroid(cid)
        if c is None or c.get("locked"):
            return False
        x = min(0.92, max(0.02, float(x)))
        y = min(0.92, max(0.10, float(y)))
        if not self.update_card_assign(card_id, cid):
            return False
        self.meta.set(f"pos:{card_id}", {"x": x, "y": y})
        return True

    def set_card_pos(self, card_id: str, x: float, y: float):
        self.meta.set(f"pos:{card_id}", {"x": x, "y": y})

    def get_card_pos(self, card_id: str):
        return self.meta.get(f"pos:{card_id}")

    def shuffle_unassigned(self):
        A = [c for c in self.cards if c.get("assignedTo")]
        U = [c for c in self.cards if not c.get("assignedTo")]
        for i in range(len(U) - 1, 0, -1):
            j = int(self.rng.random() * (i + 1))
            U[i], U[j] = U[j], U[i]
        self.cards = A + U
        self.log.append(("shuffle_unassigned",))

    # ------------------------------------------------- top-control utilities
    def share_link(self, base_url: str = "") -> str:
        """The reference's "Copy link" (app.mjs:239-242) copies ``location.href``, i.e.
        the page URL carrying ``?room=<code>`` (written by app.mjs:17)."""
        sep = "&" if "?" in base_url else "?"
        return f"{base_url}{sep}room={self.room}"

    def coin(self) -> str:
        """``Math.random() < 0.5 ? "Heads" : "Tails"`` (app.mjs:254)."""
        return "Heads" if self.rng.random() < 0.5 else "Tails"

    def d12(self) -> int:
        """``1 + floor(Math.random() * 12)`` (app.mjs:255)."""
        return 1 + int(self.rng.random() * 12)

    def shuffled_titles(self) -> list[str]:
        """The "Shuffle names" suggestion (app.mjs:256-260): a Fisher-Yates permutation of
        every card title, from the last index down; the board itself is not changed."""
        n = [c["title"] for c in self.cards]
        for i in range(len(n) - 1, 0, -1):
            j = int(self.rng.random() * (i + 1))
            n[i], n[j] = n[j], n[i]
        return n

    def restart_all(self):
        self.cards = [{**c, "assignedTo": None} if c.get("assignedTo") else c for c in self.cards]
        for k in self.meta.keys():
            if str(k).startswith("pos:"):
                self.meta.delete(k)
        self.log.append(("restart_all",))

    def delete_card(self, card_id: str):
        self.cards = [c for c in self.cards if c.get("id") != card_id]
        self.meta.delete(f"pos:{card_id}")
        self.log.append(("delete_card", card_id))

    # ------------------------------------------------------------------ seeds
    def ensure_jessica_once(self):
        seeded = self.meta.get("seededJessica")
        has = any(c.get("id") == JESSICA["id"] for c in self.cards)
        if not seeded and not has:
            self.add_card(JESSICA["title"], JESSICA["traits"], card_id=JESSICA["id"], created_by="seed")
            self.meta.set("seededJessica", True)

    def dedupe_seeds(self):
        seen, keep = set(), []
        for c in self.cards:
            cid = c.get("id")
            if isinstance(cid, str) and cid.startswith("seed:"):
                if cid in seen:
                    continue
                seen.add(cid)
            keep.append(c)
        self.cards = keep

    def populate_test_data(self):
        existing = {c.get("id") for c in self.cards}
        for cid, title, a, b in TEST_ITEMS:
            if cid not in existing:
                self.cards.append({"id": cid, "title": title, "traits": [a, b], "assignedTo": None,
                                   "createdBy": "seed"})
        self.dedupe_seeds()
        self.log.append(("populate_test_data",))

    def hard_reset(self, mode: str | None = None):
        """Clear the board, re-seed Jessica (app.mjs:225-237).  The mode written is the
        current mode selector's value (``mode`` overrides it), and the iteration hook then
        runs as the reference's observer does after the transaction (app.mjs:498-505):
        resetting from a nonzero iteration snapshots the fresh board as ``prevSnapshot``."""
        mode = self._mode_select if mode is None else mode
        for k in self.meta.keys():
            if str(k).startswith("pos:"):
                self.meta.delete(k)
        self.cards = []
        self.centroids = []
        self.meta.set("iteration", 0)
        self._set_meta_mode(mode or "learn")
        self.meta.set("seededJessica", False)
        self.cards.append({**JESSICA, "traits": list(JESSICA["traits"]), "assignedTo": None, "createdBy": "seed"})
        self.meta.set("seededJessica", True)
        self.meta.delete("prevSnapshot")
        self._iteration_hook()
        self.log.append(("hard_reset", mode))

    # ------------------------------------------------------------- meta / iter
    MODES = ("learn", "playtest", "custom")   # the <select>'s options (index.html:125-127)

    def _set_meta_mode(self, mode):
        self.meta.set("mode", mode)
        if mode:  # syncMeta: a truthy mode is copied into the select ("" if no option matches)
            self._mode_select = mode if mode in self.MODES else ""

    def _iteration_hook(self):
        """The meta observer (app.mjs:498-505), run after any transaction that set
        ``iteration``: when it differs from the last seen value (JS ``!==``; arrays and
        objects never compare equal), the current metrics become ``prevSnapshot``."""
        cur = self.meta.get("iteration")
        if _js_strict_ne(cur, self._last_iter):
            self.meta.set("prevSnapshot", self.snapshot_metrics())
            self._last_iter = cur

    def set_mode(self, mode: str):
        self._set_meta_mode(mode)

    def set_iteration(self, value):
        """Advance the iteration label; on change, freeze the current metrics as
        ``prevSnapshot`` (the baseline for dashboard deltas, app.mjs:498-505)."""
        try:
            it = int(value) if value not in (None, "") else 0
        except (TypeError, ValueError):
            it = 0
        self.meta.set("iteration", it)
        self._iteration_hook()

    # ---------------------------------------------------------------- metrics
    def members(self, cid: str) -> list[dict]:
        return [c for c in self.cards if c.get("assignedTo") == cid]

    def snapshot_metrics(self) -> dict:
        return tr.snapshot_metrics(self.cards, self.centroids)

    def dashboard(self) -> dict:
        """Text of every dashboard element, exactly as renderKMeans would show it."""
        now = self.snapshot_metrics()
        prev = self.meta.get("prevSnapshot")
        total = len(self.cards)
        unassigned = sum(1 for c in self.cards if not c.get("assignedTo"))
        chips = [f"k = {len(self.centroids)}", f"balance gap = {now['balance']['gap']}",
                 f"avg cohesion = {mm.avg_cohesion_pct(now['avgCohesion'])}%", f"unassigned = {unassigned}"]
        deltas = []
        if prev:
            deltas = [mm.delta_gap_text(now["balance"]["gap"], prev["balance"]["gap"]),
                      mm.delta_pp_text(now["avgCohesion"], prev["avgCohesion"])]
        rows = []
        for c in self.centroids:
            cid = c["id"]
            count = now["counts"].get(cid, 0)
            coh = now["cohesion"].get(cid, 1)
            cnts = tr.trait_counts(self.members(cid))
            sug = tr.suggestion(cnts)
            row = {
                "id": cid,
                "name": f"{c['name']}: {count}",
                "bar_pct": mm.bar_pct(count, total),
                "color": c.get("color"),
                "cohesion": f"cohesion = {mm.cohesion_pct(coh)}%",
                "top": tr.top_text(cnts),
                "suggested": f"Suggested: {sug}" if sug else "Suggested: —",
                "suggestion": sug,
            }
            if prev:
                p = (prev.get("cohesion") or {}).get(cid, 1)
                row["cohesion_delta"] = mm.delta_pp_text(coh, p)
            rows.append(row)
        return {"chips": chips, "deltas": deltas, "rows": rows, "metrics": now}

    # --------------------------------------------------------------------- IO
    def export_obj(self) -> dict:
        return {"cards": self.cards, "centroids": self.centroids, "meta": self.meta.to_dict()}

    def export_json(self) -> str:
        """``JSON.stringify({cards, centroids, meta}, null, 2)``: byte-exact, no trailing newline."""
        return jsjson.stringify(self.export_obj(), 2)

    @property
    def export_filename(self) -> str:
        return f"kmeans-room-{self.room}.json"

    def import_json(self, text: str, *, compat: bool = False):
        """Replace cards / centroids and MERGE meta (app.mjs:272-279), then dedupe seeds.

        ``compat=True`` reproduces the reference exactly, including clearing cards
        and centroids when the file lacks those fields (defect #9)."""
        data = jsjson.parse(text)
        if not isinstance(data, dict):
            raise ValueError("room JSON must be an object")
        if compat or isinstance(data.get("cards"), list):
            self.cards = list(data["cards"]) if isinstance(data.get("cards"), list) else []
        if compat or isinstance(data.get("centroids"), list):
            self.centroids = list(data["centroids"]) if isinstance(data.get("centroids"), list) else []
        meta = data.get("meta")
        if isinstance(meta, dict):
            for k, v in meta.items():
                if k == "mode":
                    self._set_meta_mode(v)
                else:
                    self.meta.set(k, v)
            # the observer runs at the end of the import transaction, before dedupeSeeds
            # (app.mjs:272-279): an imported iteration that differs from the last seen one
            # overwrites the imported prevSnapshot with the (pre-dedupe) board's metrics
            if "iteration" in meta:
                self._iteration_hook()
        self.dedupe_seeds()
        self.log.append(("import",))

    @classmethod
    def from_json(cls, text: str, room_id: str | None = None, **kw) -> "Room":
        r = cls(room_id, seed_jessica=False, **kw)
        r.import_json(text)
        return r

    # ------------------------------------------------------- numeric k-means
    def auto_assign(self, *, seed: int = 0, max_iter: int = 50, device="cpu") -> dict:
        """Cluster the cards with numeric k-means on multi-hot trait vectors.

        K = number of unlocked centroids; locked centroids keep their members and
        take no new cards.  Seeds: the members' mean for a centroid that already
        has cards, else k-means++ over the free cards.  Returns the new dashboard."""
        import numpy as np
        import torch

        from ..api import KMeans

        free_c = [c for c in self.centroids if not c.get("locked")]
        locked_ids = {c["id"] for c in self.centroids if c.get("locked")}
        cards = [c for c in self.cards if c.get("assignedTo") not in locked_ids]
        if not free_c or not cards:
            return self.dashboard()
        X, vocab = tr.encode_traits(cards)
        K = min(len(free_c), len(cards))
        init = []
        rng = np.random.default_rng(seed)
        for c in free_c[:K]:
            idx = [i for i, card in enumerate(cards) if card.get("assignedTo") == c["id"]]
            init.append(X[idx].mean(0) if idx else None)
        if any(v is None for v in init):
            from ..models.init import init_kmeanspp
            from ..parallel.comm import Comm

            pp = init_kmeanspp(torch.from_numpy(X), X.shape[1], K, len(cards), 0, Comm.local(), seed).numpy()
            init = [v if v is not None else pp[j] for j, v in enumerate(init)]
        km = KMeans(K, init=np.stack(init).astype(np.float32), max_iter=max_iter, tol=0, device=device,
                    seed=seed).fit(X)
        labels = km.labels_.cpu().numpy() if torch.is_tensor(km.labels_) else km.labels_
        for card, lab in zip(cards, labels):
            self.update_card_assign(card["id"], free_c[int(lab)]["id"])
        del rng
        return self.dashboard()
