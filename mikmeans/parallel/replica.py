"""Replicated trait-card room over ``torch.distributed`` (the reference's P2P/CRDT layer).

The reference keeps one Yjs document per browser tab and floods every
transaction's delta to all WebRTC peers (``broadcastUpdate``, app.mjs:68, :121;
``Y.applyUpdate`` on receipt, :110), sends ``HELLO``/``ROSTER`` presence messages
(:66-67, :94-95) and intends a full-state sync when a peer connects
(``encodeStateAsUpdate``, :96 -- broken in the reference).  That
design is eventually consistent and duplicates records when two peers edit the
same card at once.

Here every rank holds a :class:`~mikmeans.models.room.Room` replica and the ranks
replicate by **bulk-synchronous total-order broadcast**:

* join = full-state sync: rank 0 builds (or imports) the room and broadcasts its
  export JSON plus the room code; every other replica starts from those bytes;
* local edits are queued as JSON ops (ids, random draws and positions resolved
  by the issuing rank, so applying an op is a pure function of the state);
* :meth:`RoomReplica.sync` all-gathers the queued ops (one variable-length byte
  collective, no pickling) and every replica applies the same ops in the same
  (rank, sequence) order, so replicas stay byte-identical -- concurrent edits to
  one card resolve deterministically instead of duplicating it;
* presence (``HELLO``/``ROSTER``) rides on the same collective; ``digest`` /
  :meth:`RoomReplica.check` detect divergence (which the reference cannot).
"""
from __future__ import annotations

import hashlib
import json
import random as _random

from ..models.room import Room
from .comm import Comm

#: Room methods that may be replicated, with the reference lines they mirror.
OPS = {
    "add_centroid": "app.mjs:126-129",
    "remove_centroid": "app.mjs:130-142",
    "rename_centroid": "app.mjs:332-338",
    "toggle_lock": "app.mjs:341-347",
    "apply_suggested_name": "app.mjs:571-573",
    "add_card": "app.mjs:143-145",
    "update_card_assign": "app.mjs:146-156",
    "drop_card": "app.mjs:358-371",
    "delete_card": "app.mjs:179-186",
    "set_card_pos": "app.mjs:157",
    "shuffle_unassigned": "app.mjs:159-166",
    "restart_all": "app.mjs:167-178",
    "populate_test_data": "app.mjs:202-224",
    "hard_reset": "app.mjs:225-237",
    "set_mode": "app.mjs:287",
    "set_iteration": "app.mjs:288, :498-505",
    "import_json": "app.mjs:268-282",
    "auto_assign": "(new) numeric k-means over trait vectors",
}


class RoomReplica:
    def __init__(self, comm: Comm, room_id: str | None = None, *, user: str | None = None, seed: int = 0,
                 state_json: str | None = None, clock=None):
        self.comm = comm
        self._rng = _random.Random(seed * 1_000_003 + comm.rank)  # per-rank ids / draws
        if comm.rank == 0:
            if state_json is not None:
                base = Room.from_json(state_json, room_id, seed=seed, clock=clock)
            else:
                base = Room(room_id, seed=seed, clock=clock)
            hello = json.dumps({"room": base.room, "state": base.export_json()}).encode()
        else:
            hello = None
        init = json.loads(comm.broadcast_bytes(hello, 0).decode())
        self.room = Room.from_json(init["state"], init["room"], seed=seed, clock=clock)
        self.room.user = user or f"Guest {self.room.room}"
        self.room._last_iter = self.room.meta.get("iteration")
        self._pending: list[dict] = []
        self._seq = 0
        self.round = 0
        self.roster: list[str] = []
        self.sync()

    # ------------------------------------------------------------ local edits
    def submit(self, op: str, *args, **kw) -> dict:
        if op not in OPS:
            raise ValueError(f"unknown room op {op!r}")
        rec = {"op": op, "args": list(args), "kw": kw, "rank": self.comm.rank, "seq": self._seq,
               "user": self.room.user}
        self._seq += 1
        self._pending.append(rec)
        return rec

    def _new_id(self, prefix: str) -> str:
        from ..models.room import js_base36_fraction

        return f"{prefix}:{self.room.clock()}-{js_base36_fraction(self._rng.random())}"

    def add_centroid(self, name: str | None = None) -> str:
        cid = self._new_id("c")
        self.submit("add_centroid", name, cid=cid)
        return cid

    def add_card(self, title: str, traits) -> str:
        card_id = self._new_id("card")
        self.submit("add_card", title, list(traits), card_id=card_id, created_by=self.room.user)
        return card_id

    def shuffle_unassigned(self):
        self.submit("shuffle_unassigned", seed=self._rng.getrandbits(52))

    def auto_assign(self, seed: int | None = None):
        self.submit("auto_assign", seed=int(self._rng.getrandbits(31) if seed is None else seed))

    def __getattr__(self, name):
        if name in OPS:
            return lambda *a, **k: self.submit(name, *a, **k)
        raise AttributeError(name)

    # ---------------------------------------------------------- replication
    def _apply(self, rec: dict) -> bool:
        """Apply one op; an op that raises (a malformed import, say) raises on every replica
        alike -- same state, same op -- so it is skipped everywhere and the round goes on."""
        try:
            self._apply_op(rec)
            return True
        except (ValueError, TypeError, KeyError, AttributeError, IndexError):
            return False

    def _apply_op(self, rec: dict):
        r = self.room
        op, args, kw = rec["op"], rec["args"], rec["kw"]
        if op == "shuffle_unassigned":
            saved, r.rng = r.rng, _random.Random(kw["seed"])
            try:
                r.shuffle_unassigned()
            finally:
                r.rng = saved
            return
        if op == "auto_assign":
            r.auto_assign(seed=kw["seed"], device="cpu")
            return
        getattr(r, op)(*args, **kw)

    def sync(self) -> list[dict]:
        """One replication round: exchange queued ops + presence, apply in total order."""
        msg = json.dumps({"user": self.room.user, "ops": self._pending}).encode()
        self._pending = []
        parts = [json.loads(b.decode()) for b in self.comm.all_gather_bytes(msg)]
        self.roster = [p["user"] for p in parts]
        applied = []
        for p in parts:                      # rank order, then per-rank sequence order
            for rec in p["ops"]:
                self._apply(rec)
                applied.append(rec)
        self.round += 1
        return applied

    # ------------------------------------------------------------- presence
    @property
    def peers(self) -> int:
        """``Peers: N`` of the reference status chip (app.mjs:51-58)."""
        return self.comm.world - 1

    def digest(self) -> str:
        return hashlib.sha256(self.room.export_json().encode()).hexdigest()

    def check(self) -> bool:
        """True iff every replica's export JSON is byte-identical."""
        ds = self.comm.all_gather_bytes(self.digest().encode())
        return len(set(ds)) == 1
