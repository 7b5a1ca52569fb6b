"""Live membership for the replicated room: ranks join and leave a running session.

The reference's peers come and go at any time: ``p2p.on("peerconnect")`` adds a peer and
(intends to) send it the full state, ``peerclose`` drops it (app.mjs:82-105, full-state
sync at :96).  A ``torch.distributed`` default group has a fixed world, so here a session
is a sequence of **membership epochs**, each its own gloo process group built on a prefix
of one shared TCPStore (the rendezvous the trackers stand for, app.mjs:39-45):

* ``mk/join/n`` + ``mk/join/<i>`` -- join requests, appended by a newcomer;
* ``mk/leave/<member>`` -- a member's notice that it is leaving;
* ``mk/epoch/<e>`` -- the member ids of epoch e, in rank order.

Every :meth:`ElasticRoomReplica.sync` round is bulk-synchronous.  The epoch's rank 0 reads
the pending requests from the store *before* the round and puts the next epoch's member
list into its own message, so every member learns the change from the same all-gather and
applies it after the round's ops: survivors and newcomers form the epoch-(e+1) group
(``ProcessGroupGloo`` on ``PrefixStore("mk/e<e+1>")``), the new rank 0 broadcasts the room
export JSON (the full-state sync the reference's ``sendInitial`` intends), and leavers
close.  Replicas therefore stay byte-identical across every change (``check``).

A member that dies without notice stalls the round until the group's timeout, as a dead
rank stalls any collective (utils/faults.py); recovery then is the checkpoint path.
"""
from __future__ import annotations

import datetime
import json
import os
import random as _random
import zlib

import torch
import torch.distributed as dist

from ..models.room import Room
from .comm import Comm
from .replica import RoomReplica

_PREFIX = "mk/"


class GroupComm(Comm):
    """A CPU :class:`Comm` over an explicit gloo process-group object (one membership
    epoch), so a new group can be formed without re-initialising the default one."""

    def __init__(self, pg, rank: int, world: int):
        super().__init__(rank=rank, world=world, local_rank=rank, backend="gloo", device=torch.device("cpu"))
        self.pg = pg

    @property
    def grouped(self) -> bool:
        return self.pg is not None

    def allreduce_(self, t):
        if self.pg is not None:
            self.pg.allreduce([t]).wait()
        return t

    def allreduce_max_(self, t):
        if self.pg is not None:
            opts = dist.AllreduceOptions()
            opts.reduceOp = dist.ReduceOp.MAX
            self.pg.allreduce([t], opts).wait()
        return t

    def broadcast_(self, t, src: int = 0):
        if self.pg is not None:
            opts = dist.BroadcastOptions()
            opts.rootRank = src
            self.pg.broadcast([t], opts).wait()
        return t

    def all_gather(self, t):
        if self.pg is None:
            return t.unsqueeze(0).clone()
        src = t.contiguous()
        outs = [torch.empty_like(src) for _ in range(self.world)]
        self.pg.allgather([outs], [src]).wait()
        return torch.stack(outs)

    def all_gather_object(self, obj):
        raise NotImplementedError("GroupComm moves bytes, never pickles: use all_gather_bytes")

    def broadcast_object(self, obj, src: int = 0):
        raise NotImplementedError("GroupComm moves bytes, never pickles: use broadcast_bytes")

    def barrier(self):
        if self.pg is not None:
            self.pg.barrier().wait()

    def close(self):
        self.pg = None


class ElasticRoomReplica(RoomReplica):
    """A :class:`RoomReplica` whose membership may change between rounds.

    ``found`` starts a session (epoch 0, this process alone); ``join`` enters a running one
    (blocks until a round admits it, then receives the full state); ``leave`` departs at
    the next round.  ``member`` is this process's unique id (the reference's peer id)."""

    def __init__(self, store, member: str, *, user: str | None = None, seed: int = 0, clock=None,
                 timeout_s: float = 120.0):
        # (use found() / join(); the base class's constructor is not run)
        self.store = store
        self.member = member
        self.timeout = datetime.timedelta(seconds=timeout_s)
        self.seed = seed
        self.clock = clock
        self._rng = _random.Random(seed * 1_000_003 + zlib.crc32(member.encode()))   # per-member ids / draws
        self._pending: list[dict] = []
        self._seq = 0
        self.round = 0
        self.roster: list[str] = []
        self.epoch = -1
        self.members: list[str] = []
        self.left = False
        self._user = user
        self._joins_seen = 0
        # join slots counted (join/n) but not written yet -- a newcomer slow or dead between its
        # add and its set: re-checked every round instead of blocking rank 0 on a get
        self._join_holes: list[int] = []

    # ------------------------------------------------------------ lifecycle
    @classmethod
    def found(cls, store, member: str, room_id: str | None = None, *, state_json: str | None = None,
              **kw) -> "ElasticRoomReplica":
        rep = cls(store, member, **kw)
        base = (Room.from_json(state_json, room_id, seed=rep.seed, clock=rep.clock) if state_json is not None
                else Room(room_id, seed=rep.seed, clock=rep.clock))
        rep._set_room(base.export_json(), base.room, 0)
        store.set(_PREFIX + "epoch/0", json.dumps([member]))
        rep._form(0, [member])
        return rep

    @classmethod
    def join(cls, store, member: str, **kw) -> "ElasticRoomReplica":
        """Ask to join; returns once a round of the running session has admitted this member
        and the full state has arrived (the reference's peerconnect + sendInitial)."""
        rep = cls(store, member, **kw)
        i = store.add(_PREFIX + "join/n", 1) - 1
        store.set(_PREFIX + f"join/{i}", member)
        # the admitting round names its epoch under this join's own slot (a member id that
        # left and rejoins must not take an old epoch that listed it)
        store.wait([_PREFIX + f"admit/{i}"], rep.timeout)
        e = int(store.get(_PREFIX + f"admit/{i}").decode())
        if e < 0:
            raise ValueError(f"member id {member!r} is already in the session")
        members = json.loads(store.get(_PREFIX + f"epoch/{e}").decode())
        rep._form(e, members)
        rep._receive_state()
        return rep

    def leave(self):
        """Announce departure; the next :meth:`sync` round releases this member."""
        self.store.set(_PREFIX + f"leave/{self.member}", "1")

    # ------------------------------------------------------------- epochs
    def _form(self, epoch: int, members: list[str]):
        rank = members.index(self.member)
        pre = dist.PrefixStore(_PREFIX + f"e{epoch}", self.store)
        pg = None
        if len(members) > 1:
            opts = dist.ProcessGroupGloo._Options()
            opts._timeout = self.timeout
            # the address peers reach this process on (MIKMEANS_GLOO_HOST; loopback for a
            # one-host session -- the container hostname may not resolve)
            host = os.environ.get("MIKMEANS_GLOO_HOST", "127.0.0.1")
            opts._devices = [dist.ProcessGroupGloo.create_device(hostname=host)]
            pg = dist.ProcessGroupGloo(pre, rank, len(members), opts)
        self.comm = GroupComm(pg, rank, len(members))
        self.epoch = epoch
        self.members = list(members)

    def _set_room(self, state_json: str, room_id: str, rnd: int):
        self.room = Room.from_json(state_json, room_id, seed=self.seed, clock=self.clock)
        self.room.user = self._user or f"Guest {self.room.room}"
        self.room._last_iter = self.room.meta.get("iteration")
        self.round = rnd

    def _full_state(self):
        """The epoch's rank 0 sends room code, round and export JSON to every member."""
        if self.comm.rank == 0:
            blob = json.dumps({"room": self.room.room, "round": self.round, "joins_seen": self._joins_seen,
                               "join_holes": self._join_holes, "state": self.room.export_json()}).encode()
        else:
            blob = None
        return json.loads(self.comm.broadcast_bytes(blob, 0).decode())

    def _receive_state(self):
        init = self._full_state()
        self._set_room(init["state"], init["room"], init["round"])
        self._joins_seen = init["joins_seen"]
        self._join_holes = list(init.get("join_holes", []))

    def _pending_change(self) -> dict | None:
        """(epoch rank 0) the next epoch's member list, if anyone asked to join or leave."""
        n = self.store.add(_PREFIX + "join/n", 0)
        joins, holes, slots = [], [], []
        for i in [*self._join_holes, *range(self._joins_seen, n)]:
            key = _PREFIX + f"join/{i}"
            if self.store.check([key]):
                joins.append(self.store.get(key).decode())
                slots.append(i)
            else:
                holes.append(i)
        leaves = [m for m in self.members if self.store.check([_PREFIX + f"leave/{m}"])]
        if not joins and not leaves:
            if holes != self._join_holes or n != self._joins_seen:
                # (only new holes: nobody to admit yet; remember them through the next round)
                return {"epoch": None, "members": None, "joins_seen": n, "join_holes": holes}
            return None
        # A member id that leaves and joins again before this round is both released (its old
        # process closes) and admitted (its new one takes the id's place).  An id already in the
        # session and not leaving, or asked for twice, is refused through its own slot (-1).
        members = [m for m in self.members if m not in leaves]
        admit, refuse = [], []
        for m, i in zip(joins, slots):
            if m in members:
                refuse.append(i)
            else:
                members.append(m)
                admit.append(i)
        return {"epoch": self.epoch + 1, "members": members, "joins_seen": n, "join_holes": holes,
                "leaves": leaves, "admit": admit, "refuse": refuse}

    # ---------------------------------------------------------- replication
    def sync(self) -> list[dict]:
        """One round: exchange queued ops (+ presence and, from rank 0, any membership
        change), apply them in (rank, sequence) order, then move to the next epoch."""
        parts = self.round_exchange(self.round_begin())
        applied, change = self.round_apply(parts)
        if change is not None:
            self.round_transition(change)
        return applied

    # A round in four steps, so a server (serve.py) holds its board lock only for the local
    # ones -- begin (take the queued ops) and apply -- and runs the collectives without it.
    def round_begin(self) -> bytes:
        """The round's message: this member's queued ops, its name and (rank 0) the change."""
        if self.left:
            raise RuntimeError(f"member {self.member} has left the session")
        change = self._pending_change() if self.comm.rank == 0 else None
        msg = json.dumps({"user": self.room.user, "ops": self._pending, "change": change}).encode()
        self._pending = []
        return msg

    def round_exchange(self, msg: bytes) -> list[dict]:
        """The round's collective: every member's message."""
        return [json.loads(b.decode()) for b in self.comm.all_gather_bytes(msg)]

    def round_apply(self, parts: list[dict]):
        """Apply the gathered ops in (rank, sequence) order; returns (applied ops, the
        membership change to move to, or None)."""
        self.roster = [p["user"] for p in parts]
        applied = []
        for p in parts:
            for rec in p["ops"]:
                self._apply(rec)
                applied.append(rec)
        self.round += 1
        change = parts[0]["change"]
        if change is None:
            return applied, None
        self._joins_seen = change["joins_seen"]
        self._join_holes = list(change.get("join_holes", []))
        if change["epoch"] is None:   # bookkeeping only (unwritten join slots), same members
            return applied, None
        return applied, change

    def round_transition(self, change: dict) -> bool:
        """Move to the change's epoch: publish it (rank 0), close this group, then leave or
        form the new group and take the full state.  True when this member stays."""
        if self.comm.rank == 0:       # publish before anyone forms the new group
            self.store.set(_PREFIX + f"epoch/{change['epoch']}", json.dumps(change["members"]))
            for i in change.get("admit", []):
                self.store.set(_PREFIX + f"admit/{i}", str(change["epoch"]))
            for i in change.get("refuse", []):
                self.store.set(_PREFIX + f"admit/{i}", "-1")
            for m in change.get("leaves", []):   # applied: a member id may rejoin later
                try:
                    self.store.delete_key(_PREFIX + f"leave/{m}")
                except Exception:  # noqa: BLE001 -- a store without deletes keeps the notice
                    pass
        self.comm.close()
        if self.member in change.get("leaves", []) or self.member not in change["members"]:
            self.left = True          # the reference's peerclose, seen from this side
            return False
        self._form(change["epoch"], change["members"])
        st = self._full_state()       # newcomers take it; survivors already hold it
        assert st["state"] == self.room.export_json() and st["round"] == self.round, "replica diverged"
        return True

    def submit(self, op: str, *args, **kw) -> dict:
        rec = super().submit(op, *args, **kw)
        rec["rank"] = self.member     # ranks change between epochs; the member id does not
        return rec

    @property
    def peers(self) -> int:
        return len(self.members) - 1
