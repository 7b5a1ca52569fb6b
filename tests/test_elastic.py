"""Live membership of the replicated room (parallel/elastic.py): members join and leave a
running session -- the reference's peerconnect / peerclose with full-state sync on join
(app.mjs:82-105, :96) -- and every member reports the same room after every round.

CPU processes on 127.0.0.1 around one TCPStore the test hosts (the tracker's role)."""
import datetime
import json
import time

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from mikmeans.parallel.launch import free_port

ROUNDS = 30


def _store(port, master=False):
    return dist.TCPStore("127.0.0.1", port, is_master=master, wait_for_workers=False,
                         timeout=datetime.timedelta(seconds=60))


def _record(store, rep):
    store.set(f"dig/{rep.member}/{rep.round}", json.dumps({"d": rep.digest(), "epoch": rep.epoch,
                                                          "peers": rep.peers}))


def _member(port, member, delay, leave_at):
    from mikmeans.parallel.elastic import ElasticRoomReplica

    store = _store(port)
    time.sleep(delay)
    if member == "A":
        rep = ElasticRoomReplica.found(store, member, "ROOM", user=member, seed=3)
    else:
        rep = ElasticRoomReplica.join(store, member, user=member, seed=3)
    store.set(f"joined/{member}", str(rep.round))
    asked = False
    first = True
    while rep.round < ROUNDS and not rep.left:
        if rep.round % 3 == 0 or first:     # (a late joiner under load still leaves a card)
            rep.add_card(f"{member}-{rep.round}", ["Mint", "Choc"])
            first = False
        if member == "A" and rep.round == 5:
            rep.add_centroid("Fresh")
        if leave_at is not None and rep.round >= leave_at and not asked:
            rep.leave()
            asked = True
        rep.sync()
        if not rep.left:
            _record(store, rep)
        time.sleep(0.05)
    store.set(f"done/{member}", json.dumps({"round": rep.round, "left": rep.left,
                                            "cards": [c["title"] for c in rep.room.cards]}))
    if not rep.left:
        assert rep.check()          # one more collective: every remaining replica identical


@pytest.mark.timeout(240)
def test_members_join_and_leave_a_running_session():
    port = free_port()
    store = _store(port, master=True)
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_member, args=(port, "A", 0.0, None)),
             ctx.Process(target=_member, args=(port, "B", 0.3, 12)),     # joins early, leaves
             ctx.Process(target=_member, args=(port, "C", 0.9, None))]   # joins later
    for p in procs:
        p.start()
    for p in procs:
        p.join(200)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    done = {m: json.loads(store.get(f"done/{m}").decode()) for m in "ABC"}
    assert done["A"]["round"] == done["C"]["round"] == ROUNDS
    assert done["B"]["left"] and done["B"]["round"] < ROUNDS
    joined = {m: int(store.get(f"joined/{m}").decode()) for m in "BC"}
    assert 0 < joined["B"] < joined["C"] < ROUNDS
    # every member present after a round reports the same room (digest) that round
    for r in range(1, ROUNDS + 1):
        ds = []
        for m in "ABC":
            if store.check([f"dig/{m}/{r}"]):
                ds.append(json.loads(store.get(f"dig/{m}/{r}").decode()))
        assert ds and len({d["d"] for d in ds}) == 1, (r, ds)
        # (a member admitted in round r records from round r + 1 on)
        assert len({(d["epoch"], d["peers"]) for d in ds}) == 1, (r, ds)
    # the final room holds every member's cards, B's from before it left
    cards = done["A"]["cards"]
    assert cards == done["C"]["cards"]
    assert any(t.startswith("B-") for t in cards) and any(t.startswith("C-") for t in cards)


def test_cli_session_found_and_join(tmp_path):
    """`python -m mikmeans session`: a founder hosting the rendezvous and a joiner editing the
    same room end with byte-identical exports holding both members' edits."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    port = str(free_port())
    base = [sys.executable, "-m", "mikmeans", "session", "--port", port, "--until-round", "40",
            "--interval", "0.1"]
    a = subprocess.Popen(base + ["--found", "CLIR", "--user", "Ann", "--centroid", "Sweet",
                                 "--card", "Mango:Fruity,Sweet", "--export", str(tmp_path / "a.json")],
                         cwd=root, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    b = subprocess.Popen(base + ["--join", "--user", "Bob", "--card", "Lime:Sour", "--export",
                                 str(tmp_path / "b.json")],
                         cwd=root, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    out_a, err_a = a.communicate(timeout=120)
    out_b, err_b = b.communicate(timeout=120)
    assert a.returncode == 0 and b.returncode == 0, (err_a[-2000:], err_b[-2000:])
    ja, jb = (tmp_path / "a.json").read_text(), (tmp_path / "b.json").read_text()
    assert ja == jb
    titles = [c["title"] for c in json.loads(ja)["cards"]]
    assert "Mango" in titles and "Lime" in titles
    last_b = json.loads(out_b.strip().splitlines()[-1])
    assert last_b["round"] == 40 and last_b["peers"] == 1 and sorted(last_b["roster"]) == ["Ann", "Bob"]


def _rejoiner(port, member, rounds):
    """A member that joins, leaves, then joins again under the same id."""
    from mikmeans.parallel.elastic import ElasticRoomReplica

    store = _store(port)
    for visit in range(2):
        rep = ElasticRoomReplica.join(store, member, user=member, seed=3)
        store.set(f"visit/{member}/{visit}", json.dumps({"epoch": rep.epoch, "round": rep.round}))
        rep.add_card(f"{member}-visit{visit}", ["Tart"])
        for _ in range(rounds):
            rep.sync()
            time.sleep(0.05)
        rep.leave()
        while not rep.left:
            rep.sync()
    store.set(f"done/{member}", "1")


def _host(port, deadline_s):
    from mikmeans.parallel.elastic import _PREFIX, ElasticRoomReplica

    store = _store(port)
    rep = ElasticRoomReplica.found(store, "A", "ROOM2", user="A", seed=3)
    # a join slot counted but never written (a newcomer that died between its add and its set)
    store.add(_PREFIX + "join/n", 1)
    # rounds until the rejoiner is done, under a wall-clock deadline (a round cap raced the
    # rejoiner's two visits on a loaded box)
    t_end = time.monotonic() + deadline_s
    while not store.check(["done/R"]) and time.monotonic() < t_end:
        rep.sync()
        time.sleep(0.05)
    store.set("done/A", json.dumps({"round": rep.round, "cards": [c["title"] for c in rep.room.cards],
                                    "holes": rep._join_holes}))


@pytest.mark.timeout(240)
def test_member_rejoins_and_dead_join_slot_does_not_block():
    """ A member id that left can join again: its leave notice was deleted once
    applied and it is admitted through its own join slot, not an old epoch that listed it.  A
    join slot counted but never written does not block the session: it stays a hole that is
    re-checked each round."""
    port = free_port()
    store = _store(port, master=True)
    ctx = mp.get_context("spawn")
    host = ctx.Process(target=_host, args=(port, 180.0))
    host.start()
    time.sleep(0.5)
    r = ctx.Process(target=_rejoiner, args=(port, "R", 4))
    r.start()
    for p in (r, host):
        p.join(200)
    assert host.exitcode == 0 and r.exitcode == 0, (host.exitcode, r.exitcode)
    v0 = json.loads(store.get("visit/R/0").decode())
    v1 = json.loads(store.get("visit/R/1").decode())
    assert v1["epoch"] > v0["epoch"] + 1 and v1["round"] > v0["round"]
    done = json.loads(store.get("done/A").decode())
    assert "R-visit0" in done["cards"] and "R-visit1" in done["cards"]
    assert done["holes"] == [0]


def test_leave_and_rejoin_in_one_round_and_duplicate_ids():
    """ A member id whose leave notice and new join request are pending in the
    same round is released (its old process closes) AND admitted (the new process takes the
    id); a join under an id still in the session is refused through its own slot."""
    from mikmeans.parallel.elastic import _PREFIX, ElasticRoomReplica

    port = free_port()
    store = _store(port, master=True)
    rep = ElasticRoomReplica.found(store, "A", "ROOM3", user="A", seed=3)
    rep.members = ["A", "R", "S"]          # (as if R and S had been admitted earlier)
    store.set(_PREFIX + "leave/R", "1")
    for m in ("R", "S", "Q"):             # R rejoins, S is a duplicate, Q is new
        i = store.add(_PREFIX + "join/n", 1) - 1
        store.set(_PREFIX + f"join/{i}", m)
    ch = rep._pending_change()
    assert ch["members"] == ["A", "S", "R", "Q"]
    assert ch["leaves"] == ["R"] and ch["admit"] == [0, 2] and ch["refuse"] == [1]
