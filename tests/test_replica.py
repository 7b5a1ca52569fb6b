"""Room replication over torch.distributed (gloo ranks): the P2P/CRDT analogue."""
import json

from mikmeans.parallel.launch import spawn_local


def _session(comm):
    from mikmeans.parallel.replica import RoomReplica

    rep = RoomReplica(comm, "ROOM" if comm.rank == 0 else None, user=f"user{comm.rank}", seed=7)
    out = {"room": rep.room.room, "roster": list(rep.roster), "peers": rep.peers}
    # round 1: rank 0 adds centroids and test data, others add their own card
    if comm.rank == 0:
        a = rep.add_centroid("Sweet")
        b = rep.add_centroid("Fresh")
        rep.populate_test_data()
    else:
        rep.add_card(f"card from {comm.rank}", ["Sweet", "Fresh"])
    rep.sync()
    ids = [c["id"] for c in rep.room.centroids]
    # round 2: concurrent conflicting edits on the same card / centroid
    if comm.rank == 0:
        rep.toggle_lock(ids[0])                       # lock first (rank order) ...
    rep.drop_card("seed:t1", ids[0], 0.5, 0.5)        # ... so every drop on it is refused
    rep.update_card_assign("seed:t2", ids[comm.rank % 2])
    rep.shuffle_unassigned()
    rep.sync()
    # round 3: iteration change snapshot + numeric auto-assign
    if comm.rank == comm.world - 1:
        rep.set_iteration(1)
        rep.auto_assign(seed=3)
    rep.sync()
    out.update(consistent=rep.check(), export=rep.room.export_json(), n_cards=len(rep.room.cards),
               t1=next(c for c in rep.room.cards if c["id"] == "seed:t1")["assignedTo"],
               locked=rep.room.centroids[0]["locked"])
    return out


def test_replicas_converge_deterministically():
    res = spawn_local(_session, 3)
    assert all(r["consistent"] for r in res)
    assert len({r["export"] for r in res}) == 1
    assert {r["room"] for r in res} == {"ROOM"}
    assert res[0]["roster"] == ["user0", "user1", "user2"] and res[1]["peers"] == 2
    assert res[0]["n_cards"] == 1 + 11 + 2                       # Jessica + test data + 2 peer cards
    assert res[0]["locked"] is True
    exp = json.loads(res[0]["export"])
    assert exp["meta"]["iteration"] == 1 and "prevSnapshot" in exp["meta"]
    assert sum(1 for c in exp["cards"] if c["id"] == "seed:jessica") == 1  # no duplicated seeds
    assert len({c["id"] for c in exp["cards"]}) == len(exp["cards"])


def _join_from_state(comm, state):
    from mikmeans.parallel.replica import RoomReplica

    rep = RoomReplica(comm, "R2", state_json=state if comm.rank == 0 else None)
    return rep.room.export_json()


def test_full_state_sync_on_join():
    from mikmeans.models.room import Room

    r = Room("R2", seed=1)
    r.populate_test_data()
    r.add_centroid("X")
    r.update_card_assign("seed:t3", r.centroids[0]["id"])
    res = spawn_local(_join_from_state, 2, r.export_json())
    assert res[0] == res[1] == r.export_json()
