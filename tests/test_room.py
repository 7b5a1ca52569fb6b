"""Trait-card room model: mutations, seeds, dashboard, byte-exact export/import."""
import json
import re

import pytest

from mikmeans.models.room import COLORS, OrderedMeta, Room, js_base36_fraction, room_code
from mikmeans.utils import jsjson

from .jsnode import NODE, run_js


def make_room(**kw):
    t = iter(range(1700000000000, 1700000001000))
    return Room("ABCD", user="Ada", seed=1, clock=lambda: next(t), **kw)


def test_room_code_and_ids():
    code = room_code()
    assert re.fullmatch(r"[ABCDEFGHJKLMNPQRSTUVWXYZ23456789]{4}", code)
    r = make_room()
    c = r.add_centroid()
    assert re.fullmatch(r"c:\d{13}-[0-9a-z]{1,5}", c["id"])
    assert c == {"id": c["id"], "name": "Centroid 1", "color": COLORS[0], "locked": False}
    assert js_base36_fraction(0.5) == "i"


def test_jessica_seeded_once():
    r = make_room()
    assert [c["id"] for c in r.cards] == ["seed:jessica"]
    assert r.meta.get("seededJessica") is True
    r.ensure_jessica_once()
    assert len(r.cards) == 1


def test_centroid_limit_colors_and_remove():
    r = make_room()
    cs = [r.add_centroid(n) for n in ("Sweet", None, "Rich")]
    assert r.add_centroid("extra") is None
    assert [c["color"] for c in cs] == COLORS[:3]
    assert cs[1]["name"] == "Centroid 2"
    r.populate_test_data()
    assert r.drop_card("seed:t1", cs[0]["id"], 0.5, 0.5)
    r.remove_centroid(cs[0]["id"])
    assert r.get_card_pos("seed:t1") is None
    assert next(c for c in r.cards if c["id"] == "seed:t1")["assignedTo"] is None
    assert r.add_centroid()["color"] == COLORS[0]  # first free colour again


def test_populate_idempotent_and_dedupe():
    r = make_room()
    r.populate_test_data()
    r.populate_test_data()
    assert len(r.cards) == 12
    r.cards.append(dict(r.cards[3]))
    r.dedupe_seeds()
    assert len(r.cards) == 12


def test_drop_lock_and_clamp():
    r = make_room()
    r.populate_test_data()
    a, b = r.add_centroid("A"), r.add_centroid("B")
    assert r.drop_card("seed:t2", a["id"], 1.5, -3)
    assert r.get_card_pos("seed:t2") == {"x": 0.92, "y": 0.10}
    r.toggle_lock(b["id"])
    assert not r.drop_card("seed:t3", b["id"], 0.5, 0.5)
    # the lock also holds on the <select> path (reference defect #3 fixed)
    assert not r.update_card_assign("seed:t3", b["id"])
    r.toggle_lock(b["id"])
    assert r.update_card_assign("seed:t3", b["id"])
    assert r.update_card_assign("seed:t2", None)
    assert r.get_card_pos("seed:t2") is None


def test_restart_shuffle_delete_reset():
    r = make_room()
    r.populate_test_data()
    a = r.add_centroid()
    for cid in ("seed:t1", "seed:t5"):
        r.drop_card(cid, a["id"], 0.3, 0.3)
    r.shuffle_unassigned()
    assert [c["assignedTo"] for c in r.cards[:2]] == [a["id"], a["id"]]
    r.restart_all()
    assert all(c["assignedTo"] is None for c in r.cards)
    assert not [k for k in r.meta.keys() if k.startswith("pos:")]
    r.delete_card("seed:t1")
    assert len(r.cards) == 11
    r.hard_reset("playtest")
    assert [c["id"] for c in r.cards] == ["seed:jessica"] and r.centroids == []
    assert r.meta.get("mode") == "playtest" and r.meta.get("iteration") == 0


def test_iteration_snapshot_and_dashboard():
    r = make_room()
    r.populate_test_data()
    a, b, c = (r.add_centroid(n) for n in ("A", "B", "C"))
    for cid in ("seed:t1", "seed:t5", "seed:t8"):
        r.drop_card(cid, a["id"], 0.5, 0.5)
    for cid in ("seed:jessica", "seed:t2"):
        r.drop_card(cid, b["id"], 0.5, 0.5)
    for cid in ("seed:t7", "seed:t9"):
        r.drop_card(cid, c["id"], 0.5, 0.5)
    r.set_iteration(1)
    prev = r.meta.get("prevSnapshot")
    assert prev["balance"] == {"max": 3, "min": 2, "gap": 1, "ratio": 1.5}
    r.drop_card("seed:t11", a["id"], 0.5, 0.5)
    d = r.dashboard()
    assert d["chips"] == ["k = 3", "balance gap = 2", "avg cohesion = 91%", "unassigned = 4"]
    assert d["deltas"] == [" (↓ looser 1)", " (-8pp)"]
    row = d["rows"][0]
    assert row["name"] == "A: 4" and row["bar_pct"] == 33 and row["cohesion"] == "cohesion = 75%"
    assert row["cohesion_delta"] == " (-25pp)"
    assert row["top"] == "Top: Creamy (2), Sweet (2), Colorful (1)"
    assert row["suggested"] == "Suggested: Creamy + Sweet"
    r.apply_suggested_name(a["id"], row["suggestion"])
    assert r.centroids[0]["name"] == "Creamy + Sweet"


def test_ordered_meta_keeps_slot():
    m = OrderedMeta()
    m.set("mode", "learn")
    m.set("iteration", 0)
    m.set("pos:x", {"x": 1})
    m.delete("mode")
    m.set("z", 1)
    m.set("mode", "custom")
    assert m.keys() == ["mode", "iteration", "pos:x", "z"]


def test_export_import_roundtrip():
    r = make_room()
    r.populate_test_data()
    a = r.add_centroid("A")
    r.drop_card("seed:t1", a["id"], 0.25, 0.5)
    r.set_mode("custom")
    r.set_iteration(2)
    text = r.export_json()
    assert not text.endswith("\n") and text.startswith('{\n  "cards": [\n    {\n      "id": "seed:jessica"')
    assert r.export_filename == "kmeans-room-ABCD.json"
    r2 = Room.from_json(text, "WXYZ")
    assert r2.export_json() == text
    # meta is merged: keys not in the file survive
    r3 = make_room()
    r3.meta.set("pos:old", {"x": 0.5, "y": 0.5})
    r3.import_json(text)
    assert r3.meta.get("pos:old") == {"x": 0.5, "y": 0.5}
    # absent fields: kept by default, cleared in reference-compat mode
    r4 = make_room()
    r4.import_json('{"meta": {"mode": "learn"}}')
    assert len(r4.cards) == 1
    r4.import_json('{"meta": {"mode": "learn"}}', compat=True)
    assert r4.cards == [] and r4.centroids == []


@pytest.mark.skipif(NODE is None, reason="node not installed")
def test_export_is_byte_identical_to_json_stringify():
    r = make_room()
    r.populate_test_data()
    a = r.add_centroid("Sweet • Creamy")
    r.drop_card("seed:t1", a["id"], 1 / 3, 0.5)
    r.set_iteration(1)
    text = r.export_json()
    js = "process.stdout.write(JSON.stringify(INPUT, null, 2))"
    assert run_js(js, json.loads(text)) == text


def test_auto_assign_clusters_traits():
    r = make_room()
    r.populate_test_data()
    a, b, c = (r.add_centroid(n) for n in ("A", "B", "C"))
    d = r.auto_assign(seed=0)
    counts = [int(x["name"].split(": ")[1]) for x in d["rows"]]
    assert sum(counts) == 12 and min(counts) >= 1
    # locked centroids keep their members and take no new cards
    members = [x["id"] for x in r.cards if x["assignedTo"] == a["id"]]
    r.toggle_lock(a["id"])
    r.auto_assign(seed=1)
    assert sorted(x["id"] for x in r.cards if x["assignedTo"] == a["id"]) == sorted(members)
    assert jsjson.parse(r.export_json())["centroids"][0]["locked"] is True


class _Scripted:
    """Stands in for Math.random(): returns the scripted values in order."""

    def __init__(self, vals):
        self.vals = list(vals)

    def random(self):
        return self.vals.pop(0)


def test_top_control_utilities():
    # app.mjs:239-260: copy link, coin, d12, shuffled title order (board unchanged)
    r = make_room()
    assert r.share_link("https://x.test/k/") == "https://x.test/k/?room=ABCD"
    assert r.share_link("https://x.test/k/?v=2") == "https://x.test/k/?v=2&room=ABCD"
    r.populate_test_data()
    before = [c["id"] for c in r.cards]
    r.rng = _Scripted([0.49999, 0.5, 0.0, 0.999999])
    assert (r.coin(), r.coin()) == ("Heads", "Tails")
    assert (r.d12(), r.d12()) == (1, 12)
    titles = [c["title"] for c in r.cards]
    n = len(titles)
    # j = floor(u * (i + 1)) with u = 0 for every i: each position swaps with index 0
    r.rng = _Scripted([0.0] * (n - 1))
    exp = list(titles)
    for i in range(n - 1, 0, -1):
        exp[i], exp[0] = exp[0], exp[i]
    assert r.shuffled_titles() == exp
    assert sorted(exp) == sorted(titles) and [c["id"] for c in r.cards] == before


def test_cli_room_utilities(tmp_path, capsys):
    from mikmeans import cli

    assert cli.main(["room", "--room", "WXYZ", "--populate", "--link", "https://h/p", "--coin", "--d12",
                     "--shuffle-names"]) == 0
    out = capsys.readouterr().out.splitlines()
    assert out[0] == "https://h/p?room=WXYZ"
    assert out[1] in ("Heads", "Tails")
    assert re.fullmatch(r"d12 → ([1-9]|1[0-2])", out[2])
    assert out[3] == "Suggested order:"


def test_hard_reset_keeps_current_mode_and_runs_iteration_hook():
    """hardReset writes the mode selector's value (app.mjs:231) and, when the iteration
    was nonzero, the observer snapshots the fresh board (app.mjs:230, :498-505)."""
    r = make_room()
    r.populate_test_data()
    a = r.add_centroid("A")
    r.drop_card("seed:t1", a["id"], 0.5, 0.5)
    r.set_mode("custom")
    r.set_iteration(3)
    r.hard_reset()
    assert r.meta.get("mode") == "custom" and r.meta.get("iteration") == 0
    snap = r.meta.get("prevSnapshot")
    assert snap == r.snapshot_metrics() and snap["counts"] == {}
    # from iteration 0 the key stays deleted (no change -> no snapshot)
    r.hard_reset()
    assert r.meta.get("prevSnapshot") is None and "prevSnapshot" not in r.meta
    # a mode outside the select's options leaves the select blank -> "learn"
    r.set_mode("weird")
    r.hard_reset()
    assert r.meta.get("mode") == "learn"
    text = r.export_json()
    assert '"prevSnapshot"' not in text


def test_import_with_new_iteration_overwrites_prev_snapshot():
    """After an import that changes ``iteration`` the reference's observer replaces the
    imported prevSnapshot with the imported board's metrics, before dedupeSeeds."""
    src = make_room()
    src.populate_test_data()
    a = src.add_centroid("A")
    src.drop_card("seed:t1", a["id"], 0.5, 0.5)
    src.set_iteration(5)
    src.drop_card("seed:t2", a["id"], 0.5, 0.5)   # board differs from the stored snapshot
    obj = src.export_obj()
    obj = {**obj, "cards": obj["cards"] + [dict(obj["cards"][1])]}   # a duplicate seed card
    text = jsjson.stringify(obj, 2)
    r = make_room()
    r.set_iteration(2)
    r.import_json(text)
    snap = r.meta.get("prevSnapshot")
    assert snap != src.meta.get("prevSnapshot")
    # the snapshot saw the duplicate seed card (pre-dedupe: t1, t2 and t1 again); the board
    # itself is deduplicated afterwards
    assert snap["counts"] == {a["id"]: 3} and r._last_iter == 5
    assert len(r.cards) == len(src.cards) and r.snapshot_metrics()["counts"] == {a["id"]: 2}
    # same iteration -> the imported snapshot is kept
    r2 = make_room()
    r2.set_iteration(5)
    r2.import_json(src.export_json())
    assert r2.meta.get("prevSnapshot") == src.meta.get("prevSnapshot")
