"""Property-based tests (hypothesis, CPU): invariants the example tests pin only at points.

- the order-free inertia slots (csrc/common.h ``slot_add`` / ``slot_decode``): a Python mirror
  of the digit encoding -- any order of the same contributions gives the same words, and the
  decoded total is the exact 2^-64 fixed-point sum (``mikmeans.ops.native.slot_totals`` decodes
  the device's words the same way);
- ECMAScript number formatting: the Python formatter round-trips every finite double and
  equals the C++ one bit for bit;
- row sharding: the shards partition [0, n), are balanced to one alignment unit and start on
  the alignment grid (so near-tie resolution is the same on any world size);
- the CPU assign: the chosen centre is the nearest one up to the float32 score rounding.
"""
import math
from fractions import Fraction

import numpy as np
import pytest
import torch

hyp = pytest.importorskip("hypothesis")
from hypothesis import given, settings, strategies as st  # noqa: E402

from mikmeans import ops  # noqa: E402
from mikmeans.ops import native  # noqa: E402
from mikmeans.parallel.shard import ROW_ALIGN, shard_range  # noqa: E402
from mikmeans.utils import jsjson  # noqa: E402

M64 = (1 << 64) - 1
SLOT_OVF = native.SLOT_OVF


def _slot_add(w: list[int], v: float, cnt: int = 0):
    """Python mirror of csrc/common.h slot_add (uint64 words, wrapping adds)."""
    if cnt:
        w[7] = (w[7] + cnt) & M64
    if v == 0.0:
        return
    bits = int(np.float64(v).view(np.uint64))
    neg = bits >> 63
    ex = (bits >> 52) & 0x7FF
    if ex == 0x7FF:
        w[6] = (w[6] + SLOT_OVF) & M64
        return
    m = (bits & ((1 << 52) - 1)) | ((1 << 52) if ex else 0)
    s = (ex if ex else 1) - 1075 + 64
    if s < 0:
        m = 0 if -s >= 64 else m >> -s
        s = 0
    j0, o = s >> 5, s & 31
    if j0 > 4:
        w[6] = (w[6] + SLOT_OVF) & M64
        return
    lo = (m << o) & M64
    hi = (m >> (64 - o)) if o else 0
    for i, d in enumerate((lo & 0xFFFFFFFF, lo >> 32, hi)):
        if d:
            w[j0 + i] = (w[j0 + i] + ((-d) & M64 if neg else d)) & M64


def _decode(w: list[int]) -> float:
    t = torch.tensor([x - (1 << 64) if x >= (1 << 63) else x for x in w], dtype=torch.int64)
    return native.slot_totals(t.view(torch.float64))[0]


finite_pos = st.floats(min_value=0.0, max_value=2.0**90, allow_nan=False, allow_infinity=False)


@settings(max_examples=200, deadline=None)
@given(st.lists(finite_pos, min_size=1, max_size=40), st.randoms(use_true_random=False))
def test_slots_are_order_free_and_exact(vals, rnd):
    a = [0] * 8
    for v in vals:
        _slot_add(a, v, 1)
    b = [0] * 8
    perm = list(vals)
    rnd.shuffle(perm)
    for v in perm:
        _slot_add(b, v, 1)
    assert a == b                                  # integer words: any order, same bits
    exact = sum(Fraction(v) for v in vals)
    trunc = sum(Fraction(math.floor(Fraction(v) * 2**64), 2**64) for v in vals)   # digits below 2^-64 dropped
    got = _decode(a)
    assert a[7] == len(vals)
    assert got == float(trunc) or abs(Fraction(got) - trunc) <= abs(trunc) * Fraction(1, 2**52)
    assert abs(Fraction(got) - exact) <= len(vals) * Fraction(1, 2**64) + abs(exact) * Fraction(1, 2**52)


def test_slots_overflow_flag():
    w = [0] * 8
    _slot_add(w, float("inf"))
    assert math.isinf(_decode(w))
    w = [0] * 8
    _slot_add(w, 2.0**200)
    assert math.isinf(_decode(w))


doubles = st.floats(allow_nan=False, allow_infinity=False, width=64)


@settings(max_examples=500, deadline=None)
@given(doubles)
def test_js_number_round_trips(x):
    s = jsjson.js_number(x)
    assert float(s) == x or (x == 0 and s == "0")
    a = abs(x)
    if a != 0 and 1e-6 <= a < 1e21:
        assert "e" not in s                       # plain notation in ECMAScript's window
    elif a != 0:
        assert "e" in s


@pytest.mark.skipif(not native.available(), reason="native extension not built")
@settings(max_examples=500, deadline=None)
@given(doubles)
def test_js_number_python_equals_native(x):
    assert jsjson.js_number(x) == native.require().js_format(x)


@settings(max_examples=300, deadline=None)
@given(st.integers(min_value=0, max_value=10**10), st.integers(min_value=1, max_value=64),
       st.sampled_from([1, 64, 256, ROW_ALIGN]))
def test_shards_partition_rows(n, world, align):
    spans = [shard_range(n, r, world, align) for r in range(world)]
    assert spans[0][0] == 0 and spans[-1][1] == n
    for (a0, a1), (b0, b1) in zip(spans, spans[1:]):
        assert a1 == b0 and a0 <= a1
    for s0, s1 in spans:
        assert s0 % align == 0 or s0 == n
    units = [-(-(s1 - s0) // align) for s0, s1 in spans]
    assert max(units) - min(units) <= 1


@settings(max_examples=60, deadline=None)
@given(st.integers(min_value=1, max_value=200), st.integers(min_value=1, max_value=12),
       st.integers(min_value=1, max_value=24), st.integers(min_value=0, max_value=2**31 - 1))
def test_cpu_assign_picks_a_nearest_centre(n, d, k, seed):
    g = torch.Generator().manual_seed(seed)
    X = torch.randn(n, d, generator=g) * 3
    C = torch.randn(k, d, generator=g) * 3
    lab, mind = ops.assign(X, C)
    D2 = ((X.double()[:, None, :] - C.double()[None, :, :]) ** 2).sum(-1)
    best = D2.min(1).values
    chosen = D2.gather(1, lab.long()[:, None])[:, 0]
    # float32 scores |c|^2 - 2 x.c: ties within their rounding may go either way
    slack = 1e-5 * (X.double().pow(2).sum(1) + C.double().pow(2).sum(1).max() + 1.0)
    assert bool((chosen <= best + slack).all())
    assert bool(((mind.double() - chosen).abs() <= slack + 1e-4 * chosen).all())


# -------------------------------------------------------------- the room model
_ops = st.lists(st.one_of(
    st.tuples(st.just("add_centroid"), st.sampled_from(["Sweet", "Fresh", "  Bold  ", ""])),
    st.tuples(st.just("add_card"), st.sampled_from(["Mango", "Lime", "Chili"]),
              st.lists(st.sampled_from(["sweet", "sour", "hot", "crisp"]), max_size=3)),
    st.tuples(st.just("assign"), st.integers(0, 9), st.integers(-1, 3)),
    st.tuples(st.just("drop"), st.integers(0, 9), st.integers(0, 3),
              st.floats(-2, 3, allow_nan=False), st.floats(-2, 3, allow_nan=False)),
    st.tuples(st.just("lock"), st.integers(0, 3)),
    st.tuples(st.just("rename"), st.integers(0, 3), st.sampled_from(["Tart", " ", "Zing"])),
    st.tuples(st.just("remove_centroid"), st.integers(0, 3)),
    st.tuples(st.just("delete_card"), st.integers(0, 9)),
    st.tuples(st.just("shuffle"),),
    st.tuples(st.just("restart"),),
), max_size=40)


@settings(max_examples=150, deadline=None)
@given(_ops)
def test_room_invariants_and_export_round_trip(ops_seq):
    """Any sequence of board operations keeps the room consistent -- at most max_centroids,
    every assignment names a live centroid, a position only for an assigned card and inside
    the drop clamps -- and its export re-imports to the same export, byte for byte."""
    from mikmeans.models.room import Room

    room = Room("PROP1", seed=3)

    def card(i):
        return room.cards[i % len(room.cards)]["id"] if room.cards else "none"

    def cent(i):
        return room.centroids[i % len(room.centroids)]["id"] if room.centroids else "none"

    for op in ops_seq:
        kind = op[0]
        if kind == "add_centroid":
            room.add_centroid(op[1] or None)
        elif kind == "add_card":
            room.add_card(op[1], op[2])
        elif kind == "assign":
            room.update_card_assign(card(op[1]), None if op[2] < 0 else cent(op[2]))
        elif kind == "drop":
            room.drop_card(card(op[1]), cent(op[2]), op[3], op[4])
        elif kind == "lock":
            room.toggle_lock(cent(op[1]))
        elif kind == "rename":
            room.rename_centroid(cent(op[1]), op[2])
        elif kind == "remove_centroid":
            room.remove_centroid(cent(op[1]))
        elif kind == "delete_card":
            room.delete_card(card(op[1]))
        elif kind == "shuffle":
            room.shuffle_unassigned()
        else:
            room.restart_all()
    assert len(room.centroids) <= room.max_centroids
    live = {c["id"] for c in room.centroids}
    assigned = {c["id"] for c in room.cards if c.get("assignedTo")}
    assert all(c.get("assignedTo") in live for c in room.cards if c.get("assignedTo"))
    for k, v in room.meta.items():
        if str(k).startswith("pos:"):
            assert k[4:] in assigned
            assert 0.02 <= v["x"] <= 0.92 and 0.10 <= v["y"] <= 0.92
    exp = room.export_json()
    assert Room.from_json(exp, "PROP1", seed=3).export_json() == exp
    room.dashboard()    # (computable on any reachable board)
