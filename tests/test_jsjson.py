"""Byte-exact JSON.stringify emulation and flat-float centroid JSON."""
import json
import math
import random
import struct

import numpy as np
import pytest
import torch

from mikmeans.ops import native
from mikmeans.utils import jsjson

from .jsnode import NODE, run_js

B2 = [(1.0, "1"), (-0.0, "0"), (1e-7, "1e-7"), (1e-6, "0.000001"), (1e16, "10000000000000000"),
      (1e21, "1e+21"), (float("nan"), "null"), (float("inf"), "null"), (float("-inf"), "null"),
      (float(np.float32(0.1)), "0.10000000149011612"), (123.456, "123.456"), (-2.5e-8, "-2.5e-8"),
      (5e-324, "5e-324"), (1.7976931348623157e308, "1.7976931348623157e+308"), (0.5, "0.5"),
      (123456789012345680000.0, "123456789012345680000"), (1.5e21, "1.5e+21"), (100.0, "100")]


@pytest.mark.parametrize("v,exp", B2)
def test_js_number_table(v, exp):
    assert jsjson.js_number(v) == exp


@pytest.mark.parametrize("v,exp", B2)
def test_native_formatter_matches(v, exp):
    if not native.available():
        pytest.skip("native extension not built")
    assert native.require().js_format(v) == exp


def _random_doubles(n, seed=0):
    rng = random.Random(seed)
    out = []
    for _ in range(n):
        k = rng.random()
        if k < 0.3:
            out.append(struct.unpack("<d", struct.pack("<Q", rng.getrandbits(64)))[0])
        elif k < 0.6:
            out.append(float(np.float32(rng.uniform(-1e3, 1e3))))
        elif k < 0.8:
            out.append(rng.uniform(-1, 1) * 10 ** rng.randint(-30, 30))
        else:
            out.append(float(rng.randint(-10**6, 10**6)))
    return [x for x in out if math.isfinite(x)]


def test_python_and_native_agree_on_random_doubles():
    if not native.available():
        pytest.skip("native extension not built")
    C = native.require()
    for x in _random_doubles(20000, 1):
        assert jsjson.js_number(x) == C.js_format(x), x


@pytest.mark.skipif(NODE is None, reason="node not installed")
def test_numbers_match_node():
    xs = _random_doubles(3000, 2)
    got = [jsjson.js_number(x) for x in xs]
    # feed exact bit patterns to node via hex so no formatting happens on the way in
    hexes = [struct.pack(">d", x).hex() for x in xs]
    js = """
      const out = INPUT.map(h => { const b = Buffer.from(h, 'hex'); return JSON.stringify(b.readDoubleBE(0)); });
      console.log(JSON.stringify(out));
    """
    assert json.loads(run_js(js, hexes)) == got


@pytest.mark.skipif(NODE is None, reason="node not installed")
def test_stringify_matches_node_on_structures():
    rng = random.Random(7)

    def rand_str():
        alphabet = ['a', 'B', ' ', '"', '\\', '\n', '\t', '\x01', '\x1f', 'é', '•', '🍦', ' ', '/', '<']
        return "".join(rng.choice(alphabet) for _ in range(rng.randint(0, 8)))

    def rand_val(depth=0):
        k = rng.random()
        if depth > 3 or k < 0.4:
            return rng.choice([None, True, False, rng.randint(-1000, 1000), rng.uniform(-1e6, 1e6),
                               float(np.float32(rng.random())), rand_str()])
        if k < 0.7:
            return [rand_val(depth + 1) for _ in range(rng.randint(0, 4))]
        d = {}
        for _ in range(rng.randint(0, 4)):
            key = rng.choice(["id", "name", "2", "10", "0", "x", "pos:seed:t1", rand_str()])
            d[key] = rand_val(depth + 1)
        return d

    vals = [rand_val() for _ in range(200)]
    for indent in (None, 2):
        # node receives the value via JSON.parse of Python's (lossless) encoding
        js = f"console.log(JSON.stringify(INPUT.map(v => JSON.stringify(v, null, {json.dumps(indent)}))))"
        exp = json.loads(run_js(js, vals))
        got = [jsjson.stringify(v, indent) for v in vals]
        assert got == exp


def test_array_index_keys_first():
    assert jsjson.stringify({"b": 1, "2": 2, "a": 3, "1": 4, "01": 5}) == '{"1":4,"2":2,"b":1,"a":3,"01":5}'


def test_flat_centroid_json_roundtrip():
    C = torch.tensor([[0.5, -1.25, 0.1], [1e-8, 3.0, -0.0]], dtype=torch.float32)
    s = jsjson.centroids_to_json(C)
    assert s == "[0.5,-1.25,0.10000000149011612,9.99999993922529e-9,3,0]"
    back = jsjson.centroids_from_json(s, 3)
    assert np.array_equal(back, C.numpy())
