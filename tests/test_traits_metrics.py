"""Trait analytics + dashboard metrics parity (SURVEY.md Appendix A golden values)."""
import json
import math
import random

import numpy as np
import pytest

from mikmeans.data.cards import demo_cards
from mikmeans.utils import metrics as mm
from mikmeans.utils import traits as tr

from .jsnode import NODE, run_js

TOKEN_CASES = [
    ("Mint/Choc", ["mint", "choc"]),
    ("Salt & Pepper", ["salt", "pepper"]),
    ("Nuts and Honey", ["nuts", "honey"]),
    ("Band", ["band"]),
    ("x • y", ["x", "y"]),
    ("Fresh,,Sorbet", ["fresh", "sorbet"]),
    ("  ", []),
    ("Not Sweet", ["not sweet"]),
    ("", []),
    (None, []),
    ("A AND B", ["a", "b"]),
    ("sand and hand", ["sand", "hand"]),
    ("a|b+c", ["a", "b", "c"]),
]


@pytest.mark.parametrize("s,exp", TOKEN_CASES)
def test_norm_tokens(s, exp):
    assert tr.norm_tokens(s) == exp


def test_title_case():
    assert tr.title_case("à la mode") == "à La Mode"
    assert tr.title_case("not sweet") == "Not Sweet"
    assert tr.title_case("creamy") == "Creamy"
    assert tr.title_case("9lives _x") == "9lives _x"


# Appendix A.5 clustering rows (computed with the reference's own functions)
ROW1 = {"c1": ["seed:t1", "seed:t5", "seed:t8", "seed:t11"],
        "c2": ["seed:jessica", "seed:t2", "seed:t3", "seed:t6"],
        "c3": ["seed:t7", "seed:t9", "seed:t4", "seed:t10"]}
ROW2 = {"c1": ["seed:t1", "seed:t5", "seed:t8"], "c2": ["seed:jessica", "seed:t2"], "c3": ["seed:t7", "seed:t9"]}


def _assigned(row):
    return demo_cards({cid: c for c, ids in row.items() for cid in ids})


CENTROIDS = [{"id": "c1", "name": "A", "color": "#6EE7B7", "locked": False},
             {"id": "c2", "name": "B", "color": "#93C5FD", "locked": False},
             {"id": "c3", "name": "C", "color": "#FBCFE8", "locked": False}]


def test_golden_row1():
    cards = _assigned(ROW1)
    snap = tr.snapshot_metrics(cards, CENTROIDS)
    assert snap["counts"] == {"c1": 4, "c2": 4, "c3": 4}
    assert snap["cohesion"] == {"c1": 0.75, "c2": 0.5, "c3": 0.5}
    assert snap["balance"] == {"max": 4, "min": 4, "gap": 0, "ratio": 1}
    assert snap["avgCohesion"] == 0.5833333333333334
    sug = [tr.suggestion(tr.trait_counts([c for c in cards if c["assignedTo"] == k])) for k in ("c1", "c2", "c3")]
    assert sug == ["Creamy + Sweet", "Fresh + Sorbet", "Rich + Bitter"]
    tops = [[(t["label"], t["count"]) for t in tr.top_traits(tr.trait_counts(
        [c for c in cards if c["assignedTo"] == k]))] for k in ("c1", "c2", "c3")]
    assert tops == [[("Creamy", 2), ("Sweet", 2), ("Colorful", 1)],
                    [("Fresh", 2), ("Sorbet", 2), ("Chocolatey", 1)],
                    [("Rich", 2), ("Bitter", 1), ("Espresso", 1)]]


def test_golden_row2_and_empty():
    snap = tr.snapshot_metrics(_assigned(ROW2), CENTROIDS)
    assert snap["counts"] == {"c1": 3, "c2": 2, "c3": 2}
    assert snap["cohesion"] == {"c1": 1, "c2": 1, "c3": 1}
    assert snap["balance"] == {"max": 3, "min": 2, "gap": 1, "ratio": 1.5}
    assert snap["avgCohesion"] == 1
    empty = tr.snapshot_metrics(demo_cards(), CENTROIDS[:1])
    assert empty["counts"] == {"c1": 0} and empty["cohesion"] == {"c1": 1}
    assert empty["balance"] == {"max": 0, "min": 0, "gap": 0, "ratio": 1}
    none = tr.snapshot_metrics(demo_cards(), [])
    assert none["avgCohesion"] == 1 and none["balance"]["ratio"] == 1


def test_balance_ratio_rules():
    assert mm.balance([3, 0])["ratio"] == math.inf
    assert mm.balance([0, 0])["ratio"] == 1
    assert mm.balance([])["max"] == 0
    assert mm.balance([6, 3])["ratio"] == 2


def test_cohesion_count_rule_matches_pairwise():
    rng = random.Random(0)
    vocab = ["sweet", "creamy", "rich", "nutty", "fresh", "bitter", "salt", "mint"]
    for _ in range(2000):
        n = rng.randint(0, 7)
        cards = [{"traits": [rng.choice(vocab + [""]), " & ".join(rng.sample(vocab, rng.randint(0, 2)))]}
                 for _ in range(n)]
        assert tr.cohesion(cards) == tr.cohesion_from_counts(cards)


def test_js_display_rounding():
    assert mm.avg_cohesion_pct(0.5833333333333334) == 58       # (x*100|0)
    assert mm.cohesion_pct(0.125) == 13                          # Math.round(12.5) = 13
    assert mm.js_round(-2.5) == -2                               # Math.round(-2.5) = -2
    assert mm.bar_pct(1, 3) == 33 and mm.bar_pct(0, 0) == 0
    assert mm.delta_gap_text(1, 3) == " (↑ tighter 2)"
    assert mm.delta_gap_text(3, 1) == " (↓ looser 2)"
    assert mm.delta_pp_text(0.5, 0.5) == " (±0)"
    assert mm.delta_pp_text(0.75, 0.5) == " (+25pp)"
    assert mm.delta_pp_text(0.5, 0.75) == " (-25pp)"


def test_multi_hot_bridge_suggestion_equals_top2_coordinates():
    cards = _assigned(ROW1)
    X, vocab = tr.encode_traits(cards)
    assert X.shape == (12, len(vocab)) and set(np.unique(X)) <= {0.0, 1.0}
    for k, exp in zip(("c1", "c2", "c3"), ["Creamy + Sweet", "Fresh + Sorbet", "Rich + Bitter"]):
        idx = [i for i, c in enumerate(cards) if c["assignedTo"] == k]
        centroid = X[idx].mean(0)
        assert tr.label_clusters(centroid[None], [len(idx)], vocab) == [exp]
        assert tr.counts_from_centroid(centroid, len(idx), vocab) == \
            {t: v for t, v in tr.trait_counts([cards[i] for i in idx]).items()}


@pytest.mark.skipif(NODE is None, reason="node not installed")
def test_tokenizer_matches_javascript_regex():
    # the split regex and titleCase regex exactly as documented in SURVEY.md Appendix A.1
    inputs = [s for s, _ in TOKEN_CASES if s] + ["Vanilla and Fudge", "ÉCLAIR / crème", "a\tand\tb",
                                                 "x　and　y", "  trim me  ", "one,two&three•four+five|six"]
    js = r"""
      const split = s => String(s).split(/[/,&•+]|(?:\s+and\s+)|\||,/gi).map(x => x.trim()).filter(Boolean).map(x => x.toLowerCase());
      const tc = s => s.replace(/\w\S*/g, w => w[0].toUpperCase() + w.slice(1));
      console.log(JSON.stringify(INPUT.map(s => [split(s), tc(s.toLowerCase())])));
    """
    out = json.loads(run_js(js, inputs))
    for s, (toks, title) in zip(inputs, out):
        assert tr.norm_tokens(s) == toks, s
        assert tr.title_case(s.lower()) == title, s


@pytest.mark.skipif(NODE is None, reason="node not installed")
def test_locale_compare_matches_javascript():
    words = ["Sweet", "sweet", "Creamy", "creamy", "Éclair", "Eclair", "apple", "Banana", "banana split",
             "Not Sweet", "Nutty", "Rich", "rich", "Zest", "9 Lives", "_x", "x-ray", "X Ray", "Ørange", "Ice"]
    js = "console.log(JSON.stringify(INPUT.map(a => INPUT.map(b => Math.sign(a.localeCompare(b))))))"
    try:
        out = json.loads(run_js(js, words))
    except RuntimeError as e:  # pragma: no cover
        pytest.skip(f"node without ICU: {e}")
    mism = [(a, b, out[i][j], tr.locale_compare(a, b)) for i, a in enumerate(words) for j, b in enumerate(words)
            if out[i][j] != tr.locale_compare(a, b)]
    # parity is exact for the letter/case/accent cases the dashboard produces
    core = [m for m in mism if not any(ch in (m[0] + m[1]) for ch in "_-Ø9")]
    assert core == [], core
