"""Trait tokenisation and trait-cluster analytics, exact parity with the reference.

Re-implements (not translates) the semantics of the reference's dashboard
analytics:

* :func:`norm_tokens`     normTokens   app.mjs:436-443
* :func:`title_case`      titleCase    app.mjs:444
* :func:`tokens_for_card` tokensForCard app.mjs:445-449
* :func:`trait_counts`    traitCountsFor app.mjs:450-461
* :func:`cohesion`        cohesionFor  app.mjs:462-475 (plus the O(n) count rule)
* :func:`suggestion`      suggestionFromCounts app.mjs:476-480
* :func:`top_traits`      "Top:" list  app.mjs:549
* :func:`snapshot_metrics` snapshotMetrics app.mjs:481-496

and bridges them to numeric k-means: :func:`encode_traits` turns cards into
multi-hot vectors, so ``count_t = n_k * centroid_k[t]`` and the suggested name of
a cluster is the two largest coordinates of its centroid.
"""
from __future__ import annotations

import re
import unicodedata

import numpy as np

# ECMAScript WhiteSpace + LineTerminator (the \s class and String.prototype.trim)
JS_WS = "\t\n\v\f\r \u00a0\u1680\u2000-\u200a\u2028\u2029\u202f\u205f\u3000\ufeff"
_SPLIT = re.compile(rf"[/,&•+]|(?:[{JS_WS}]+and[{JS_WS}]+)|\||,", re.IGNORECASE)
_WORD = re.compile(rf"[A-Za-z0-9_][^{JS_WS}]*")
_TRIM = re.compile(rf"^[{JS_WS}]+|[{JS_WS}]+$")


def js_trim(s: str) -> str:
    return _TRIM.sub("", s)


def norm_tokens(s) -> list[str]:
    """Split a trait string into lower-case tokens (no whitespace splitting)."""
    if not s:
        return []
    parts = (js_trim(p) for p in _SPLIT.split(str(s)))
    return [p.lower() for p in parts if p]


def title_case(s: str) -> str:
    """Upper-case the first (ASCII word) character of every ``\\w\\S*`` run."""
    return _WORD.sub(lambda m: m.group(0)[0].upper() + m.group(0)[1:], s)


def _traits(card) -> list:
    t = card.get("traits") if isinstance(card, dict) else getattr(card, "traits", None)
    return list(t) if t else []


def tokens_for_card(card) -> list[str]:
    """Ordered set of both traits' tokens (no double counting within a card)."""
    tr = _traits(card)
    a = norm_tokens(tr[0] if len(tr) > 0 else None)
    b = norm_tokens(tr[1] if len(tr) > 1 else None)
    return list(dict.fromkeys(a + b))


def trait_counts(cards) -> dict[str, dict]:
    """token -> {"label": titleCase(token), "count": #cards containing it}, insertion-ordered."""
    out: dict[str, dict] = {}
    for c in cards:
        for t in tokens_for_card(c):
            e = out.setdefault(t, {"label": title_case(t), "count": 0})
            e["count"] += 1
    return out


def cohesion(cards) -> float:
    """Share of members sharing >= 1 token with another member (1 for n <= 1)."""
    n = len(cards)
    if n <= 1:
        return 1
    sets = [set(tokens_for_card(c)) for c in cards]
    share = 0
    for i in range(n):
        if any(i != j and sets[i] & sets[j] for j in range(n)):
            share += 1
    return share / n


def cohesion_from_counts(cards, counts: dict | None = None) -> float:
    """O(n) equivalent: member i counts iff one of its tokens has count >= 2 in the cluster."""
    n = len(cards)
    if n <= 1:
        return 1
    counts = counts if counts is not None else trait_counts(cards)
    share = sum(1 for c in cards if any(counts[t]["count"] >= 2 for t in tokens_for_card(c)))
    return share / n


# ---------------------------------------------------------------- localeCompare
def _collation_key(s: str):
    """Approximation of ICU root collation (what ``String.prototype.localeCompare`` uses
    in a full-ICU JavaScript engine) for Latin text: primary = base letters ignoring
    case and accents, with spaces/punctuation < digits < letters; secondary = accents;
    tertiary = lower case before upper case."""
    prim, sec, ter = [], [], []
    for ch in s:
        d = unicodedata.normalize("NFD", ch)
        base = d[0]
        marks = d[1:]
        if base.isalpha():
            cls = 2
        elif base.isdigit():
            cls = 1
        else:
            cls = 0
        prim.append((cls, base.casefold()))
        sec.append(marks)
        ter.append(0 if base == base.lower() else 1)
    return (prim, sec, ter)


def locale_compare(a: str, b: str) -> int:
    ka, kb = _collation_key(a), _collation_key(b)
    return (ka > kb) - (ka < kb)


def _sorted_entries(counts: dict) -> list[dict]:
    import functools

    def cmp(x, y):
        return (y["count"] - x["count"]) or locale_compare(x["label"], y["label"])

    return sorted(counts.values(), key=functools.cmp_to_key(cmp))


def suggestion(counts: dict):
    """``"A + B"`` from the top-2 tokens (count desc, then localeCompare), ``"A"``, or ``None``."""
    arr = _sorted_entries(counts)
    if not arr:
        return None
    return f"{arr[0]['label']} + {arr[1]['label']}" if len(arr) > 1 else arr[0]["label"]


def top_traits(counts: dict, k: int = 3) -> list[dict]:
    return _sorted_entries(counts)[:k]


def top_text(counts: dict) -> str:
    top = top_traits(counts)
    return "Top: " + ", ".join(f"{t['label']} ({t['count']})" for t in top) if top else "Top: —"


def snapshot_metrics(cards, centroids) -> dict:
    """``{counts, cohesion, balance, avgCohesion}`` keyed by centroid id."""
    from .metrics import balance

    counts, coh = {}, {}
    for c in centroids:
        cid = c["id"]
        cs = [x for x in cards if x.get("assignedTo") == cid]
        counts[cid] = len(cs)
        coh[cid] = cohesion(cs)
    vals = list(coh.values())
    avg = sum(vals) / len(vals) if vals else 1
    return {"counts": counts, "cohesion": coh, "balance": balance(list(counts.values())), "avgCohesion": avg}


# ------------------------------------------------------------ numeric bridge
def build_vocab(cards) -> list[str]:
    vocab: dict[str, None] = {}
    for c in cards:
        for t in tokens_for_card(c):
            vocab.setdefault(t, None)
    return list(vocab)


def encode_traits(cards, vocab: list[str] | None = None) -> tuple[np.ndarray, list[str]]:
    """Multi-hot float32 matrix ``[n_cards, |vocab|]`` (1 where the card has the token)."""
    vocab = vocab if vocab is not None else build_vocab(cards)
    index = {t: i for i, t in enumerate(vocab)}
    X = np.zeros((len(cards), len(vocab)), dtype=np.float32)
    for r, c in enumerate(cards):
        for t in tokens_for_card(c):
            if t in index:
                X[r, index[t]] = 1.0
    return X, vocab


def counts_from_centroid(centroid: np.ndarray, n_members: int, vocab: list[str]) -> dict:
    """Recover ``traitCountsFor`` of a cluster from its multi-hot mean (count = n * c_t)."""
    out = {}
    for t, v in zip(vocab, np.asarray(centroid, dtype=np.float64)):
        cnt = int(round(float(v) * n_members))
        if cnt > 0:
            out[t] = {"label": title_case(t), "count": cnt}
    return out


def label_clusters(centroids: np.ndarray, counts, vocab: list[str]) -> list:
    """Suggested name of every cluster from its centroid (top-2 coordinates)."""
    return [suggestion(counts_from_centroid(c, int(n), vocab)) for c, n in zip(centroids, counts)]
