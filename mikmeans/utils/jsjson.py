"""Byte-exact ``JSON.stringify`` emulation and the flat-float centroid JSON.

The reference's only persisted artefact is the room export
``JSON.stringify({cards, centroids, meta}, null, 2)`` (app.mjs:263-267); Python's
``json`` differs on numbers (``1.0`` vs ``1``, ``1e-07`` vs ``1e-7``, ``NaN`` vs
``null``, ...) so this module re-implements the
ECMAScript algorithm: shortest round-trip digits, plain notation for
``1e-7 < |x| < 1e21``, exponent form otherwise, non-finite -> ``null``,
``-0`` -> ``0``; strings escaped exactly like ``JSON.stringify`` (control
characters as ``\\u00xx``, lone surrogates as ``\\udxxx``, everything else raw
UTF-8); ``indent`` handling identical to the spec (``[]``/``{}`` for empty
containers, ``"key": value``).

Bulk number formatting (K*D centroid floats) uses the native C++ formatter in
``mikmeans._C`` when built, with this module's Python implementation as the
always-available equivalent (tests check they agree).
"""
from __future__ import annotations

import math

import numpy as np


def js_number(x) -> str:
    """ECMAScript ``Number::toString`` as used by ``JSON.stringify``."""
    x = float(x)
    if math.isnan(x) or math.isinf(x):
        return "null"
    if x == 0:
        return "0"
    sign = "-" if x < 0 else ""
    r = repr(abs(x))  # shortest round-trip digits
    if "e" in r or "E" in r:
        mant, exp = r.lower().split("e")
        e10 = int(exp)
    else:
        mant, e10 = r, 0
    if "." in mant:
        ip, fp = mant.split(".")
    else:
        ip, fp = mant, ""
    digits = (ip + fp).lstrip("0")
    # position of the decimal point relative to the first significant digit
    lead = len(ip + fp) - len((ip + fp).lstrip("0"))
    n = len(ip) - lead + e10
    digits = digits.rstrip("0") or "0"
    k = len(digits)
    if k <= n <= 21:
        s = digits + "0" * (n - k)
    elif 0 < n <= 21:
        s = digits[:n] + "." + digits[n:]
    elif -6 < n <= 0:
        s = "0." + "0" * (-n) + digits
    else:
        ee = n - 1
        s = digits[0] + ("." + digits[1:] if k > 1 else "") + "e" + ("+" if ee >= 0 else "-") + str(abs(ee))
    return sign + s


def _quote(s: str) -> str:
    out = ['"']
    for ch in s:
        o = ord(ch)
        if ch == '"':
            out.append('\\"')
        elif ch == "\\":
            out.append("\\\\")
        elif ch == "\b":
            out.append("\\b")
        elif ch == "\f":
            out.append("\\f")
        elif ch == "\n":
            out.append("\\n")
        elif ch == "\r":
            out.append("\\r")
        elif ch == "\t":
            out.append("\\t")
        elif o < 0x20 or 0xD800 <= o <= 0xDFFF:
            out.append(f"\\u{o:04x}")
        else:
            out.append(ch)
    out.append('"')
    return "".join(out)


def _is_array_index(k: str) -> bool:
    return k.isdigit() and (k == "0" or not k.startswith("0")) and int(k) < 2**32 - 1


def js_key_order(items):
    """OrdinaryOwnPropertyKeys order: array-index keys ascending, then insertion order."""
    idx = sorted((kv for kv in items if _is_array_index(kv[0])), key=lambda kv: int(kv[0]))
    return idx + [kv for kv in items if not _is_array_index(kv[0])]


def stringify(value, indent: int | str | None = None) -> str:
    """``JSON.stringify(value, null, indent)`` for JSON-like Python values.

    dict keys keep insertion order; ``None`` -> ``null``; tuples/lists -> arrays;
    non-finite floats -> ``null``; numpy scalars/arrays are converted.
    """
    gap = " " * min(int(indent), 10) if isinstance(indent, (int, float)) else (indent or "")[:10]

    def ser(v, cur):
        if v is None:
            return "null"
        if v is True:
            return "true"
        if v is False:
            return "false"
        if isinstance(v, (int, np.integer)) and not isinstance(v, bool):
            return js_number(float(v)) if abs(int(v)) >= 2**53 else str(int(v))
        if isinstance(v, (float, np.floating)):
            return js_number(v)
        if isinstance(v, str):
            return _quote(v)
        if isinstance(v, np.ndarray):
            v = v.tolist()
        if isinstance(v, (list, tuple)):
            if not v:
                return "[]"
            if not gap:
                return "[" + ",".join(ser(e, cur) for e in v) + "]"
            inner = cur + gap
            return "[\n" + ",\n".join(inner + ser(e, inner) for e in v) + "\n" + cur + "]"
        if isinstance(v, dict):
            items = js_key_order([(str(k), e) for k, e in v.items() if not callable(e)])
            if not items:
                return "{}"
            if not gap:
                return "{" + ",".join(_quote(k) + ":" + ser(e, cur) for k, e in items) + "}"
            inner = cur + gap
            return "{\n" + ",\n".join(inner + _quote(k) + ": " + ser(e, inner) for k, e in items) + "\n" + cur + "}"
        if hasattr(v, "tolist"):
            return ser(v.tolist(), cur)
        raise TypeError(f"not JSON serialisable: {type(v).__name__}")

    return ser(value, "")


def parse(text: str):
    """``JSON.parse`` equivalent (duplicate keys: last wins, as in JS)."""
    import json

    return json.loads(text)


# ------------------------------------------------------------ flat centroids
def centroids_to_json(centers) -> str:
    """Flat JSON array of ``K*D`` numbers, row-major, each float32 widened to f64:
    exactly ``JSON.stringify(Array.from(new Float32Array(C.flat())))``."""
    import torch

    t = centers.detach().to("cpu", torch.float32).contiguous() if torch.is_tensor(centers) \
        else torch.as_tensor(np.asarray(centers, dtype=np.float32))
    try:
        from ..ops import native

        if native.available():
            return native.require().js_array(t)
    except Exception:  # pragma: no cover - formatter is optional
        pass
    return "[" + ",".join(js_number(float(v)) for v in t.reshape(-1).tolist()) + "]"


def centroids_from_json(text: str, n_features: int) -> np.ndarray:
    flat = np.asarray(parse(text), dtype=np.float32)
    if flat.size % n_features:
        raise ValueError("flat centroid array length is not a multiple of n_features")
    return flat.reshape(-1, n_features)
