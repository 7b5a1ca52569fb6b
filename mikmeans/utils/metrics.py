"""Cluster metrics with exact parity to the reference dashboard (app.mjs:435-570).

Numeric clusters: ``counts``, ``balance`` {max, min, gap, ratio} (snapshotMetrics,
app.mjs:481-496), inertia / shift from the engine.  Trait ("flavor card")
clusters additionally get ``cohesion`` (app.mjs:462-475), ``avgCohesion``,
top-3 traits (app.mjs:549) and the suggested name (app.mjs:476-480) -- see
:mod:`mikmeans.utils.traits`.  Display helpers reproduce the reference's
rounding rules (truncating ``|0`` for the average chip, ``Math.round`` for the
per-cluster chips and bars, app.mjs:520, :539, :543).
"""
from __future__ import annotations

import math


def balance(counts) -> dict:
    """``{max, min, gap, ratio}`` over per-centroid counts (app.mjs:488-492).

    ``ratio`` is ``max/min``; with ``min == 0`` it is ``Infinity`` when ``max > 0``
    and ``1`` otherwise; an empty centroid list gives max = min = gap = 0, ratio 1.
    """
    vals = list(counts)
    mx = max(vals) if vals else 0
    mn = min(vals) if vals else 0
    gap = mx - mn
    ratio = (mx / mn) if mn else (math.inf if mx else 1)
    return {"max": mx, "min": mn, "gap": gap, "ratio": ratio}


def js_round(x: float) -> int:
    """JavaScript ``Math.round`` (half rounds toward +infinity)."""
    return math.floor(x + 0.5)


def js_trunc_int(x: float) -> int:
    """JavaScript ``x | 0`` for values in int32 range."""
    return int(x) if x >= 0 else -int(-x)


def avg_cohesion_pct(avg: float) -> int:
    return js_trunc_int(avg * 100)


def cohesion_pct(c: float) -> int:
    return js_round(c * 100)


def bar_pct(count: int, total: int) -> int:
    return js_round(count / total * 100) if total else 0


def delta_gap_text(now_gap: int, prev_gap: int) -> str:
    d = now_gap - prev_gap
    return f" (↑ tighter {abs(d)})" if d <= 0 else f" (↓ looser {d})"


def delta_pp_text(now: float, prev: float) -> str:
    d = js_round((now - prev) * 100)
    if d == 0:
        return " (±0)"
    return f" (+{d}pp)" if d > 0 else f" ({d}pp)"


def iteration_record(it: int, counts, *, inertia=None, shift=None, n_changed=None, time_ms=None,
                     world=1, n_points=None) -> dict:
    """One metrics JSONL record per Lloyd iteration."""
    rec = {"iter": it, "counts": [int(c) for c in counts], "balance": balance([int(c) for c in counts]),
           "world": world}
    if inertia is not None:
        rec["inertia"] = inertia
    if shift is not None:
        rec["shift"] = shift
    if n_changed is not None:
        rec["n_changed"] = n_changed
    if time_ms is not None:
        rec["time_ms"] = time_ms
        rec["iters_per_s"] = 1000.0 / time_ms if time_ms > 0 else None
        if n_points is not None and time_ms > 0:
            rec["assign_per_s"] = n_points * 1000.0 / time_ms
    return rec


class MetricsLogger:
    """Per-iteration JSONL records on rank 0.

    One line per checked iteration: ``iter, inertia, shift, max_shift, n_changed,
    counts, balance, time_ms, iters_per_s, assign_per_s, world``.  It is the
    numeric counterpart of the reference dashboard, which recomputes
    ``snapshotMetrics`` on every change (app.mjs:481-496, :498-508).
    """

    def __init__(self, path, *, rank: int = 0, world: int = 1, n_points: int = 0, run_id=None):
        import time

        self._time = time.perf_counter
        self.rank, self.world, self.n_points, self.run_id = rank, world, n_points, run_id
        self.f = open(path, "a", encoding="utf-8") if (path and rank == 0) else None
        self._t = self._time()
        self._it = None

    def log(self, stats, counts=None):
        now = self._time()
        it = stats.iteration
        steps = it - self._it if self._it is not None else max(it, 1)
        dt = (now - self._t) / max(steps, 1)
        self._t, self._it = now, it
        if self.f is None:
            return None
        rec = dict(stats.as_dict())
        if counts is not None:
            counts = [int(c) if float(c).is_integer() else float(c) for c in counts]
            rec["counts"] = counts
            rec["balance"] = balance(counts)
            if math.isinf(rec["balance"]["ratio"]):
                rec["balance"]["ratio"] = "Infinity"
        rec.update(time_ms=dt * 1e3, iters_per_s=1.0 / dt if dt > 0 else None,
                   assign_per_s=self.n_points / dt if dt > 0 else None, world=self.world)
        if self.run_id:
            rec["run_id"] = self.run_id
        import json

        self.f.write(json.dumps(rec) + "\n")
        self.f.flush()
        return rec

    def close(self):
        if self.f is not None:
            self.f.close()
            self.f = None
