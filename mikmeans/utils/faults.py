"""Fault injection for failure-detection / elastic-resume tests.

The reference detects a lost peer through P2PT's ``peerclose`` (app.mjs:105) and
degrades to local-only mode (:72, :117); state lives only in open tabs.  Here a
lost rank surfaces as a ``torch.distributed`` error or timeout in the next
collective (``Comm.from_env(timeout_s=...)``); recovery is "resume from the last
checkpoint with any world size".  ``MIKMEANS_FAULT="<rank>:<iteration>"`` makes
that rank raise :class:`InjectedFault` right after the given Lloyd iteration, so
tests can kill a rank mid-fit and check the resumed result.
"""
from __future__ import annotations

import os


class InjectedFault(RuntimeError):
    pass


def _spec():
    s = os.environ.get("MIKMEANS_FAULT", "")
    if not s:
        return None
    r, it = s.split(":")
    return int(r), int(it)


def maybe_fail(rank: int, iteration: int) -> None:
    """Raise if ``MIKMEANS_FAULT`` names this (rank, iteration).  With
    ``MIKMEANS_FAULT_ONCE=<path>`` the fault fires only while ``path`` does not exist (and
    creates it), so a supervised job restarted by ``mikmeans launch`` recovers."""
    spec = _spec()
    if spec is not None and spec == (rank, iteration):
        once = os.environ.get("MIKMEANS_FAULT_ONCE")
        if once:
            if os.path.exists(once):
                return
            with open(once, "w") as f:
                f.write(f"{rank}:{iteration}\n")
        raise InjectedFault(f"injected fault on rank {rank} after iteration {iteration}")
