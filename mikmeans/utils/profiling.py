"""Tracing / profiling helpers.

* :func:`range` -- roctx ranges (``torch.cuda.nvtx`` maps to roctx on ROCm), so
  rocprofv3 ``--marker-trace`` shows assign / update / allreduce / finalize;
* :class:`EventTimer` -- device-event timing of a region, no host sync until read;
* :func:`rocprof_cmd` -- the rocprofv3 command line the repo's profiles use.
"""
from __future__ import annotations

import contextlib
import time

import torch


@contextlib.contextmanager
def range(name: str):  # noqa: A001 - mirrors nvtx.range
    on = torch.cuda.is_available()
    if on:
        try:
            torch.cuda.nvtx.range_push(name)
        except Exception:
            on = False
    try:
        yield
    finally:
        if on:
            torch.cuda.nvtx.range_pop()


class EventTimer:
    """Accumulates device time of repeated regions: ``with t.region(): ...``; ``t.ms()``."""

    def __init__(self, enabled: bool | None = None):
        self.enabled = torch.cuda.is_available() if enabled is None else enabled
        self.pairs = []
        self._host = []

    @contextlib.contextmanager
    def region(self):
        if self.enabled:
            a = torch.cuda.Event(enable_timing=True)
            b = torch.cuda.Event(enable_timing=True)
            a.record()
            yield
            b.record()
            self.pairs.append((a, b))
        else:
            t0 = time.perf_counter()
            yield
            self._host.append((time.perf_counter() - t0) * 1e3)

    def ms(self) -> list[float]:
        if self.enabled:
            torch.cuda.synchronize()
            return [a.elapsed_time(b) for a, b in self.pairs]
        return list(self._host)


def rocprof_cmd(out_dir: str, *argv: str, pmc: list[str] | None = None) -> list[str]:
    """``rocprofv3 --kernel-trace --stats -d OUT -- argv`` (or a PMC-only run)."""
    cmd = ["rocprofv3", "--kernel-trace", "--stats", "--output-format", "csv", "-d", out_dir]
    if pmc:
        cmd += ["--pmc", *pmc]
    return cmd + ["--", *argv]
