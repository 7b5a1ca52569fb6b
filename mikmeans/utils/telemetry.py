"""GPU clock / power telemetry over a timed region (amdsmi; ``None`` when unavailable).

The headline's box-to-box spread (41.9-44.3 it/s on the same code) tracks the
GFX clock the card sustains under the MFMA load, which depends on the box's power and thermal
state.  :class:`ClockSampler` polls the GPU's current GFX clock and socket power on a
background thread while a timed region runs, so a bench line carries the clock it was
measured at and a kernel regression can be told from a slow box (work per clock cycle:
``value / clock_mhz``).

Only reads (no clock or power setting).  The sampling thread does not touch HIP.
"""
from __future__ import annotations

import statistics
import threading
import time


def _amdsmi():
    try:
        import amdsmi  # noqa: PLC0415

        return amdsmi
    except Exception:  # noqa: BLE001 -- absent or broken library: no telemetry
        return None


def _bdf_of_torch_device(index: int) -> str | None:
    """``dddd:bb:dd`` PCI address of torch device ``index`` (None if torch does not say)."""
    try:
        import torch

        p = torch.cuda.get_device_properties(index)
        return f"{int(p.pci_domain_id):04x}:{int(p.pci_bus_id):02x}:{int(p.pci_device_id):02x}"
    except Exception:  # noqa: BLE001
        return None


def _first_number(d: dict, keys) -> float | None:
    """The first usable value among ``keys`` of an amdsmi record (lists: the mean of the
    valid entries, e.g. one clock per XCD); 'N/A' and the 0xFFFF.. sentinels are skipped."""
    for k in keys:
        v = d.get(k)
        vals = v if isinstance(v, (list, tuple)) else [v]
        ok = [float(x) for x in vals if isinstance(x, (int, float)) and 0 < float(x) < 0xFFFF]
        if ok:
            return sum(ok) / len(ok)
    return None


class ClockSampler:
    """Background sampler of one GPU's GFX clock (MHz) and socket power (W).

    ``with ClockSampler(device_index) as s: ...timed region...`` then ``s.summary()``:
    ``{"clock_mhz": mean, "clock_mhz_min": .., "clock_mhz_max": .., "power_w": mean,
    "samples": n}`` or ``None`` when amdsmi is unavailable or yielded no sample."""

    GFX_KEYS = ("current_gfxclk", "current_gfxclks", "average_gfxclk_frequency")
    POWER_KEYS = ("current_socket_power", "average_socket_power")

    def __init__(self, device_index: int = 0, period_s: float = 0.05):
        self.period = float(period_s)
        self.clock: list[float] = []
        self.power: list[float] = []
        self.error: str | None = None
        self._stop = threading.Event()
        self._thread = None
        self._smi = _amdsmi()
        self._handle = None
        if self._smi is None:
            self.error = "amdsmi not importable"
            return
        try:
            self._smi.amdsmi_init()
            handles = self._smi.amdsmi_get_processor_handles()
            want = _bdf_of_torch_device(device_index)
            for h in handles:
                try:
                    bdf = str(self._smi.amdsmi_get_gpu_device_bdf(h)).lower()
                except Exception:  # noqa: BLE001
                    continue
                if want and bdf.startswith(want):
                    self._handle = h
                    break
            if self._handle is None and len(handles) == 1:
                self._handle = handles[0]
            if self._handle is None:
                self.error = f"no amdsmi handle for device {device_index} ({want}) among {len(handles)}"
        except Exception as e:  # noqa: BLE001
            self.error = f"amdsmi: {type(e).__name__}: {e}"
            self._handle = None

    def _sample(self):
        smi, h = self._smi, self._handle
        clk = pw = None
        try:
            m = smi.amdsmi_get_gpu_metrics_info(h)
            clk = _first_number(m, self.GFX_KEYS)
            pw = _first_number(m, self.POWER_KEYS)
        except Exception:  # noqa: BLE001 -- older metric tables: the per-query calls
            pass
        if clk is None:
            try:
                clk = _first_number(smi.amdsmi_get_clock_info(h, smi.AmdSmiClkType.GFX), ("clk", "cur_clk"))
            except Exception:  # noqa: BLE001
                pass
        if pw is None:
            try:
                pw = _first_number(smi.amdsmi_get_power_info(h), self.POWER_KEYS)
            except Exception:  # noqa: BLE001
                pass
        if clk is not None:
            self.clock.append(clk)
        if pw is not None:
            self.power.append(pw)

    def _run(self):
        while not self._stop.is_set():
            self._sample()
            self._stop.wait(self.period)

    def __enter__(self):
        if self._handle is not None:
            self._sample()
            self._thread = threading.Thread(target=self._run, name="mikmeans-clock", daemon=True)
            self._thread.start()
        return self

    def __exit__(self, *exc):
        if self._thread is not None:
            self._stop.set()
            self._thread.join(timeout=2.0)
            self._sample()
        return False

    def summary(self) -> dict | None:
        if not self.clock and not self.power:
            return None
        out = {"samples": max(len(self.clock), len(self.power))}
        if self.clock:
            out.update(clock_mhz=round(statistics.fmean(self.clock), 1), clock_mhz_min=round(min(self.clock), 1),
                       clock_mhz_max=round(max(self.clock), 1))
        if self.power:
            out["power_w"] = round(statistics.fmean(self.power), 1)
        return out


def sample_for(seconds: float, device_index: int = 0) -> dict | None:
    """Idle-clock probe: sample for ``seconds`` (tests / session notes)."""
    with ClockSampler(device_index) as s:
        time.sleep(seconds)
    return s.summary()
