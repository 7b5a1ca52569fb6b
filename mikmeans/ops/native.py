"""Loader for the in-tree native extension ``mikmeans._C`` (gfx950 HIP kernels).

The extension is built by :mod:`mikmeans._build` (``hipcc --offload-arch=gfx950``)
and lives next to the package so it ships with the repository.  GPU code paths
call :func:`require`, which fails loudly when the extension is missing: a GPU run
must never silently fall back to eager PyTorch.
"""
from __future__ import annotations

import importlib
import os

import torch  # noqa: F401  (torch's HIP runtime must be loaded before _C)

_mod = None
_err: BaseException | None = None

DT_F32 = 0
DT_BF16 = 1


def _load():
    global _mod, _err
    if _mod is not None or _err is not None:
        return _mod
    try:
        _mod = importlib.import_module("mikmeans._C")
    except BaseException as e:  # ImportError, OSError (missing symbols), ...
        _err = e
        if os.environ.get("MIKMEANS_AUTOBUILD", "0") == "1":
            from .. import _build

            _build.build(verbose=False)
            _err = None
            _mod = importlib.import_module("mikmeans._C")
    return _mod


def available() -> bool:
    return _load() is not None


def require():
    """Return the native module or raise with the build instructions."""
    m = _load()
    if m is None:
        raise RuntimeError(
            "mikmeans native extension is not built (mikmeans/_C*.so missing or unloadable: "
            f"{_err!r}). Build it with `python -m mikmeans._build` (hipcc, gfx950)."
        )
    return m


def dtype_code(dtype: torch.dtype) -> int:
    if dtype == torch.bfloat16:
        return DT_BF16
    if dtype == torch.float32:
        return DT_F32
    raise TypeError(f"mikmeans: unsupported compute dtype {dtype}")


def vec_elems(dtype: torch.dtype) -> int:
    """Elements per 16-byte piece: the column padding granule of the vector path."""
    return 8 if dtype == torch.bfloat16 else 4


WIDE_DPADS = (384, 512, 768, 1024)


def dpad_for(D: int, dtype: torch.dtype) -> int:
    """Padded feature width the assign kernel is instantiated for (0 = unsupported): a power
    of two of at least four 16-byte pieces (one per lane group of the 16x16 MFMA tile) up to
    256, then the wide-row widths 384 / 512 / 768 / 1024 (csrc/plan.h ``assign_dpad``)."""
    d = 4 * vec_elems(dtype)
    while d < D and d < 256:
        d *= 2
    if D <= d:
        return d
    return next((w for w in WIDE_DPADS if D <= w), 0)


_warned: set = set()


def warn_once(msg: str) -> None:
    if msg not in _warned:
        _warned.add(msg)
        import warnings

        warnings.warn("mikmeans: " + msg, stacklevel=3)


def _variant_index(name: str) -> int:
    names = [n.lower() for n in require().variant_names()]
    key = name.lower().removeprefix("mikmeans_")
    if key not in names:
        raise KeyError(f"unknown kernel variant {name!r} (known: {names})")
    return names.index(key)


def get_variant(name: str) -> int:
    """Current value of a kernel A/B switch (-1 = the built-in rule)."""
    return int(require().get_variant(_variant_index(name)))


def set_variant(name: str, value: int) -> None:
    """Set a kernel A/B switch (``assign_varg``, ``assign_pmaj``, ``assign_geom``,
    ``update_ks``, ``update_ks_gm``, ``blobs_tpr``, ``assign_top2_geom``, ``assign_epi``,
    ``assign_early``; -1 = built-in rule).  The launchers never read the environment:
    ``MIKMEANS_<NAME>`` is read once when the extension loads."""
    require().set_variant(_variant_index(name), int(value))


class variant:
    """``with native.variant("assign_varg", 1): ...`` -- a switch for the block's launches."""

    def __init__(self, name: str, value):
        self.name, self.value = name, -1 if value is None else int(value)

    def __enter__(self):
        self.old = get_variant(self.name)
        set_variant(self.name, self.value)
        return self

    def __exit__(self, *exc):
        set_variant(self.name, self.old)
        return False


NSLOT, SLOT_STRIDE = 256, 8   # csrc/kernels.h
SLOT_OVF = 1 << 61            # csrc/common.h


def slot_totals(slots: torch.Tensor) -> tuple[float, int]:
    """(inertia, changed rows) held by the assign kernel's order-free slots (csrc/common.h
    ``slot_add``): integer digit words summed over the slots, decoded high word first --
    the same value ``reduce_kernel`` writes into the packed message."""
    w = slots.detach().reshape(-1).view(torch.int64).reshape(-1, SLOT_STRIDE).sum(0).tolist()
    if w[6] >= SLOT_OVF >> 1:
        return float("inf"), int(w[7])
    import math

    v = 0.0
    for j in range(6, -1, -1):
        v += math.ldexp(float(w[j]), 32 * j - 64)
    return v, int(w[7])


def loaded_path() -> str | None:
    m = _load()
    return getattr(m, "__file__", None) if m is not None else None
