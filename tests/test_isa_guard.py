"""ISA guard for the assign kernels' seed-add workaround (CPU: hipcc + LLVM tools, no GPU).

A packed ``v_pk_add_f32`` that builds an MFMA's accumulator seed intermittently reached the
matrix core wrong on gfx950 (5 of 12 launches gave one point block wrong labels,
profiles/r3_15_ppo_seed_race.md): the toolchain emits no wait state between the packed
VALU write and the MFMA's srcC read.  csrc/assign16.hip therefore adds seeds as scalar
``v_add_f32`` and is compiled with ``-fno-slp-vectorize`` (mikmeans/_build.py).  These tests
read the built gfx950 code object and fail if any assign16 MFMA's srcC was last written by
a packed-f32 op -- and show that dropping the flag brings the pattern back, so the guard
is live.  scripts/microbench/seed_hazard.hip is the standalone repro.
"""
import shutil
from pathlib import Path

import pytest

from mikmeans import _build
from mikmeans.utils import isa

pytestmark = pytest.mark.skipif(shutil.which(_build._hipcc()) is None and not Path(_build._hipcc()).exists(),
                                reason="hipcc not available")
SRC = _build.CSRC / "assign16.hip"


def _hazards(obj: Path, tmp: Path):
    funcs = isa.functions(isa.disassemble(isa.device_elf(obj, tmp / "dev.o")))
    assert any("assign16_kernel" in f for f in funcs), "no assign16 kernels in the code object"
    return isa.packed_seed_hazards(funcs), funcs


def test_built_assign16_has_no_packed_seed_writes(tmp_path):
    """The production object (same flags and sources as the shipped _C .so; cached)."""
    flags = _build.source_flags(SRC.name)
    assert "-fno-slp-vectorize" in flags
    obj = _build._compile(SRC, flags, verbose=False)
    hz, funcs = _hazards(obj, tmp_path)
    assert not hz, [(h.function[:80], h.writer, h.mfma) for h in hz[:5]]
    # the bf16 kernels really use the per-point-offset seeds (the path the flag protects)
    assert sum("assign16_kernelIt" in f for f in funcs) >= 8


@pytest.mark.slow
def test_guard_detects_packed_seeds_without_the_flag(tmp_path):
    """Negative control: the same source without -fno-slp-vectorize vectorises seed_add into
    v_pk_add_f32 feeding MFMA srcC, and the checker flags it (so removing the flag from
    _build.py fails the test above's premise, not silently)."""
    flags = [f for f in _build.source_flags(SRC.name) if f != "-fno-slp-vectorize"]
    obj = _build._compile(SRC, flags, verbose=False, build_dir=tmp_path / "build")
    hz, _ = _hazards(obj, tmp_path)
    assert hz, "expected packed-f32 seed writes without -fno-slp-vectorize"
    assert all(h.writer.startswith("v_pk_") for h in hz)


def test_launchers_never_read_the_environment():
    """Kernel geometry switches live in one registry (kernels.h ``Variant``), read from the
    environment once when the extension loads; no .hip launcher calls getenv (verdict r3:
    per-launch reads were silently frozen into captured graphs)."""
    for src in sorted(_build.CSRC.glob("*.hip")) + sorted(_build.CSRC.glob("*.h")):
        assert "getenv" not in src.read_text(), src.name
    assert _build.CSRC.joinpath("binding.cpp").read_text().count("getenv(") == 1


def test_assign_kernels_register_budget(tmp_path):
    """Spill guard (round 4): every bounded-E-step (TOP2) instantiation and the headline
    geometry (bf16 D=128, 4 blocks at 4 waves/SIMD) fit their register budget.  TOP2 builds
    of the bf16 D=64/128/256 default geometries spilled 500-940 VGPRs and ran 5.7x slower
    (profiles/r4_05_hamerly_ab_top2_spills.log), which no functional test notices."""
    obj = _build._compile(SRC, _build.source_flags(SRC.name), verbose=False)
    res = isa.kernel_resources(isa.device_elf(obj, tmp_path / "dev.o"))
    a16 = [(r, isa.assign16_template_args(r.name)) for r in res]
    a16 = [(r, t) for r, t in a16 if t]
    assert len(a16) > 30
    top2 = [(r, t) for r, t in a16 if t[10] == "true"]     # (TOP2; t[11]: its exact epilogue XV)
    assert top2, "no TOP2 instantiations"
    # TOP2 geometries (top2_geom) spill nothing, except the 4-block D = 128 one (the default
    # since round 4: 14 VGPRs, outside the MFMA loop; profiles/r4_16_top2_register_study.md)
    bad = [(t[:7], r.vgpr_spills) for r, t in top2
           if r.vgpr_spills > (16 if (t[1] in ("64", "128") and t[2] == "4") else 0)]
    assert not bad, bad
    head = [r for r, t in a16 if t[:7] == ["unsigned short", "128", "4", "4", "2", "4", "4"]
            and t[8:] == ["false", "1", "false", "false"]]
    assert head and max(r.vgpr_spills for r in head) <= 2, [(r.name[-60:], r.vgpr_spills) for r in head]


def test_colstats_bf16_register_budget(tmp_path):
    """The packed bf16 column-statistics kernels (csrc/finalize.hip) stay at 4 waves/SIMD
    without spills: the per-element f64 form held 148 VGPRs (3 waves/SIMD) and a first packed
    form with a rare-path branch reached 177 and spilled under a 3-wave cap -- 27 % slower
    than the kernel it replaced (profiles/r6_11_ab_colstats_d128.log)."""
    src = _build.CSRC / "finalize.hip"
    obj = _build._compile(src, _build.source_flags(src.name), verbose=False)
    res = [r for r in isa.kernel_resources(isa.device_elf(obj, tmp_path / "dev.o"))
           if "col_absmax_kernel<unsigned short, true" in r.name]
    assert len(res) >= 3, [r.name for r in res]
    bad = [(r.name, r.vgprs, r.vgpr_spills) for r in res if r.vgprs > 128 or r.vgpr_spills]
    assert not bad, bad


def test_wide_assign_two_wave_budget(tmp_path):
    """The wide-row bf16 assign kernels sized for 2 waves/SIMD (D = 384 with 4 point blocks,
    512 with 3, 768 with 2) stay at or under 256 VGPRs and spill nothing: crossing 256 drops
    them to one wave per SIMD (D=384 with its A reads 4 ahead took 265 VGPRs and ran 15 %
    slower, profiles/r6_44_ab_wide_d384_bf16.log; 3 blocks at D=512 gained 18-26 % over 4 at
    one wave, profiles/r6_45_ab_d512_*.log)."""
    obj = _build._compile(SRC, _build.source_flags(SRC.name), verbose=False)
    res = isa.kernel_resources(isa.device_elf(obj, tmp_path / "dev.o"))
    want = {"384": "4", "512": "3", "768": "2"}
    wide = [(r, t) for r, t in ((r, isa.assign16_template_args(r.name)) for r in res)
            if t and t[0] == "unsigned short" and t[1] in want]
    assert {t[1] for _, t in wide} == set(want), [t[:3] for _, t in wide]
    assert all(t[2] == want[t[1]] for _, t in wide), [t[:3] for _, t in wide]
    bad = [(t[:3], r.vgprs, r.vgpr_spills) for r, t in wide if r.vgprs > 256 or r.vgpr_spills]
    assert not bad, bad
