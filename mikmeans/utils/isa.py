"""gfx950 ISA inspection of the built kernels (CPU only: LLVM tools, no GPU).

Used by the ISA guard test (tests/test_isa_guard.py): the bf16 assign kernels must never
seed an MFMA accumulator with a packed-f32 VALU result.  A ``v_pk_add_f32`` that builds an
MFMA's srcC (the per-point seed offsets of csrc/assign16.hip) intermittently reached the
matrix core wrong on gfx950 -- the toolchain inserts no wait state between the two
(profiles/r3_15_ppo_seed_race.md) -- so assign16.hip is compiled with
``-fno-slp-vectorize`` and adds the seeds as scalar ``v_add_f32`` (``seed_add``).  The
check here finds, for every MFMA that accumulates onto registers it did not itself write,
the instruction that last wrote those registers, and flags packed-f32 writers.
"""
from __future__ import annotations

import re
import subprocess
import tempfile
from dataclasses import dataclass
from pathlib import Path

LLVM = Path("/opt/rocm/llvm/bin")
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"

_FUNC = re.compile(r"^[0-9a-f]+ <(?P<name>[^>]+)>:$")
_REG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")
_PACKED_F32 = ("v_pk_add_f32", "v_pk_fma_f32", "v_pk_mul_f32", "v_pk_mov_b32")


def _tool(name: str) -> str:
    p = LLVM / name
    return str(p) if p.exists() else name


def device_elf(obj: Path, out: Path) -> Path:
    """The gfx950 code object inside a hipcc ``-c`` host object (its .hip_fatbin bundle)."""
    with tempfile.TemporaryDirectory() as d:
        fat = Path(d) / "fat.bin"
        subprocess.run([_tool("llvm-objcopy"), f"--dump-section=.hip_fatbin={fat}", str(obj),
                        str(Path(d) / "host.o")], check=True, capture_output=True)
        subprocess.run([_tool("clang-offload-bundler"), "--unbundle", "--type=o", f"--targets={TARGET}",
                        f"--input={fat}", f"--output={out}"], check=True, capture_output=True)
    return out


def disassemble(elf: Path) -> str:
    r = subprocess.run([_tool("llvm-objdump"), "-d", "--mcpu=gfx950", str(elf)], check=True,
                       capture_output=True, text=True)
    return r.stdout


def functions(asm: str) -> dict[str, list[str]]:
    """Mangled function name -> its instruction lines (comments / encodings stripped)."""
    out: dict[str, list[str]] = {}
    cur = None
    for line in asm.splitlines():
        m = _FUNC.match(line.strip())
        if m:
            cur = out.setdefault(m.group("name"), [])
            continue
        if cur is None or not line.startswith("\t"):
            continue
        ins = line.strip().split("//")[0].strip()
        if ins:
            cur.append(ins)
    return out


def _regs(op: str) -> set[int]:
    s: set[int] = set()
    for m in _REG.finditer(op):
        if m.group(3) is not None:
            s.add(int(m.group(3)))
        else:
            s.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return s


def _operands(ins: str) -> tuple[str, list[str]]:
    parts = ins.split(None, 1)
    ops = [o.strip() for o in parts[1].split(",")] if len(parts) > 1 else []
    return parts[0], ops


def _vgpr_dest(ins: str) -> set[int]:
    """VGPRs an instruction writes (its first operand for VALU / MFMA / loads into VGPRs)."""
    op, ops = _operands(ins)
    if not ops or not (op.startswith("v_") or op.startswith("ds_") or op.startswith("buffer_")
                       or op.startswith("global_") or op.startswith("flat_") or op.startswith("scratch_")):
        return set()
    if ("store" in op or op.startswith("ds_write") or op.startswith("v_cmp") or op.startswith("v_readfirstlane")
            or op.startswith("v_readlane") or op.startswith("v_accvgpr_write") or " lds" in ins
            or op.startswith("global_load_lds") or op.startswith("buffer_load_lds")):
        return set()
    if op.startswith("ds_") and not op.startswith(("ds_read", "ds_load", "ds_bpermute", "ds_permute",
                                                     "ds_swizzle", "ds_add_rtn", "ds_min_rtn", "ds_max_rtn")):
        return set()
    return _regs(ops[0])


@dataclass
class Hazard:
    function: str
    mfma: str
    writer: str
    distance: int


def packed_seed_hazards(funcs: dict[str, list[str]], name_filter: str = "assign16_kernel") -> list[Hazard]:
    """MFMAs whose srcC was last written by a packed-f32 VALU op (linear backward scan)."""
    found = []
    for fn, lines in funcs.items():
        if name_filter not in fn:
            continue
        for i, ins in enumerate(lines):
            op, ops = _operands(ins)
            if not op.startswith("v_mfma") or len(ops) < 4:
                continue
            src_c = _regs(ops[3])
            if not src_c:
                continue
            for j in range(i - 1, -1, -1):
                dst = _vgpr_dest(lines[j])
                if dst & src_c:
                    if lines[j].split(None, 1)[0] in _PACKED_F32:
                        found.append(Hazard(fn, ins, lines[j], i - j))
                    break
    return found


def packed_ops(funcs: dict[str, list[str]], name_filter: str = "assign16_kernel") -> int:
    return sum(1 for fn, ls in funcs.items() if name_filter in fn for x in ls if x.split(None, 1)[0] in _PACKED_F32)


@dataclass
class KernelResources:
    name: str            # demangled
    vgprs: int
    vgpr_spills: int
    scratch_bytes: int   # .private_segment_fixed_size


def kernel_resources(elf: Path) -> list[KernelResources]:
    """Per-kernel register use from the code object's AMDGPU metadata note."""
    r = subprocess.run([_tool("llvm-readelf"), "--notes", str(elf)], check=True, capture_output=True,
                       text=True).stdout
    raw = []
    for blk in r.split("- .agpr_count")[1:]:
        name = re.search(r"\.name:\s+(\S+)", blk)
        vg = re.search(r"\.vgpr_count:\s+(\d+)", blk)
        sp = re.search(r"\.vgpr_spill_count:\s+(\d+)", blk)
        pr = re.search(r"\.private_segment_fixed_size:\s+(\d+)", blk)
        if name and vg:
            raw.append((name.group(1), int(vg.group(1)), int(sp.group(1)) if sp else 0,
                        int(pr.group(1)) if pr else 0))
    dem = subprocess.run(["c++filt"], input="\n".join(x[0] for x in raw), capture_output=True,
                         text=True).stdout.splitlines() if raw else []
    if len(dem) != len(raw):
        dem = [x[0] for x in raw]
    return [KernelResources(d, v, s_, p_) for (_, v, s_, p_), d in zip(raw, dem)]


def assign16_template_args(demangled: str) -> list[str] | None:
    """The template arguments of an assign16_kernel instantiation (T, DPAD, P, CT, NBUF, OCC,
    NW, FULLD, VARG, PMAJ, TOP2, XV), or None."""
    if "assign16_kernel<" not in demangled:
        return None
    inner = demangled[demangled.index("assign16_kernel<") + len("assign16_kernel<"):]
    inner = inner[: inner.rindex(">(")]
    return [a.strip() for a in inner.split(",")]
