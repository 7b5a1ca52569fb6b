"""Build the native extension ``mikmeans._C`` with hipcc for gfx950.

No ``torch.utils.cpp_extension`` (whose ROCm path hipifies sources): every HIP
translation unit is compiled by ``hipcc --offload-arch=gfx950`` directly and the
binding is linked against torch's own libraries, so exactly one HIP runtime
(torch's ``libamdhip64``) is loaded in-process.  Objects are cached by a hash of
(source, headers, flags); the resulting ``.so`` lives in-tree next to this file
so it travels with the repository snapshot to the GPU box.

Usage: ``python -m mikmeans._build [--force] [-j N]``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import subprocess
import sys
import sysconfig
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
BUILD = PKG.parent / "build" / "native"
ARCH = os.environ.get("MIKMEANS_ARCH", "gfx950")
HIP_SOURCES = ["assign16.hip", "update.hip", "finalize.hip", "kpp.hip", "rows.hip", "transform.hip"]
BINDING = "binding.cpp"

DEVICE_FLAGS = [
    f"--offload-arch={ARCH}",
    "-O3",
    "-std=c++17",
    "-fPIC",
    # MFMA accumulators in arch VGPRs (gfx950 has a unified file): the epilogue
    # then reads them without v_accvgpr_read copies.
    "-mllvm",
    "-amdgpu-mfma-vgpr-form=1",
    "-Wno-unused-result",
]


# Per-source extras.  The assign kernel: no SLP vectorizer, so the MFMA seed adds stay
# scalar v_add_f32 (packed v_pk_add_f32 seeds intermittently corrupted a point block's
# scores on gfx950; see seed_add in common.h).
SOURCE_FLAGS = {"assign16.hip": ["-fno-slp-vectorize"]}


def source_flags(name: str, csrc: Path = CSRC) -> list[str]:
    """hipcc flags of one HIP translation unit (tests/test_isa_guard.py rebuilds with them)."""
    return [*DEVICE_FLAGS, *SOURCE_FLAGS.get(name, []), f"-I{csrc}"]


def ext_path() -> Path:
    return PKG / ("_C" + sysconfig.get_config_var("EXT_SUFFIX"))


def _torch_paths():
    import torch

    root = Path(torch.__file__).resolve().parent
    inc = [root / "include", root / "include" / "torch" / "csrc" / "api" / "include"]
    lib = root / "lib"
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if cand and (os.path.isabs(cand) and os.path.exists(cand) or not os.path.isabs(cand)):
            return cand
    return "hipcc"


def _digest(paths, flags) -> str:
    h = hashlib.sha256()
    for p in sorted(paths):
        h.update(p.name.encode())
        h.update(p.read_bytes())
    h.update(" ".join(flags).encode())
    return h.hexdigest()[:16]


def _headers(csrc: Path = CSRC):
    return sorted(csrc.glob("*.h"))


def _compile(src: Path, flags, verbose: bool, build_dir: Path = BUILD) -> Path:
    build_dir.mkdir(parents=True, exist_ok=True)
    tag = _digest([src, *_headers(src.parent)], flags)
    obj = build_dir / f"{src.stem}.{tag}.o"
    if obj.exists():
        return obj
    cmd = [_hipcc(), *flags, "-c", str(src), "-o", str(obj) + ".tmp"]
    if verbose:
        print("[mikmeans build]", " ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src.name}:\n{r.stdout}\n{r.stderr}")
    os.replace(str(obj) + ".tmp", obj)
    for old in build_dir.glob(f"{src.stem}.*.o"):  # keep only the current object per source
        if old != obj:
            old.unlink(missing_ok=True)
    return obj


def build(force: bool = False, verbose: bool = True, jobs: int | None = None, *, csrc: Path = CSRC,
          build_dir: Path = BUILD, out: Path | None = None, module: str = "_C") -> Path:
    """Compile every HIP TU for gfx950 and link ``mikmeans/_C*.so``; return its path.

    ``csrc`` / ``build_dir`` / ``out`` / ``module`` build another checkout of the kernel
    sources into a separately named module (scripts/ab_ext.py: A/B against a git ref)."""
    inc, lib, abi = _torch_paths()
    py_inc = sysconfig.get_paths()["include"]
    binding_flags = [
        *DEVICE_FLAGS,
        "-x",
        "hip",
        f"-DTORCH_EXTENSION_NAME={module}",
        "-DTORCH_API_INCLUDE_EXTENSION_H",
        f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
        *[f"-I{p}" for p in inc],
        f"-I{py_inc}",
        f"-I{csrc}",
        "-w",
    ]
    if force and build_dir.exists():
        for o in build_dir.glob("*.o"):
            o.unlink()
    jobs = jobs or min(8, os.cpu_count() or 4)
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        # (another checkout -- scripts/ab_ext.py -- compiles every HIP TU it has, its own list)
        sources = ([s for s in HIP_SOURCES if (csrc / s).exists()] if csrc == CSRC
                   else sorted(p.name for p in csrc.glob("*.hip")))
        futs = [ex.submit(_compile, csrc / s, source_flags(s, csrc), verbose, build_dir) for s in sources]
        futs.append(ex.submit(_compile, csrc / BINDING, binding_flags, verbose, build_dir))
        objs = [f.result() for f in futs]
    out = out or ext_path()
    link_tag = _digest(objs, ["link", str(out)])
    stamp = build_dir / "link.stamp"
    if not force and out.exists() and stamp.exists() and stamp.read_text() == link_tag:
        return out
    cmd = [
        _hipcc(),
        f"--offload-arch={ARCH}",
        "-shared",
        "-fPIC",
        *map(str, objs),
        "-o",
        str(out) + ".tmp",
        f"-L{lib}",
        "-lc10",
        "-ltorch",
        "-ltorch_cpu",
        "-ltorch_python",
        "-lc10_hip",
        "-ltorch_hip",
        f"-Wl,-rpath,{lib}",
    ]
    if verbose:
        print("[mikmeans build]", " ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    os.replace(str(out) + ".tmp", out)
    stamp.write_text(link_tag)
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=None)
    ap.add_argument("-q", "--quiet", action="store_true")
    a = ap.parse_args(argv)
    p = build(force=a.force, verbose=not a.quiet, jobs=a.jobs)
    print(p)
    return 0


if __name__ == "__main__":
    sys.exit(main())
