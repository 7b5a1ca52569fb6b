#!/usr/bin/env python3
"""One-process A/B of the production kernels against the SAME kernels at a git ref.

No hand-maintained kernel copies: ``build`` checks ``mikmeans/csrc`` out of a git ref
(``git archive``) and compiles it, with the production build (``mikmeans/_build.py``),
into a separately named extension module under ``scripts/abbin/`` (in-tree, so it
travels to the GPU box; built here on the CPU).  ``run`` (GPU) loads the current
``mikmeans._C`` and that module side by side and times their kernels on identical
inputs in interleaved rounds, so box-to-box clock differences cancel.

  python scripts/ab_ext.py build HEAD~1            # prints the module path
  python scripts/ab_ext.py run scripts/abbin/_C_ab_<sha>.so --n 20000000 --d 128 --k 1024
"""
from __future__ import annotations

import argparse
import importlib.util
import json
import os
import statistics
import subprocess
import sys
import tarfile
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
ABBIN = ROOT / "scripts" / "abbin"


def cmd_build(ref: str) -> Path:
    from mikmeans import _build

    sha = subprocess.run(["git", "-C", str(ROOT), "rev-parse", ref], check=True, capture_output=True,
                         text=True).stdout.strip()[:12]
    src_root = ROOT / "build" / "ab" / sha
    csrc = src_root / "mikmeans" / "csrc"
    if not csrc.exists():
        src_root.mkdir(parents=True, exist_ok=True)
        with tempfile.NamedTemporaryFile(suffix=".tar") as tf:
            subprocess.run(["git", "-C", str(ROOT), "archive", "-o", tf.name, sha, "mikmeans/csrc"], check=True)
            with tarfile.open(tf.name) as t:
                t.extractall(src_root)
    ABBIN.mkdir(parents=True, exist_ok=True)
    module = f"_C_ab_{sha}"
    out = ABBIN / f"{module}.so"
    _build.build(verbose=False, csrc=csrc, build_dir=src_root / "obj", out=out, module=module)
    (ABBIN / f"{module}.json").write_text(json.dumps({"ref": ref, "sha": sha}))
    print(out)
    return out


def load_module(path: str):
    import torch  # noqa: F401  (torch's HIP runtime first)

    name = Path(path).stem
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _timed(fn, reps):
    import torch

    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return ts


def cmd_run(a) -> int:
    import torch

    from mikmeans.data.blobs import blob_centers, make_blobs
    from mikmeans.models.init import init_random
    from mikmeans.models.lloyd import LloydEngine
    from mikmeans.ops import native
    from mikmeans.parallel import Comm

    mods = {"head": native.require()}
    for p in a.modules:
        meta = Path(p).with_suffix(".json")
        tag = json.loads(meta.read_text())["ref"] if meta.exists() else Path(p).stem
        mods[tag] = load_module(p)
    dt = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    dev = torch.device("cuda")
    comm = Comm.local(dev)
    X = make_blobs(a.n, a.d, a.k, seed=0, dtype=dt, device=dev, centers=blob_centers(a.k, a.d, 10.0, 0, device=dev))
    eng = LloydEngine(X, a.k, comm=comm).set_centers(init_random(X, a.d, a.k, a.n, 0, comm, 0))
    for _ in range(3):
        eng.step()
    Cen = eng.C.contiguous()
    code = native.dtype_code(dt)
    dpad = native.dpad_for(eng.Dp, dt)
    per = {}
    for tag, m in mods.items():
        kpad = m.assign_kpad(code, dpad, a.k)
        pack = torch.zeros(kpad * dpad, dtype=dt, device=dev)
        cn = torch.zeros(m.assign_cn_len(kpad), dtype=torch.float32, device=dev)
        m.finalize(0, None, Cen, None, None, None, pack, cn, None, None, dpad, kpad)
        lab = torch.empty(a.n, dtype=torch.int32, device=dev)
        mind = torch.empty(a.n, dtype=torch.float32, device=dev)
        slots = torch.zeros(m.NSLOT * m.SLOT_STRIDE, dtype=torch.float64, device=dev)
        per[tag] = dict(m=m, pack=pack, cn=cn, kpad=kpad, lab=lab, mind=mind, slots=slots, ts=[])

    def run_assign(t):
        t["m"].assign(eng.X, t["pack"], t["cn"], eng.xn, t["lab"], t["mind"], t["slots"], t["kpad"], dpad, True,
                      None)

    def run_update(t):   # the full M-step pass on the engine's labels into each module's own slab
        m = t["m"]
        if "slab" not in t:
            t["nch"] = m.update_n_chunks(code, a.k, eng.Dp, a.n, False)
            t["slab"] = torch.empty(t["nch"] * a.k * eng.Dp, dtype=torch.int64, device=dev)
            t["cnt"] = torch.empty(t["nch"] * a.k, dtype=torch.int64, device=dev)
        m.update(eng.X, eng.labels, a.k, t["slab"], t["cnt"], t["nch"], None, eng.col_exp, eng.cnt_exp, False)

    def run_blobs(t):    # the on-device generator (+ fused row norms) into each module's own buffer
        if "bx" not in t:
            t["bx"] = torch.empty_like(eng.X)
            t["bn"] = torch.empty(a.n, dtype=torch.float32, device=dev)
            t["bc"] = blob_centers(a.k, a.d, 10.0, 0, device=dev)
        t["m"].blobs(t["bx"], 0, t["bc"], 1.0, 7, None, t["bn"])

    def run_colstats(t):  # the setup pass: column statistics + fused row norms
        m = t["m"]
        t.setdefault("cs", (torch.zeros(eng.Dp, dtype=torch.int32, device=dev),
                            torch.zeros(3 * eng.Dp, dtype=torch.float64, device=dev),
                            torch.zeros(eng.Dp, dtype=torch.int64, device=dev),
                            torch.zeros(eng.Dp, dtype=torch.int32, device=dev),
                            torch.empty(a.n, dtype=torch.float32, device=dev)))
        out, fst, nnz, lowbit, xn = t["cs"]
        out.zero_(); nnz.zero_(); lowbit.fill_(1 << 30)
        m.col_absmax(eng.X, out, fst, nnz, lowbit, xn)

    def run_rownorms(t):  # the plain row-norm pass
        t.setdefault("rn", torch.empty(a.n, dtype=torch.float32, device=dev))
        t["m"].row_sqnorm(eng.X, t["rn"])

    fn = {"update": run_update, "blobs": run_blobs, "colstats": run_colstats,
          "rownorms": run_rownorms}.get(a.what, run_assign)
    for t in per.values():          # warm-up (kernel attributes, code objects)
        fn(t)
    torch.cuda.synchronize()
    for _ in range(a.rounds):
        for t in per.values():
            t["ts"] += _timed(lambda t=t: fn(t), a.reps)
    base = per["head"]
    if a.what == "blobs":           # the same rows and norms from every module
        for tag, t in per.items():
            t["same"] = bool(torch.equal(t["bx"], per["head"]["bx"]) and torch.equal(t["bn"], per["head"]["bn"]))
    if a.what == "colstats":        # the same max / counts / norms; the f64 sums to ~1e-12
        h = per["head"]["cs"]
        for tag, t in per.items():
            c = t["cs"]
            t["same"] = bool(torch.equal(c[0], h[0]) and torch.equal(c[2], h[2]) and torch.equal(c[3], h[3])
                             and torch.equal(c[4], h[4]) and torch.allclose(c[1], h[1], rtol=1e-12, atol=0))
            t["fsums_bitwise"] = bool(torch.equal(c[1], h[1]))
    if a.what == "rownorms":        # the same bits from every module
        for tag, t in per.items():
            t["same"] = bool(torch.equal(t["rn"], per["head"]["rn"]))
    if a.what == "update":          # the same integer sums from every module
        red = {tag: (t["slab"].view(t["nch"], -1).sum(0), t["cnt"].view(t["nch"], -1).sum(0)) for tag, t in per.items()}
        for tag, t in per.items():
            t["same"] = bool(torch.equal(red[tag][0], red["head"][0]) and torch.equal(red[tag][1], red["head"][1]))
    out = {"n": a.n, "d": a.d, "k": a.k, "dtype": a.dtype, "what": a.what, "variants": {}}
    for tag, t in per.items():
        med = statistics.median(t["ts"])
        out["variants"][tag] = {
            "median_ms": round(med, 4), "min_ms": round(min(t["ts"]), 4),
            "tflops": round(2.0 * a.n * a.k * a.d / (med * 1e-3) / 1e12, 1),
            "x_TBps": round(a.n * a.d * (2 if a.dtype == "bf16" else 4) / (med * 1e-3) / 1e12, 2),
            "label_mismatch_vs_head": int((t["lab"] != base["lab"]).sum()) if a.what == "assign" else None,
            "outputs_equal_head": t.get("same"),
            **({"fsums_bitwise": t["fsums_bitwise"]} if "fsums_bitwise" in t else {}),
            "vs_head": round(statistics.median(base["ts"]) / med, 4),
        }
    print(json.dumps(out), flush=True)
    return 0


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    sub = ap.add_subparsers(dest="cmd", required=True)
    b = sub.add_parser("build")
    b.add_argument("ref")
    r = sub.add_parser("run")
    r.add_argument("modules", nargs="+")
    r.add_argument("--n", type=int, default=20_000_000)
    r.add_argument("--d", type=int, default=128)
    r.add_argument("--k", type=int, default=1024)
    r.add_argument("--dtype", default="bf16")
    r.add_argument("--rounds", type=int, default=5)
    r.add_argument("--reps", type=int, default=5)
    r.add_argument("--what", default="assign", choices=["assign", "update", "blobs", "colstats", "rownorms"])
    a = ap.parse_args(argv)
    if a.cmd == "build":
        cmd_build(a.ref)
        return 0
    return cmd_run(a)


if __name__ == "__main__":
    sys.exit(main())
