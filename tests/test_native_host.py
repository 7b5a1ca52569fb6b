"""Host-code sanitizers: the native JS number formatter built with
AddressSanitizer + UndefinedBehaviorSanitizer (host only -- GPU ASan is not used), fed
random and edge-case doubles, must agree with the Python formatter byte for byte."""
import os
import shutil
import struct
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
def test_jsnum_under_asan_ubsan(tmp_path):
    from mikmeans.utils.jsjson import js_number

    exe = tmp_path / "jsnum_fuzz"
    src = os.path.join(ROOT, "tests", "native", "jsnum_fuzz.cpp")
    inc = os.path.join(ROOT, "mikmeans", "csrc")
    r = subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined",
                        "-fno-sanitize-recover=all", "-I", inc, src, "-o", str(exe)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    rng = np.random.default_rng(0)
    vals = list(rng.standard_normal(3000) * 10.0 ** rng.integers(-30, 30, 3000))
    vals += list(rng.integers(0, 2**64 - 1, 3000, dtype=np.uint64).view(np.float64))
    vals += [0.0, -0.0, 1e21, 1e-7, 1e-6, 123456789012345678901.0, 5e-324, 1.7976931348623157e308,
             float("nan"), float("inf"), -float("inf"), 0.1, 1 / 3, 100.0, 1e20]
    inp = "".join(f"{struct.unpack('<Q', struct.pack('<d', float(v)))[0]:016x}\n" for v in vals)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="halt_on_error=1")
    out = subprocess.run([str(exe)], input=inp, capture_output=True, text=True, env=env, timeout=120)
    assert out.returncode == 0, out.stderr[-2000:]
    got = out.stdout.splitlines()
    assert len(got) == len(vals)
    for v, s in zip(vals, got):
        exp = "null" if not np.isfinite(v) else js_number(float(v))
        assert s == exp, (v, s, exp)


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
def test_launch_planning_under_asan_ubsan(tmp_path):
    """csrc/plan.h (M-step slice width / LDS bytes / chunks, fixed-point exponent, assign
    Kpad) swept over K in [1, 2^20], D in [1, 256] under ASan + UBSan."""
    exe = tmp_path / "plan_fuzz"
    src = os.path.join(ROOT, "tests", "native", "plan_fuzz.cpp")
    inc = os.path.join(ROOT, "mikmeans", "csrc")
    r = subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined",
                        "-fno-sanitize-recover=all", "-I", inc, src, "-o", str(exe)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1", UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    out = subprocess.run([str(exe)], capture_output=True, text=True, env=env, timeout=600)
    assert out.returncode == 0 and out.stdout.startswith("ok "), out.stdout[-2000:] + out.stderr[-2000:]
