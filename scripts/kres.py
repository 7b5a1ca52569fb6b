#!/usr/bin/env python3
"""Per-kernel register / scratch / occupancy table of one HIP source (hipcc remarks).

``python scripts/kres.py mikmeans/csrc/assign16.hip [filter]`` compiles the file for
gfx950 with the production flags and prints, per kernel instantiation, the VGPR count,
scratch bytes per lane, LDS and the compiler's occupancy (waves per SIMD), so a kernel
change can be checked for register growth before any GPU run.
"""
import re
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from mikmeans._build import DEVICE_FLAGS, _hipcc  # noqa: E402


def main(argv):
    src = argv[1]
    flt = argv[2] if len(argv) > 2 else ""
    cmd = [_hipcc(), *DEVICE_FLAGS, f"-I{ROOT / 'mikmeans' / 'csrc'}", "-c", src, "-o", "/dev/null",
           "-Rpass-analysis=kernel-resource-usage"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode:
        print(r.stderr)
        return 1
    rows, cur = [], None
    for line in r.stderr.splitlines():
        m = re.search(r"remark: (.*?) \[-Rpass", line)
        if not m:
            continue
        txt = m.group(1).strip()
        if txt.startswith("Function Name:"):
            cur = {"name": txt.split(":", 1)[1].strip()}
            rows.append(cur)
        elif cur is not None and ":" in txt:
            k, v = txt.split(":", 1)
            cur[k.strip()] = v.strip()
    for c in rows:
        if flt and flt not in c["name"]:
            continue
        print(f"{c.get('VGPRs', '?'):>4} vgpr  {c.get('ScratchSize [bytes/lane]', '?'):>4} scr  "
              f"{c.get('Occupancy [waves/SIMD]', '?'):>2} occ  {c.get('LDS Size [bytes/block]', '?'):>6} lds  "
              f"{c['name']}")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
