#!/bin/bash
# Round-3 session A: smoke, kernel tests, in-process A/B of the assign vs the round-2 head
# at the three bf16 shapes, headline bench.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
set -o pipefail
AB=scripts/abbin/_C_ab_0567132016a6.so
run() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -3 "gpurun_out/$name.log"; return $rc; }
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" &&
run pytest_kern 600 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread &&
run ab128 300 python scripts/ab_ext.py run $AB --n 20000000 --d 128 --k 1024 &&
run ab64 300 python scripts/ab_ext.py run $AB --n 10000000 --d 64 --k 4096 &&
run ab256 300 python scripts/ab_ext.py run $AB --n 16777216 --d 256 --k 512 &&
run bench 600 python bench.py --steps 20 --warmup 3
