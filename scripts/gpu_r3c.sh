#!/bin/bash
# Round-3 session C: full GPU test suite (no early stop), cfg4 bench (owner-path timing).
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
run() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -4 "gpurun_out/$name.log"; return $rc; }
run pytest_gpu 1100 python -u -m pytest tests -q -m gpu --maxfail=25 --timeout 300 --timeout-method thread -p no:cacheprovider -rf
rc=$?
[ $rc -ge 124 ] && exit $rc
run bench4 300 python bench.py --config cfg4 --steps 20 --warmup 3
