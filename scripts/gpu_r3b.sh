#!/bin/bash
# Round-3 session B: full GPU test suite, cfg5 stream + resident, headline bench.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
run() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -4 "gpurun_out/$name.log"; return $rc; }
run pytest_gpu 1100 python -u -m pytest tests -q -m gpu --maxfail=25 --timeout 300 --timeout-method thread -p no:cacheprovider
rc=$?
[ $rc -ge 124 ] && exit $rc
run bench5 300 python bench.py --config cfg5 --steps 20 --warmup 3 &&
run bench5r 400 python bench.py --config cfg5 --resident --steps 20 --warmup 3 &&
run bench 400 python bench.py --steps 20 --warmup 3
