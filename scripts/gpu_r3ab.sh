#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
run() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -3 "gpurun_out/$name.log"; return $rc; }
run smoke 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
run pytest_gpu 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
exit 0
