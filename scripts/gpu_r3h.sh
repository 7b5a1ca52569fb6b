#!/bin/bash
# Round-3 session H: the D=32 packed-key mismatch repro, then the whole GPU suite.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
run() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -4 "gpurun_out/$name.log"; return $rc; }
run keys_d32 300 python -u scripts/debug/keys_d32_repro.py || exit 1
run pytest_gpu 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread || exit 1
exit 0
