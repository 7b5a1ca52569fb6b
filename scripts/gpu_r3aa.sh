#!/bin/bash
# Round-3 session AA: 8-wave rings of 32 KiB chunks by default from K=2048 at D=128: tests,
# then one-process A/B against the forced 4-wave ring at K = 2048 / 4096 / 1024.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
run() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -3 "gpurun_out/$name.log"; return $rc; }
run pytest_assign 500 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k assign || exit 1
run ab_geom128c 300 python -u scripts/varg_ab.py --env MIKMEANS_ASSIGN_GEOM --values 0,1 \
    --shapes "10000000,128,2048;5000000,128,4096;4000000,128,3072;20000000,128,1024" || exit 1
exit 0
