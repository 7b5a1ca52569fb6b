#!/bin/bash
# Round-3 session F: assign A/B switches (MFMA issue order, D=256 ring depth / point blocks).
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
run() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -4 "gpurun_out/$name.log"; return $rc; }
run ab_pmaj 300 python -u scripts/varg_ab.py --env MIKMEANS_ASSIGN_PMAJ --values 0,1 \
    --shapes "20000000,128,1024;16777216,256,512;20000000,128,2048" || exit 1
run ab_geom256 300 python -u scripts/varg_ab.py --env MIKMEANS_ASSIGN_GEOM --values 0,1,2 \
    --shapes "16777216,256,512;8388608,256,1024" || exit 1
exit 0
