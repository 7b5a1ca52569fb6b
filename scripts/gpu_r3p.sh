#!/bin/bash
# Round-3 session P: D=128 assign with 8 waves per ring (32 KiB or 16 KiB chunks) vs 4.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
run() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -3 "gpurun_out/$name.log"; return $rc; }
run ab_geom128 300 python -u scripts/varg_ab.py --env MIKMEANS_ASSIGN_GEOM --values 0,1,2 \
    --shapes "20000000,128,1024;10000000,128,2048" || exit 1
exit 0
