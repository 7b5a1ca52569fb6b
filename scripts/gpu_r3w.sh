#!/bin/bash
# Round-3 session W: the next chunk's LDS-DMA pieces spread over the tiles (PMAJ=3) vs issued
# together after the barrier (1); assign tests with it forced.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
run() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -3 "gpurun_out/$name.log"; return $rc; }
run ab_spread 400 python -u scripts/varg_ab.py --env MIKMEANS_ASSIGN_PMAJ --values 1,3 \
    --shapes "20000000,128,1024;10000000,64,4096;16777216,256,512" || exit 1
MIKMEANS_ASSIGN_PMAJ=3 run pytest_assign_spread 400 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "assign and not per_point_offset_seeds" || exit 1
exit 0
