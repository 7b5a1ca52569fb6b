#!/bin/bash
# Round-3 session G: PMAJ (point-block-major MFMA issue) A/B at the other widths and f32,
# then the headline and cfg5 benches with PMAJ on by default at D >= 128, and the assign tests.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
run() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -4 "gpurun_out/$name.log"; return $rc; }
run ab_pmaj_narrow 300 python -u scripts/varg_ab.py --env MIKMEANS_ASSIGN_PMAJ --values 0,1 \
    --shapes "10000000,64,4096;4000000,64,1024;4000000,32,1024" || exit 1
run ab_pmaj_f32 300 python -u scripts/varg_ab.py --env MIKMEANS_ASSIGN_PMAJ --values 0,1 --dtype f32 \
    --shapes "4000000,128,256;2000000,64,1024" || exit 1
run bench 300 python -u bench.py || exit 1
run bench5r 300 python -u bench.py --config cfg5 --resident || exit 1
run pytest_assign 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "assign or lloyd" || exit 1
exit 0
