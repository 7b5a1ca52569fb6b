#!/bin/bash
# Round-3 session Q: D=256 assign with 8 waves per ring; rocprof of the cfg5 resident step.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
run() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -3 "gpurun_out/$name.log"; return $rc; }
run pytest_gather 300 python -u -m pytest tests/test_gpu_minibatch.py -m gpu -x -q --timeout 120 --timeout-method thread -k gathered || exit 1
run ab_geom256b 300 python -u scripts/varg_ab.py --env MIKMEANS_ASSIGN_GEOM --values 0,1,2 \
    --shapes "16777216,256,512;8388608,256,1024" || exit 1
run ab_geom128b 300 python -u scripts/varg_ab.py --env MIKMEANS_ASSIGN_GEOM --values 0,3 \
    --shapes "20000000,128,1024" || exit 1
bash scripts/prof_cfg.sh cfg5r --config cfg5 --resident --steps 10 --warmup 3 || exit 1
exit 0
