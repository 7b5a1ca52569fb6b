#!/bin/bash
# Round-3 session Z: f32 assign / M-step and the cfg2 bench against the round's starting build.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
run() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -3 "gpurun_out/$name.log"; return $rc; }
AB=scripts/abbin/_C_ab_7868911c10ea.so
run abf_assign 200 python -u scripts/ab_ext.py run $AB --dtype f32 --n 4000000 --d 128 --k 256 || exit 1
run abf_update 200 python -u scripts/ab_ext.py run $AB --what update --dtype f32 --n 4000000 --d 128 --k 256 || exit 1
run bench2 200 python -u bench.py --config cfg2 || exit 1
exit 0
