#!/bin/bash
# Round-3 session N: column-slice M-step with LDS-staged gathered rows (cfg5) and labels
# clamped where used; K-split ping-pong.  Tests first, then one-process A/B vs HEAD and benches.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
run() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -4 "gpurun_out/$name.log"; return $rc; }
run pytest_mstep 400 python -u -m pytest tests/test_gpu_mstep.py tests/test_gpu_minibatch.py -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
run pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
AB=scripts/abbin/_C_ab_7868911c10ea.so
run abu_f32 200 python -u scripts/ab_ext.py run $AB --what update --dtype f32 --n 20000000 --d 128 --k 256 || exit 1
run abu_d256 200 python -u scripts/ab_ext.py run $AB --what update --n 16777216 --d 256 --k 512 || exit 1
run bench5r 300 python -u bench.py --config cfg5 --resident || exit 1
run bench4 300 python -u bench.py --config cfg4 || exit 1
run bench 300 python -u bench.py || exit 1
exit 0
