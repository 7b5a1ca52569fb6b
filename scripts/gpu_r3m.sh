#!/bin/bash
# Round-3 session M: K-split M-step with ping-pong register sets (no latch copy) against the
# committed HEAD module, one process; then the M-step tests.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
run() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -4 "gpurun_out/$name.log"; return $rc; }
run pytest_mstep 400 python -u -m pytest tests/test_gpu_mstep.py tests/test_gpu_minibatch.py -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
AB=scripts/abbin/_C_ab_7868911c10ea.so
run abu_d128 200 python -u scripts/ab_ext.py run $AB --what update --n 20000000 --d 128 --k 1024 || exit 1
run abu_d64 200 python -u scripts/ab_ext.py run $AB --what update --n 10000000 --d 64 --k 4096 || exit 1
run abu_d128_n1e8 300 python -u scripts/ab_ext.py run $AB --what update --n 100000000 --d 128 --k 1024 --rounds 3 --reps 3 || exit 1
exit 0
