#!/bin/bash
# Round-3 session O: the straight-line (FLAT) column-slice M-step for plain passes, A/B via
# MIKMEANS_UPDATE_FLAT against HEAD, its tests with the switch on, and the benches it serves.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
run() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -3 "gpurun_out/$name.log"; return $rc; }
MIKMEANS_UPDATE_FLAT=1 run pytest_mstep_flat 400 python -u -m pytest tests/test_gpu_mstep.py tests/test_gpu_minibatch.py -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
AB=scripts/abbin/_C_ab_7868911c10ea.so
for fl in 0 1; do
  MIKMEANS_UPDATE_FLAT=$fl run abu_f32_flat$fl 200 python -u scripts/ab_ext.py run $AB --what update --dtype f32 --n 20000000 --d 128 --k 256 || exit 1
  MIKMEANS_UPDATE_FLAT=$fl run abu_d256_flat$fl 200 python -u scripts/ab_ext.py run $AB --what update --n 16777216 --d 256 --k 512 || exit 1
done
for fl in 0 1; do
  MIKMEANS_UPDATE_FLAT=$fl run bench2_flat$fl 300 python -u bench.py --config cfg2 || exit 1
  MIKMEANS_UPDATE_FLAT=$fl run bench5s_flat$fl 300 python -u bench.py --config cfg5 || exit 1
done
exit 0
