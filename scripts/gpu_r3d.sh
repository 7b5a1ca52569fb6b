#!/bin/bash
# Round-3 session D: GPU suite twice (flake check), then the streaming test file alone.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
run() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -3 "gpurun_out/$name.log"; return $rc; }
run pytest_gpu_a 600 python -u -m pytest tests -q -m gpu --maxfail=25 --timeout 300 --timeout-method thread -p no:cacheprovider -rf
[ $? -ge 124 ] && exit 1
run pytest_gpu_b 600 python -u -m pytest tests -q -m gpu --maxfail=25 --timeout 300 --timeout-method thread -p no:cacheprovider -rf
[ $? -ge 124 ] && exit 1
run pytest_stream 300 python -u -m pytest tests/test_gpu_kernels.py -q -k "streaming" --timeout 120 --timeout-method thread -p no:cacheprovider -rf
exit 0
