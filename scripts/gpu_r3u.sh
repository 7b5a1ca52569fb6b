#!/bin/bash
# Round-3 session U: single s_setprio raise per tile (a duplicate had crept in) vs HEAD.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
run() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -3 "gpurun_out/$name.log"; return $rc; }
run pytest_assign 400 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k assign || exit 1
AB=scripts/abbin/_C_ab_f94f0842dc0c.so
run abp_d128 200 python -u scripts/ab_ext.py run $AB --n 20000000 --d 128 --k 1024 || exit 1
run abp_d64 200 python -u scripts/ab_ext.py run $AB --n 10000000 --d 64 --k 4096 || exit 1
run abp_d256 200 python -u scripts/ab_ext.py run $AB --n 16777216 --d 256 --k 512 || exit 1
exit 0
