#!/bin/bash
# bf16 D=512: 3 point blocks at 2 waves/SIMD vs 4 blocks at 1 (both with the run-ahead A reads),
# and the D=384 run-ahead depth kept under 256 VGPRs, against the committed module
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
AB=scripts/abbin/_C_ab_103a15b57687.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_bounded.py > gpurun_out/r6_45_pytest.log 2>&1 || exit $?
for cfg in "512 1024 bf16 10000000" "512 4096 bf16 5000000" "512 256 bf16 10000000" "384 1024 bf16 10000000"; do
  set -- $cfg
  timeout -k 10 300 python -u scripts/ab_ext.py run "$AB" --d $1 --k $2 --dtype $3 --n $4 --rounds 4 > gpurun_out/r6_45_ab_d$1_k$2.log 2>&1 || exit $?
done
echo done
