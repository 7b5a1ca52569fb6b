#!/bin/bash
# wide rows held to 2 waves/SIMD by launch bounds where the rows fit 192 registers (and 1-ahead
# A reads in the D=384 bounded build): kernel + bounded tests, A/B against the committed module
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
AB=scripts/abbin/_C_ab_$1.so
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_bounded.py > gpurun_out/r6_49_pytest.log 2>&1 || exit $?
for cfg in "384 1024 bf16 10000000" "512 1024 bf16 10000000" "768 1024 bf16 6000000" "384 1024 f32 2500000"; do
  set -- $cfg
  timeout -k 10 300 python -u scripts/ab_ext.py run "$AB" --d $1 --k $2 --dtype $3 --n $4 --rounds 4 > gpurun_out/r6_49_ab_d$1_$3.log 2>&1 || exit $?
done
echo done
