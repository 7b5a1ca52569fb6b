#!/bin/bash
# wide-row assign: A-fragment reads 4 ahead of their MFMAs -- kernel tests, then one-process A/B
# against HEAD's kernels at D = 512 / 768 / 1024 (bf16) and 512 (f32)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
AB=$(ls scripts/abbin/_C_ab_$(git rev-parse --short=12 HEAD 2>/dev/null || echo x)*.so 2>/dev/null | head -1)
[ -n "$AB" ] || AB=$(ls -t scripts/abbin/_C_ab_*.so | head -1)
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py > gpurun_out/r6_44_pytest_kernels.log 2>&1 || exit $?
for cfg in "512 1024 bf16 10000000" "768 1024 bf16 6000000" "1024 1024 bf16 5000000" "384 1024 bf16 10000000" "512 1024 f32 2500000"; do
  set -- $cfg
  timeout -k 10 300 python -u scripts/ab_ext.py run "$AB" --d $1 --k $2 --dtype $3 --n $4 --rounds 4 > gpurun_out/r6_44_ab_wide_d$1_$3.log 2>&1 || exit $?
done
echo done
