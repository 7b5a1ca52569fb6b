#!/bin/bash
# one-wave wide kernels (bf16 D=1024, f32 D=512): 3 point blocks vs 2 at f32 D=512 (committed module)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
AB=scripts/abbin/_C_ab_6f7edbc0ab76.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "wide or assign" > gpurun_out/r6_54_pytest.log 2>&1 || exit $?
for cfg in "512 1024 f32 2500000" "512 4096 f32 1000000" "512 256 f32 2500000"; do
  set -- $cfg
  timeout -k 10 300 python -u scripts/ab_ext.py run "$AB" --d $1 --k $2 --dtype $3 --n $4 --rounds 4 > gpurun_out/r6_54_ab_d$1_k$2_$3.log 2>&1 || exit $?
done
echo done
