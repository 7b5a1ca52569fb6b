#!/bin/bash
# K-split row groups, rule g <= 4 -> 3: the plan vs the earlier runs (r6_56, r6_57); M-step tests
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_mstep.py tests/test_gpu_kernels.py > gpurun_out/r6_58_pytest.log 2>&1 || exit $?
S="python -u scripts/assign_sweep.py --k 1024,2048,4096 --dtypes bf16 --what mstep"
timeout -k 10 200 $S --d 64,128,256 --n 10000000 > gpurun_out/r6_58_mstep_d64_256.log 2>&1 || exit $?
timeout -k 10 200 $S --d 384,512 --n 5000000 > gpurun_out/r6_58_mstep_d384_512.log 2>&1 || exit $?
echo done
