#!/bin/bash
# K-split row groups: the new rule (3 groups for whole 1-KiB rows at m = 1) vs forced 3 / 6,
# D = 384 / 512 at K = 1024 / 2048 / 4096; M-step tests
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_mstep.py > gpurun_out/r6_56_pytest_mstep.log 2>&1 || exit $?
S="python -u scripts/assign_sweep.py --n 5000000 --d 384,512 --k 1024,2048,4096 --dtypes bf16 --what mstep"
timeout -k 10 200 $S > gpurun_out/r6_56_mstep_default.log 2>&1 || exit $?
MIKMEANS_UPDATE_KS_GM=3 timeout -k 10 200 $S > gpurun_out/r6_56_mstep_gm3.log 2>&1 || exit $?
MIKMEANS_UPDATE_KS_GM=6 timeout -k 10 200 $S > gpurun_out/r6_56_mstep_gm6.log 2>&1 || exit $?
timeout -k 10 200 $S > gpurun_out/r6_56_mstep_default2.log 2>&1 || exit $?
echo done
