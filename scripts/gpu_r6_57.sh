#!/bin/bash
# K-split row groups at D = 64 / 128 / 256 (cfg4 is D=64 K=4096): the plan's choice vs forced 2 / 3 / 6
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
S="python -u scripts/assign_sweep.py --d 64,128,256 --k 1024,2048,4096 --n 10000000 --dtypes bf16 --what mstep"
timeout -k 10 200 $S > gpurun_out/r6_57_mstep_default.log 2>&1 || exit $?
MIKMEANS_UPDATE_KS_GM=2 timeout -k 10 200 $S > gpurun_out/r6_57_mstep_gm2.log 2>&1 || exit $?
MIKMEANS_UPDATE_KS_GM=3 timeout -k 10 200 $S > gpurun_out/r6_57_mstep_gm3.log 2>&1 || exit $?
MIKMEANS_UPDATE_KS_GM=6 timeout -k 10 200 $S > gpurun_out/r6_57_mstep_gm6.log 2>&1 || exit $?
timeout -k 10 200 $S > gpurun_out/r6_57_mstep_default2.log 2>&1 || exit $?
echo done
