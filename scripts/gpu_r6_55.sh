#!/bin/bash
# M-step at the wide widths and K=4096: K-split kernel (default) vs the column-slice kernel
# (MIKMEANS_UPDATE_KS=0) and the K-split's row groups in flight (MIKMEANS_UPDATE_KS_GM=2/3/6)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
S="python -u scripts/assign_sweep.py --n 5000000 --d 128,384,512 --k 1024,4096 --dtypes bf16 --what mstep"
timeout -k 10 200 $S > gpurun_out/r6_55_mstep_default.log 2>&1 || exit $?
MIKMEANS_UPDATE_KS=0 timeout -k 10 200 $S > gpurun_out/r6_55_mstep_slice.log 2>&1 || exit $?
for gm in 2 3 6; do
  MIKMEANS_UPDATE_KS_GM=$gm timeout -k 10 200 $S > gpurun_out/r6_55_mstep_gm$gm.log 2>&1 || exit $?
done
timeout -k 10 200 $S > gpurun_out/r6_55_mstep_default2.log 2>&1 || exit $?
echo done
