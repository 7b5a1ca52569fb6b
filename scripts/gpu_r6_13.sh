#!/bin/bash
# Lean bf16 column statistics: GPU tests, then a one-process A/B against the old kernel (HEAD)
# and the same kernel without the 3-waves register cap; then the ceilings script again.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_mstep.py -x -v --timeout 120 --timeout-method thread -k "col_stats or sparse or wide_column" > gpurun_out/r6_13_pytest.log 2>&1 &&
timeout -k 10 240 python -u scripts/ab_ext.py run scripts/abbin/_C_ab_1b4c98204445.so --what colstats --n 100000000 --d 128 --rounds 5 --reps 5 > gpurun_out/r6_13_ab_colstats_d128.log 2>&1 &&
timeout -k 10 240 python -u scripts/ab_ext.py run scripts/abbin/_C_ab_1b4c98204445.so --what colstats --n 16777216 --d 256 --rounds 5 --reps 5 > gpurun_out/r6_13_ab_colstats_d256.log 2>&1 &&
timeout -k 10 240 python -u scripts/hbm_ceiling.py > gpurun_out/r6_13_hbm_ceiling.log 2>&1
