#!/bin/bash
# round 6: setup pass (resident-sized grid) and blob generator A/B against round 5's kernels
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_mstep.py tests/test_gpu_kernels.py -k "col_stats or blob or norms" -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r6_04_pytest.log 2>&1 || exit $?
R5=scripts/abbin/_C_ab_98a22cc4efee.so
timeout -k 10 300 python -u scripts/ab_ext.py run $R5 --what colstats --n 100000000 --d 128 --k 1024 --rounds 4 --reps 3 > gpurun_out/r6_04_ab_colstats_d128.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/ab_ext.py run $R5 --what blobs --n 100000000 --d 128 --k 1024 --rounds 4 --reps 3 > gpurun_out/r6_04_ab_blobs_d128.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/ab_ext.py run $R5 --what blobs --n 16777216 --d 256 --k 512 --rounds 4 --reps 5 > gpurun_out/r6_04_ab_blobs_d256.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/ab_ext.py run $R5 --what colstats --n 16777216 --d 256 --k 512 --rounds 4 --reps 5 > gpurun_out/r6_04_ab_colstats_d256.log 2>&1 || exit $?
echo done
