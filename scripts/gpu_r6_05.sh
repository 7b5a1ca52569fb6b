#!/bin/bash
# round 6: the statistics grid's block cap sweep
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_mstep.py tests/test_gpu_kernels.py -k "col_stats or norms" -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r6_05_pytest.log 2>&1 || exit $?
timeout -k 10 400 python -u scripts/setup_pass_bench.py --blocks 1024,2048,4096,8192 --rounds 3 > gpurun_out/r6_05_setup_blocks_d128.log 2>&1 || exit $?
timeout -k 10 400 python -u scripts/setup_pass_bench.py --n 16777216 --d 256 --blocks 1024,2048,4096,8192 --rounds 3 > gpurun_out/r6_05_setup_blocks_d256.log 2>&1 || exit $?
echo done
