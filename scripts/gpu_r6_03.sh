#!/bin/bash
# round 6: the grid-stride blob generator (bitwise mirror tests + timing at the headline and
# cfg5 shapes), the setup pass, cfg2 and the headline.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "blob or colstat or col_stats or norms or slots" -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r6_03_pytest.log 2>&1 || exit $?
timeout -k 10 200 python -u scripts/blobs_bench.py --n 100000000 --d 128 --k 1024 --reps 5 > gpurun_out/r6_03_blobs_d128.log 2>&1 || exit $?
timeout -k 10 200 python -u scripts/blobs_bench.py --reps 10 > gpurun_out/r6_03_blobs_cfg5.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/setup_pass_bench.py > gpurun_out/r6_03_setup_pass.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --config cfg2 --steps 300 --warmup 30 > gpurun_out/r6_03_cfg2.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r6_03_bench.log 2>&1 || exit $?
echo done
