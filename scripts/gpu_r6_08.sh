#!/bin/bash
# round 6: the one-ring-per-CU assign -- bitwise tests (bounded time), then an interleaved A/B
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 python -u -m pytest tests/test_gpu_ring.py -m gpu -x -v --timeout 60 --timeout-method thread > gpurun_out/r6_08_pytest_ring.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/assign_ab.py --n 20000000 --arms "assign_ring=0;assign_ring=1" > gpurun_out/r6_08_ab_ring_d128.log 2>&1 || exit $?
timeout -k 10 400 python -u scripts/assign_ab.py --n 100000000 --rounds 4 --reps 3 --arms "assign_ring=0;assign_ring=1" > gpurun_out/r6_08_ab_ring_n1e8.log 2>&1 || exit $?
echo done
