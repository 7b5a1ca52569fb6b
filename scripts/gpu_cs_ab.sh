#!/bin/bash
# centre-stationary assign: numerics, then A/B against the streaming kernel at D=256 / D=128
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
tag=${1:-cs}
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v -k "centre_stationary" --timeout 120 \
  --timeout-method thread > gpurun_out/${tag}_pytest.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/assign_ab.py --n 16777216 --d 256 --k 512 --rounds 4 --reps 10 \
  --arms "default;assign_cs=1" > gpurun_out/${tag}_ab_d256.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/assign_ab.py --n 20000000 --d 128 --k 1024 --rounds 4 --reps 5 \
  --arms "default;assign_cs=1" > gpurun_out/${tag}_ab_d128.log 2>&1 || exit $?
echo done
