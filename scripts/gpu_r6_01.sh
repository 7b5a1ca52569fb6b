#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_determinism.py tests/test_gpu_kernels.py tests/test_gpu_bounded.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r6_01_pytest.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r6_01_bench.log 2>&1 || exit $?
echo done
