#!/bin/bash
# bounded-path kernels (asm max in the segment merge): bounded / property / determinism tests
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_bounded.py tests/test_gpu_properties.py tests/test_gpu_determinism.py tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r6_38_pytest.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/bounded_profile.py > gpurun_out/r6_38_bounded_steps.log 2>&1 || exit $?
echo done
