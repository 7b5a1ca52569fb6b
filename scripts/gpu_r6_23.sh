#!/bin/bash
# property sweeps of the assign and M-step kernels over random shapes
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_properties.py -v --timeout 600 --hypothesis-show-statistics --timeout-method thread > gpurun_out/r6_23_pytest_properties.log 2>&1 || exit $?
echo done
