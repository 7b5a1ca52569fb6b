#!/bin/bash
# throughput map of the E-step and M-step kernels over (D, K, dtype)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 900 python -u scripts/assign_sweep.py > gpurun_out/r6_43_assign_sweep.log 2>&1 || exit $?
echo done
