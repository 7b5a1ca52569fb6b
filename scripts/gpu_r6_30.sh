#!/bin/bash
# the device-counted gathered assign: grid for N rows vs grid for exactly m rows
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/count_tail_probe.py > gpurun_out/r6_30_count_tail.log 2>&1 || exit $?
echo done
