#!/bin/bash
# the bounded step's gathered assign, one feature removed at a time
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/gathered_assign_probe.py > gpurun_out/r6_33_gathered_probe.log 2>&1 || exit $?
echo done
