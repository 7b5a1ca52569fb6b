#!/bin/bash
# the full E-step + incremental M-step (algorithm='lloyd', library default M-step): steady-state kernels
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_r6_32_incr -- python3 scripts/bounded_profile.py --no-bounded --steps 12 --warmup 3 > gpurun_out/r6_32_prof_incr.log 2>&1 || exit $?
python3 scripts/trace_overlap.py gpurun_out/prof_r6_32_incr --last-steps 8 > gpurun_out/r6_32_incr_steady.json || exit $?
echo done
