#!/bin/bash
# the library default path (bounded E-step + incremental M-step) on the headline data: steps and kernels
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/bounded_profile.py > gpurun_out/r6_29_bounded_steps.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r6_29_bounded -- python3 scripts/bounded_profile.py --steps 20 --warmup 5 > gpurun_out/r6_29_prof_bounded.log 2>&1 || exit $?
python3 scripts/summarize_prof.py gpurun_out/prof_r6_29_bounded --title "bounded E-step + incremental M-step (library default), N=1e8 D=128 K=1024 bf16, 25 steps, rocprofv3" > gpurun_out/r6_29_rocprof_bounded.md || exit $?
echo done
