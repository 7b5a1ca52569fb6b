#!/bin/bash
# cfg5 streamed: kernel trace, then the concurrency of the blob prefetch with the step's kernels
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_r6_25_cfg5 -- python3 bench.py --config cfg5 --steps 12 --warmup 3 > gpurun_out/r6_25_prof_cfg5.log 2>&1 || exit $?
python3 scripts/trace_overlap.py gpurun_out/prof_r6_25_cfg5 --last-steps 10 > gpurun_out/r6_25_cfg5_overlap.json || exit $?
echo done
