#!/bin/bash
# cfg5 streamed with the side-stream blob prefetch: kernel trace and concurrency
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_r6_26_cfg5pf -- python3 bench.py --config cfg5 --prefetch --steps 12 --warmup 3 > gpurun_out/r6_26_prof_cfg5pf.log 2>&1 || exit $?
python3 scripts/trace_overlap.py gpurun_out/prof_r6_26_cfg5pf --last-steps 10 > gpurun_out/r6_26_cfg5pf_overlap.json || exit $?
timeout -k 10 300 python -u bench.py --config cfg5 --prefetch --steps 20 --warmup 3 > gpurun_out/r6_26_bench_cfg5pf.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --config cfg5 --steps 20 --warmup 3 > gpurun_out/r6_26_bench_cfg5.log 2>&1 || exit $?
echo done
