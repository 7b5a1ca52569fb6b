#!/bin/bash
# HIP stream -> hardware queue mapping and side-stream overlap (blob generator vs M-step)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/stream_queue_probe.py > gpurun_out/r6_27_stream_probe.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_r6_27_probe -- python3 scripts/stream_queue_probe.py > gpurun_out/r6_27_stream_probe_prof.log 2>&1 || exit $?
echo done
