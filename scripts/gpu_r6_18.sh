#!/bin/bash
# serving throughput: in-process predict (device / host rows) and the HTTP service
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/serve_bench.py > gpurun_out/r6_18_serve_bench.log 2>&1 || exit $?
timeout -k 10 400 python -u scripts/serve_bench.py --dtype float32 > gpurun_out/r6_18_serve_bench_f32.log 2>&1 || exit $?
echo done
