#!/bin/bash
# four-rows-per-thread bounds update: bounded tests, steps, steady-state kernels
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_bounded.py tests/test_gpu_properties.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r6_40_pytest.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/bounded_profile.py > gpurun_out/r6_40_bounded_steps.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_r6_40_bounded -- python3 scripts/bounded_profile.py --steps 20 --warmup 5 > gpurun_out/r6_40_prof_bounded.log 2>&1 || exit $?
python3 scripts/trace_overlap.py gpurun_out/prof_r6_40_bounded --last-steps 10 > gpurun_out/r6_40_bounded_steady.json || exit $?
echo done
