#!/bin/bash
# vectorised full-pass changed-row list: incremental-M-step tests and the steady-state kernels
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_mstep.py tests/test_gpu_bounded.py -x -q --timeout 300 --timeout-method thread -k "incremental or delta or bounded or auto" > gpurun_out/r6_36_pytest.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_r6_36_incr -- python3 scripts/bounded_profile.py --no-bounded --steps 12 --warmup 3 > gpurun_out/r6_36_prof_incr.log 2>&1 || exit $?
python3 scripts/trace_overlap.py gpurun_out/prof_r6_36_incr --last-steps 8 > gpurun_out/r6_36_incr_steady.json || exit $?
echo done
