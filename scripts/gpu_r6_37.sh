#!/bin/bash
# TOP2 chain without per-key canonicalisation: bounded-path tests (bitwise vs the full E-step), the gathered
# assign probe, the bounded steps, and an A/B of the gathered TOP2 assign against HEAD
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_bounded.py tests/test_gpu_properties.py tests/test_gpu_determinism.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r6_37_pytest.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/gathered_assign_probe.py > gpurun_out/r6_37_gathered_probe.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/bounded_profile.py > gpurun_out/r6_37_bounded_steps.log 2>&1 || exit $?
echo done
