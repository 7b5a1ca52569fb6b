#!/bin/bash
# round 6: full GPU suite + smoke closing run of the round;
# then the headline bench and the setup-pass bench
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r6_42_pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r6_42_smoke.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r6_42_bench.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/setup_pass_bench.py > gpurun_out/r6_42_setup_pass.log 2>&1 || exit $?
echo done
