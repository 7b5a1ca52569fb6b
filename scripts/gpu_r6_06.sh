#!/bin/bash
# round 6: full GPU suite + smoke, then the setup pass against round 5's kernels
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r6_06_pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r6_06_smoke.log 2>&1 || exit $?
R5=scripts/abbin/_C_ab_98a22cc4efee.so
timeout -k 10 300 python -u scripts/ab_ext.py run $R5 --what colstats --n 100000000 --d 128 --k 1024 --rounds 4 --reps 3 > gpurun_out/r6_06_ab_colstats_d128.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/ab_ext.py run $R5 --what colstats --n 16777216 --d 256 --k 512 --rounds 4 --reps 5 > gpurun_out/r6_06_ab_colstats_d256.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/setup_pass_bench.py > gpurun_out/r6_06_setup_pass.log 2>&1 || exit $?
echo done
