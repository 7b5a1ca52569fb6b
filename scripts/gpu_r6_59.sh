#!/bin/bash
# round 6 final tree (after the wide-row assign and M-step row-group changes): full GPU suite + smoke, then the bench lines (headline, cfg2, cfg4, cfg5
# streamed / resident)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r6_59_pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r6_59_smoke.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r6_59_bench.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --config cfg2 --steps 300 --warmup 30 > gpurun_out/r6_59_bench_cfg2.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --config cfg4 --steps 20 --warmup 3 > gpurun_out/r6_59_bench_cfg4.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --config cfg5 --steps 20 --warmup 3 > gpurun_out/r6_59_bench_cfg5.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --config cfg5 --resident --steps 20 --warmup 3 > gpurun_out/r6_59_bench_cfg5r.log 2>&1 || exit $?
echo done
