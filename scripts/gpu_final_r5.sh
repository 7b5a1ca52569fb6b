#!/bin/bash
# round-5 closing measurements: full GPU suite, smoke, then the bench configs
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r5_48_pytest_gpu_full.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5_48_smoke.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > gpurun_out/r5_48_bench.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --config cfg4 > gpurun_out/r5_48_bench_cfg4.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --config cfg5 --steps 20 --warmup 3 > gpurun_out/r5_48_bench_cfg5.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --config cfg5 --resident --steps 20 --warmup 3 > gpurun_out/r5_48_bench_cfg5r.log 2>&1 || exit $?
echo done
