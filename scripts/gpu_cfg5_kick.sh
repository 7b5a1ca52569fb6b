#!/bin/bash
# cfg5 streamed with and without the kicked prefetch; the prefetch test
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_kernels.py -x -v -k "prefetch" --timeout 120 \
  --timeout-method thread > gpurun_out/r5_27_pytest_prefetch.log 2>&1 || exit $?
for a in 1 2; do
timeout -k 10 300 python -u bench.py --config cfg5 --steps 20 --warmup 3 > gpurun_out/r5_27_cfg5_plain_$a.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --config cfg5 --prefetch --steps 20 --warmup 3 > gpurun_out/r5_27_cfg5_kick_$a.log 2>&1 || exit $?
done
echo done
