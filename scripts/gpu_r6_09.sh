#!/bin/bash
# round 6: ring assign -- where its waves' cycles go (timeline counters), skip-window A/B
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 python -u -m pytest tests/test_gpu_ring.py -m gpu -x -q --timeout 60 --timeout-method thread > gpurun_out/r6_09_pytest_ring.log 2>&1 || exit $?
for arm in 1 2 3; do
  timeout -k 10 120 python -u scripts/ring_timeline.py --arm assign_ring=$arm > gpurun_out/r6_09_ring_timeline_$arm.log 2>&1 || exit $?
done
timeout -k 10 300 python -u scripts/assign_ab.py --n 20000000 --arms "assign_ring=0;assign_ring=1;assign_ring=2;assign_ring=3" > gpurun_out/r6_09_ab_ring_skip.log 2>&1 || exit $?
echo done
