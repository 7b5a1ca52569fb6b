#!/bin/bash
# round 6: the auto-algorithm / determinism GPU tests, then a same-box A/B of cfg2 (fp32,
# N=1e6 D=128 K=256) between the round-4 tree (abtree/r4, built from d88d4b7) and HEAD,
# interleaved, plus a kernel trace of each.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_bounded.py -k "auto" tests/test_gpu_determinism.py tests/test_gpu_memplan.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r6_02_pytest.log 2>&1 || exit $?
for i in 1 2 3; do
  (cd abtree/r4 && timeout -k 10 200 python -u bench.py --config cfg2 --steps 300 --warmup 30) > gpurun_out/r6_02_cfg2_r4_$i.log 2>&1 || exit $?
  timeout -k 10 200 python -u bench.py --config cfg2 --steps 300 --warmup 30 > gpurun_out/r6_02_cfg2_head_$i.log 2>&1 || exit $?
done
(cd abtree/r4 && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_r4 -o r4 -- python -u bench.py --config cfg2 --steps 100 --warmup 10) > gpurun_out/r6_02_prof_r4.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_head -o head -- python -u bench.py --config cfg2 --steps 100 --warmup 10 > gpurun_out/r6_02_prof_head.log 2>&1 || exit $?
mkdir -p gpurun_out/r6_02_prof
find /tmp/prof_r4 /tmp/prof_head -name "*.csv" -exec cp {} gpurun_out/r6_02_prof/ \; 
ls -la gpurun_out/r6_02_prof
echo done
