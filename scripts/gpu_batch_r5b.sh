#!/bin/bash
# round-5 GPU batch b: centre-stationary assign (numerics, then A/B at D=256 / D=128), then the
# pending batch-a steps (setup pass, multi-rank W=2/4/8, cfg5 prefetch, blob RNG)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v -k "centre_stationary" --timeout 120 \
  --timeout-method thread > gpurun_out/r5_20_pytest_cs.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/assign_ab.py --n 16777216 --d 256 --k 512 --rounds 4 --reps 10 \
  --arms "default;assign_cs=1;assign_geom=4;assign_geom=5;assign_geom=6" > gpurun_out/r5_21_ab_d256_cs.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/assign_ab.py --n 20000000 --d 128 --k 1024 --rounds 4 --reps 5 \
  --arms "default;assign_cs=1" > gpurun_out/r5_22_ab_d128_cs.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests/test_gpu_bounded.py -x -v -k "gathered or trajectory" --timeout 200 \
  --timeout-method thread > gpurun_out/r5_23_pytest_bounded_cs.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/setup_pass_bench.py > gpurun_out/r5_14_setup_pass.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_multirank.py -q --timeout 600 --timeout-method thread \
  > gpurun_out/r5_15_multirank.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --config cfg5 --prefetch --steps 10 --warmup 2 > gpurun_out/r5_16_cfg5_prefetch.log 2>&1 || exit $?
timeout -k 10 120 python -u scripts/blobs_bench.py --tpr 8,4,2 > gpurun_out/r5_17_blobs_xor3.log 2>&1 || exit $?
echo batch-done
