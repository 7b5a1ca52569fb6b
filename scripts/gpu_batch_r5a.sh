#!/bin/bash
# round-5 GPU batch: D=256 geometry A/B, setup-pass timing, W=2/4/8 multi-rank tests, cfg5 with prefetch
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/assign_ab.py --n 16777216 --d 256 --k 512 --rounds 4 --reps 10 \
  --arms "default;assign_geom=3;assign_geom=4;assign_geom=5;assign_geom=6" > gpurun_out/r5_13_ab_d256_ast.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/setup_pass_bench.py > gpurun_out/r5_14_setup_pass.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_multirank.py -q --timeout 600 --timeout-method thread \
  > gpurun_out/r5_15_multirank.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --config cfg5 --prefetch --steps 10 --warmup 2 > gpurun_out/r5_16_cfg5_prefetch.log 2>&1 || exit $?
timeout -k 10 120 python -u scripts/blobs_bench.py --tpr 8,4,2 > gpurun_out/r5_17_blobs_xor3.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -k "blob or sample or philox or kpar" --timeout 200 \
  --timeout-method thread > gpurun_out/r5_17_pytest_rng.log 2>&1 || exit $?
echo batch-done
