#!/bin/bash
# round 6 closing run after the wide-row assign changes: full GPU suite + smoke, the headline
# bench, and the shape sweep (bf16 all widths incl. the wide rows, f32 D=512)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r6_47_pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r6_47_smoke.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r6_47_bench.log 2>&1 || exit $?
timeout -k 10 600 python -u scripts/assign_sweep.py --d 32,64,128,256,384,512,768,1024 --dtypes bf16 > gpurun_out/r6_47_assign_sweep_bf16.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/assign_sweep.py --d 512,1024 --dtypes f32 > gpurun_out/r6_47_assign_sweep_f32.log 2>&1 || exit $?
echo done
