cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -m gpu -k "blob or minibatch" > gpurun_out/t_pf.log 2>&1 || { tail -30 gpurun_out/t_pf.log; exit 1; }
tail -1 gpurun_out/t_pf.log
for pf in --no-prefetch --prefetch --no-prefetch --prefetch; do
timeout -k 10 300 python bench.py --config cfg5 --steps 20 --warmup 3 $pf > gpurun_out/bench_cfg5_pf.log 2>&1 || exit 1
echo "$pf $(grep -v amdgpu gpurun_out/bench_cfg5_pf.log | tail -1 | cut -c70-200)"
done
