cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/t_all.log 2>&1 || { tail -30 gpurun_out/t_all.log; exit 1; }
tail -1 gpurun_out/t_all.log
timeout -k 10 300 python bench.py --config cfg5 --steps 20 --warmup 3 > gpurun_out/bench_cfg5.log 2>&1 && grep -v amdgpu gpurun_out/bench_cfg5.log | tail -1 | cut -c1-200
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench.log 2>&1 && grep -v amdgpu gpurun_out/bench.log | tail -1 | cut -c1-200
