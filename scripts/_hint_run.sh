cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 240 python scripts/ab_hint.py > gpurun_out/ab_hint.json 2>gpurun_out/ab_hint.err || { tail -5 gpurun_out/ab_hint.err; exit 1; }
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "hint or graph or incremental or lloyd or assign" > gpurun_out/t_hint.log 2>&1 || { tail -30 gpurun_out/t_hint.log; exit 1; }
tail -2 gpurun_out/t_hint.log
