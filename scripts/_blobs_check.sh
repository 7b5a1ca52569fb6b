cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu -k "blobs or minibatch or stream" > gpurun_out/t_blobs.log 2>&1 || { tail -30 gpurun_out/t_blobs.log; exit 1; }
tail -1 gpurun_out/t_blobs.log
timeout -k 10 300 python bench.py --config cfg5 --steps 20 --warmup 3 > gpurun_out/bench_cfg5.log 2>&1 && grep -v amdgpu gpurun_out/bench_cfg5.log | tail -1 | cut -c1-260
cd gpurun_out && export TMPDIR=/tmp && rm -rf prof5 && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d prof5 -o p -- python3 ../bench.py --config cfg5 --steps 5 --warmup 1 > b5.log 2>&1 && head -5 prof5/p_kernel_stats.csv | cut -c1-160
