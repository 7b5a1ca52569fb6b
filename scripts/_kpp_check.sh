cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu -k "kpp or kmeanspp or plusplus or init" > gpurun_out/t_kpp.log 2>&1 || { tail -30 gpurun_out/t_kpp.log; exit 1; }
tail -1 gpurun_out/t_kpp.log
for r in 1 2; do
timeout -k 10 300 python bench.py --config cfg4 --steps 20 --warmup 3 > gpurun_out/bench_cfg4.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/bench_cfg4.log | grep '^{' | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('init_s', d['init_s'], 'it/s', round(d['value'],1))"
done
