cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for r in 1 2; do for u in 4 6 8; do
( cd ab_kpp/u$u && timeout -k 10 200 python bench.py --config cfg4 --steps 5 --warmup 1 > ../../gpurun_out/kpp_u$u.log 2>&1 ) || exit 1
echo "u$u $(grep -v amdgpu gpurun_out/kpp_u$u.log | grep '^{' | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('init_s', d['init_s'])")"
done; done
