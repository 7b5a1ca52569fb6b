cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -m gpu -k "col_absmax or blobs or lloyd or minibatch" > gpurun_out/t_cm.log 2>&1 || { tail -30 gpurun_out/t_cm.log; exit 1; }
tail -1 gpurun_out/t_cm.log
timeout -k 10 120 python - <<'PY'
import torch, mikmeans
from mikmeans.ops import col_max_abs
X = torch.randn(100_000_000, 128, device="cuda", dtype=torch.bfloat16)
for f, name in ((col_max_abs, "native"), (lambda X: torch.aminmax(X, dim=0), "torch.aminmax")):
    f(X); torch.cuda.synchronize()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    e[0].record()
    for _ in range(5): f(X)
    e[1].record(); torch.cuda.synchronize()
    ms = e[0].elapsed_time(e[1]) / 5
    print(f"{name}: {ms:.3f} ms  ({25.6e9 / ms / 1e9:.2f} TB/s)")
PY
