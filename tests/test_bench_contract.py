"""bench.py driver contract, rehearsed on gloo CPU ranks (same multi-rank code path as the
RCCL run the driver launches with ``torch.distributed.run --nproc-per-node N``)."""
import json
import os
import subprocess
import sys

import pytest

from mikmeans.parallel.launch import free_port

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("world", [1, 2])
def test_bench_json_line_on_cpu_ranks(world):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), "bench.py",
           "--gpus", str(world), "--steps", "2", "--warmup", "1", "--device", "cpu", "--points", "6000"]
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only, one line
    rec = json.loads(lines[0])
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
                "scaling", "vs_baseline", "dtype", "data", "config"):
        assert key in rec
    assert rec["n_gpus"] == world and rec["steps"] == 2 and rec["warmup"] == 1
    assert rec["value"] > 0 and rec["ms_per_step"] == pytest.approx(1e3 / rec["value"])
    assert rec["config"]["parallelism"] == f"dp{world}" and rec["config"]["n_clusters"] == 1024
    assert rec["metric"].startswith("Lloyd iterations/sec") and rec["dtype"] == "bf16"
