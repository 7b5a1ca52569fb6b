"""bench.py driver contract, rehearsed on gloo CPU ranks (same multi-rank code path as the
RCCL run the driver launches with ``torch.distributed.run --nproc-per-node N``)."""
import json
import os
import subprocess
import sys

import pytest

from mikmeans.parallel.launch import free_port

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_bench_json_line_on_cpu_ranks(world):
    """The driver's 1/2/4/8-rank command lines (gloo ranks standing in for GPUs)."""
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


def test_bench_self_launches_without_torchrun():
    """The driver's plain ``python bench.py --gpus N`` starts its own N ranks."""
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--steps", "2", "--warmup", "1", "--device", "cpu",
           "--points", "6000"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(CUDA_VISIBLE_DEVICES="", OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["config"]["parallelism"] == "dp2"
    assert rec["comm"] == {"backend": "gloo", "world_size": 2, "process_group": True}


def test_bench_rejects_world_mismatch():
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--steps", "1", "--warmup", "0", "--device", "cpu",
           "--points", "6000"]
    env = dict(os.environ, WORLD_SIZE="1", CUDA_VISIBLE_DEVICES="")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 2 and "WORLD_SIZE=1" in r.stderr


def test_bench_one_rank_joins_a_real_group():
    """N=1 without a launcher still runs the collective path (a one-rank gloo group here,
    RCCL on the GPU box)."""
    cmd = [sys.executable, "bench.py", "--steps", "1", "--warmup", "0", "--device", "cpu", "--points", "4000"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(CUDA_VISIBLE_DEVICES="", OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert rec["n_gpus"] == 1 and rec["comm"] == {"backend": "gloo", "world_size": 1, "process_group": True}
