"""CLI, dataset IO and checkpoint/resume (CPU)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, cwd):
    env = dict(os.environ, PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, "-m", "mikmeans", *args], cwd=cwd, env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    return r.stdout


@pytest.mark.parametrize("ext", [".npy", ".safetensors", ".csv"])
def test_io_roundtrip_and_shards(tmp_path, ext):
    from mikmeans.utils.io import load_points, num_rows, save_points

    X = torch.randn(103, 5)
    p = save_points(tmp_path / f"x{ext}", X)
    assert num_rows(p) == (103, 5)
    parts = [load_points(p, r, 4) for r in range(4)]
    assert all(n == 103 for _, n, _ in parts)
    assert [s for _, _, s in parts] == sorted(s for _, _, s in parts)
    full = torch.cat([x for x, _, _ in parts])
    tol = 1e-6 if ext == ".csv" else 0.0
    assert torch.allclose(full, X, atol=tol, rtol=tol)


def test_cli_fit_predict_room(tmp_path):
    out = _run(["blobs", "--n", "3000", "--d", "4", "--centers", "3", "--output", "p.npy", "--labels", "y.npy"],
               tmp_path)
    assert json.loads(out)["shape"] == [3000, 4]
    rec = json.loads(_run(["fit", "--input", "p.npy", "--n-clusters", "3", "--output", "m", "--save-labels",
                           "--device", "cpu"], tmp_path).strip().splitlines()[-1])
    assert sum(rec["metrics"]["counts"]) == 3000
    for f in ("centroids.json", "centroids.safetensors", "state.json", "labels.rank0.npy"):
        assert (tmp_path / "m" / f).exists()
    pred = json.loads(_run(["predict", "--model", "m", "--input", "p.npy", "--output", "pred.npy", "--device",
                            "cpu"], tmp_path).strip().splitlines()[-1])
    assert pred["counts"] == rec["metrics"]["counts"]
    assert np.array_equal(np.load(tmp_path / "pred.npy"), np.load(tmp_path / "m" / "labels.rank0.npy"))
    from sklearn.metrics import adjusted_rand_score

    assert adjusted_rand_score(np.load(tmp_path / "y.npy"), np.load(tmp_path / "pred.npy")) > 0.99
    txt = _run(["room", "--populate", "--centroid", "A", "--centroid", "B", "--auto", "--export", "r.json"],
               tmp_path)
    assert txt.startswith("k = 2")
    js = json.loads((tmp_path / "r.json").read_text())
    assert set(js) == {"cards", "centroids", "meta"} and len(js["cards"]) == 12
    again = _run(["room", "--load", "r.json"], tmp_path)
    assert again.splitlines()[:4] == txt.splitlines()[:4]


def test_cli_fit_algorithm_and_init_options(tmp_path):
    """`fit --algorithm hamerly --init k-means|| --init-sampling two-stage`: the options reach
    the estimator and its saved config (the CPU path assigns every row, so the fit is exact)."""
    _run(["blobs", "--n", "2000", "--d", "3", "--centers", "4", "--output", "p.npy"], tmp_path)
    rec = json.loads(_run(["fit", "--input", "p.npy", "--n-clusters", "4", "--output", "m", "--device", "cpu",
                           "--algorithm", "hamerly", "--init", "k-means||", "--init-sampling", "two-stage"],
                          tmp_path).strip().splitlines()[-1])
    assert sum(rec["metrics"]["counts"]) == 2000
    state = json.loads((tmp_path / "m" / "state.json").read_text())
    cfg = state.get("config", state)
    assert cfg["algorithm"] == "hamerly" and cfg["init"] == "k-means||" and cfg["init_sampling"] == "two-stage"


def test_resume_matches_uninterrupted(tmp_path):
    from mikmeans import KMeans
    from mikmeans.data.blobs import make_blobs

    X = make_blobs(4000, 6, 12, std=3.0, seed=3)
    kw = dict(init="random", seed=5, tol=-1.0, device="cpu")
    full = KMeans(12, max_iter=9, **kw).fit(X)
    part = KMeans(12, max_iter=4, checkpoint_every=2, checkpoint_dir=str(tmp_path / "ck"), **kw).fit(X)
    assert part.n_iter_ == 4
    res = KMeans(12, max_iter=9, **kw).fit(X, resume_from=str(tmp_path / "ck"))
    if full.n_iter_ > 4:
        assert torch.equal(res.cluster_centers_, full.cluster_centers_)
        assert res.inertia_ == full.inertia_


def test_metrics_jsonl(tmp_path):
    from mikmeans import KMeans
    from mikmeans.data.blobs import make_blobs

    X = make_blobs(2000, 3, 5, seed=1)
    p = tmp_path / "m.jsonl"
    km = KMeans(5, max_iter=6, tol=-1.0, device="cpu", metrics_path=str(p), run_id="ABCD").fit(X)
    recs = [json.loads(line) for line in p.read_text().splitlines()]
    assert len(recs) == km.n_iter_
    assert [r["iter"] for r in recs] == list(range(1, km.n_iter_ + 1))
    for r in recs:
        assert sum(r["counts"]) == 2000 and r["balance"]["gap"] == max(r["counts"]) - min(r["counts"])
        assert r["world"] == 1 and r["run_id"] == "ABCD" and r["time_ms"] > 0


def test_cli_export_import_roundtrip(tmp_path):
    _run(["room", "--populate", "--centroid", "Sweet", "--centroid", "Fresh", "--auto", "--export", "r.json"],
         tmp_path)
    out = _run(["import", "--room", "r.json", "--output", "ck", "--assign", "--save-room", "r2.json"], tmp_path)
    assert out.startswith("k = 2")
    st = json.loads((tmp_path / "ck" / "state.json").read_text())
    assert st["n_clusters"] == 2 and st["vocab"] and len(st["centroid_names"]) == 2
    _run(["export", "--model", "ck", "--format", "room", "--output", "r3.json"], tmp_path)
    r3 = json.loads((tmp_path / "r3.json").read_text())
    assert [c["id"] for c in r3["centroids"]] == ["c:0", "c:1"] and r3["cards"] == []
    _run(["export", "--model", "ck", "--format", "flat", "--output", "flat.json"], tmp_path)
    flat = json.loads((tmp_path / "flat.json").read_text())
    assert len(flat) == 2 * st["n_features"]


def test_init_reset_and_unassigned_predict():
    import mikmeans
    from mikmeans import KMeans

    comm = mikmeans.init("cpu")
    assert comm.world == 1 and comm.identity()["rank"] == 0
    X = np.random.default_rng(0).normal(size=(300, 3)).astype(np.float32)
    km = KMeans(3, device="cpu").fit(X)
    Y = X.copy()
    Y[5, 0] = np.nan
    Y[7, 2] = np.inf
    lab = km.predict(Y, unassign_nonfinite=True)
    assert lab[5] == -1 and lab[7] == -1 and (lab[[0, 1, 2]] >= 0).all()
    km.reset()
    with pytest.raises(RuntimeError):
        km.predict(X)


@pytest.mark.parametrize("mode", ["lloyd", "minibatch"])
def test_launch_restarts_failed_job_from_checkpoint(tmp_path, mode):
    """``mikmeans launch``: a 2-rank job whose rank 1 dies after iteration 5 is restarted
    as a fresh process tree, resumes from the iteration-4 checkpoint and ends with the
    centres of an uninterrupted run (the reference re-meshes after a
    dropped peer, app.mjs:105-117)."""
    from safetensors.torch import load_file

    common = ["--blobs", "6000,4,5", "--device", "cpu", "--n-clusters", "5", "--max-iter", "8", "--tol", "-1",
              "--checkpoint-every", "2", "--seed", "3"]
    if mode == "minibatch":   # 2 epochs of 256-row batches per rank: 24 steps, checkpoint every 2
        common = ["--blobs", "6000,4,5", "--device", "cpu", "--n-clusters", "5", "--max-iter", "2",
                  "--batch-size", "256", "--checkpoint-every", "2", "--seed", "3"]
    env = dict(os.environ, PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES="", OMP_NUM_THREADS="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    ref = subprocess.run([sys.executable, "-m", "mikmeans", "launch", "--nproc", "2", "--", "fit", *common,
                          "--checkpoint-dir", str(tmp_path / "ck_ref"), "--output", str(tmp_path / "ref")],
                         cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert ref.returncode == 0, ref.stderr[-3000:]
    env_f = dict(env, MIKMEANS_FAULT="1:5", MIKMEANS_FAULT_ONCE=str(tmp_path / "fault.once"))
    r = subprocess.run([sys.executable, "-m", "mikmeans", "launch", "--nproc", "2", "--max-restarts", "1", "--",
                        "fit", *common, "--checkpoint-dir", str(tmp_path / "ck"), "--output", str(tmp_path / "out")],
                       cwd=ROOT, env=env_f, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert (tmp_path / "fault.once").exists() and "restart 1/1" in r.stderr
    assert "resuming from" in r.stderr
    a = load_file(str(tmp_path / "ref" / "centroids.safetensors"))["centers"]
    b = load_file(str(tmp_path / "out" / "centroids.safetensors"))["centers"]
    assert torch.equal(a, b)
