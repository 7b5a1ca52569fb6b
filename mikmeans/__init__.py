"""mikmeans — an MI355X-native k-means framework (PyTorch-ROCm + gfx950 HIP kernels + RCCL).

Capabilities of the reference ``schusto/k-means-demo`` (a collaborative,
human-in-the-loop k-means classroom game) rebuilt as a GPU engine:

* :class:`KMeans` / :func:`fit` / :func:`predict` -- Lloyd k-means whose E-step is a
  hand-written MFMA kernel and whose M-step is an LDS scatter-add kernel;
* :class:`MiniBatchKMeans` -- Sculley mini-batch over device-generated streams;
* :func:`kmeans_plusplus` -- k-means++ seeding on the same kernels;
* data-parallel over one process per GPU with RCCL all-reduce (:mod:`mikmeans.parallel`);
* the reference's trait-card rooms, dashboard metrics and byte-exact JSON export
  (:mod:`mikmeans.models.room`, :mod:`mikmeans.utils`).
"""
import torch  # noqa: F401  -- torch's HIP runtime must be loaded before mikmeans._C

from .api import KMeans, MiniBatchKMeans, fit, fit_predict, kmeans_plusplus, predict
from .config import KMeansConfig
from .parallel import Comm

__version__ = "0.1.0"


def init(device: str | None = None, *, timeout_s: float = 600.0, verbose: bool = False) -> Comm:
    """Bootstrap a process (the reference's init(), app.mjs:579-589): pick the device,
    join the torchrun process group (RCCL on GPUs, gloo on CPUs), load the native
    extension (fails loudly on a GPU box without it) and make the Comm the default."""
    from .ops import native
    from .parallel import set_comm

    comm = Comm.from_env(device, timeout_s=timeout_s)
    set_comm(comm)
    if comm.device.type == "cuda":
        native.require()
    if verbose:
        import json

        roster = [json.loads(b) for b in comm.all_gather_bytes(json.dumps(comm.identity()).encode())]
        if comm.rank == 0:
            for r in roster:
                print(f"[mikmeans] rank {r['rank']}/{r['world']} {r['host']} pid {r['pid']} {r['device']}",
                      flush=True)
    return comm


__all__ = ["KMeans", "MiniBatchKMeans", "fit", "predict", "fit_predict", "kmeans_plusplus",
           "KMeansConfig", "Comm", "init", "__version__"]
