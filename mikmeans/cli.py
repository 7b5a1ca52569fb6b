"""Command line: ``python -m mikmeans <command>`` (or ``torchrun ... -m mikmeans fit`` for DP).

Commands (the reference's top-bar controls, app.mjs:240-288, as a CLI):

* ``fit``      -- k-means on a file (.npy/.safetensors/.csv) or synthetic blobs; writes a
                  checkpoint (safetensors + JSON), the flat-float ``centroids.json`` and labels
* ``predict``  -- labels of a dataset under a saved model
* ``blobs``    -- write a synthetic Gaussian-blob dataset
* ``room``     -- the trait-card game headless: seed/populate/auto-assign/dashboard/export/import
* ``session``  -- one participant of a live, replicated room session: found it (hosting the
                  rendezvous store) or join it, submit edits, leave -- the reference's tab
                  joining a room link (app.mjs:70-118)
* ``export``   -- checkpoint -> flat-float centroid JSON or room-export JSON (app.mjs:263-267)
* ``import``   -- room-export JSON -> numeric checkpoint of trait vectors (app.mjs:268-282)
* ``bench``    -- the headline benchmark (same as ``python bench.py``)
* ``launch``   -- run a command as an N-rank job with fresh-process restarts from the last
                  checkpoint (the reference's peers re-meshing after a drop, app.mjs:105-117)
* ``info``     -- device, native extension and build information
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import numpy as np
import torch


def _comm(device, timeout_s: float = 600.0):
    from .parallel import Comm, set_comm

    c = Comm.from_env(device, timeout_s=timeout_s)
    set_comm(c)
    return c


def _resume_dir(cfg):
    """``--resume auto``: the checkpoint dir when it already holds a checkpoint (a restart)."""
    from .utils.checkpoint import has_checkpoint

    if cfg.resume == "auto":
        return cfg.checkpoint_dir if cfg.checkpoint_dir and has_checkpoint(cfg.checkpoint_dir) else None
    return cfg.resume


def cmd_fit(a) -> int:
    from . import KMeans, MiniBatchKMeans
    from .config import KMeansConfig, resolve_dtype
    from .utils.io import load_points

    cfg = KMeansConfig.from_args(a)
    device = cfg.device or ("cuda" if torch.cuda.is_available() else "cpu")
    comm = _comm(device, cfg.timeout_s)
    resume = _resume_dir(cfg)
    dtype = resolve_dtype(cfg.dtype)
    if a.input:
        X, n, start = load_points(a.input, comm.rank, comm.world)
    else:
        from .data.blobs import make_blobs
        from .parallel import shard_range

        n, d, c = (int(v) for v in a.blobs.split(","))
        start, end = shard_range(n, comm.rank, comm.world)
        X = make_blobs(end - start, d, c, seed=cfg.seed, i0=start, device=comm.device, dtype=dtype)
    if cfg.batch_size > 0:
        km = MiniBatchKMeans(cfg.n_clusters, batch_size=cfg.batch_size, max_iter=cfg.max_iter, init=cfg.init,
                             dtype=dtype, device=comm.device, seed=cfg.seed, comm=comm,
                             init_sampling=cfg.init_sampling)
        if resume and comm.rank == 0:
            print(f"[mikmeans] resuming from {resume}", file=sys.stderr, flush=True)
        # batch rows are drawn by (seed, rank, step): a restart on the same world size
        # continues the interrupted fit exactly
        km.fit(X, resume_from=resume, checkpoint_every=cfg.checkpoint_every, checkpoint_dir=cfg.checkpoint_dir)
    else:
        km = KMeans.from_config(cfg, comm=comm)
        km.device = comm.device
        if resume and comm.rank == 0:
            print(f"[mikmeans] resuming from {resume}", file=sys.stderr, flush=True)
        km.fit(X, resume_from=resume)
    out = Path(a.output) if a.output else None
    if comm.rank == 0:
        rec = {"n_samples": n, "n_clusters": cfg.n_clusters, "world": comm.world}
        if hasattr(km, "inertia_"):
            rec.update(inertia=km.inertia_, n_iter=km.n_iter_, fit_time_s=round(km.fit_time_s_, 4),
                       metrics=km.metrics())
        mp = getattr(km, "memory_plan_", None)
        if mp:
            rec["memory_plan"] = {k: mp[k] for k in ("mode", "peak", "budget", "chunk_rows", "batch_rows")}
        print(json.dumps(rec, default=str))
    if out is not None:
        km.save(out)   # safetensors + state.json + flat centroids.json (mini-batch: + running counts)
        if a.save_labels and hasattr(km, "labels_"):
            lab = km.labels_
            lab = lab.cpu().numpy() if torch.is_tensor(lab) else lab
            np.save(out / f"labels.rank{comm.rank}.npy", lab.astype(np.int32), allow_pickle=False)
    comm.close()
    return 0


def cmd_predict(a) -> int:
    from . import KMeans
    from .utils.io import load_points

    comm = _comm(a.device or ("cuda" if torch.cuda.is_available() else "cpu"))
    km = KMeans.load(a.model, device=comm.device)
    X, n, start = load_points(a.input, comm.rank, comm.world)
    lab = km.predict(X.to(comm.device))
    lab = lab.cpu().numpy().astype(np.int32)
    if a.output:
        np.save(Path(a.output).with_suffix(f".rank{comm.rank}.npy") if comm.world > 1 else a.output, lab,
                allow_pickle=False)
    if comm.rank == 0:
        print(json.dumps({"n_samples": n, "counts": np.bincount(lab, minlength=km.n_clusters).tolist()}))
    comm.close()
    return 0


def cmd_blobs(a) -> int:
    from .data.blobs import make_blobs
    from .utils.io import save_points

    X, y = make_blobs(a.n, a.d, a.centers, std=a.std, seed=a.seed, return_labels=True)
    save_points(a.output, X)
    if a.labels:
        np.save(a.labels, y.numpy(), allow_pickle=False)
    print(json.dumps({"output": str(a.output), "shape": list(X.shape)}))
    return 0


def cmd_room(a) -> int:
    from .models.room import Room

    r = Room.from_json(Path(a.load).read_text(), a.room) if a.load else Room(a.room, seed=a.seed)
    if a.populate:
        r.populate_test_data()
    for name in a.centroid or []:
        r.add_centroid(name)
    if a.auto:
        r.auto_assign(seed=a.seed)
    if a.iteration is not None:
        r.set_iteration(a.iteration)
    if a.export:
        Path(a.export).write_text(r.export_json())
    if a.link is not None:
        print(r.share_link(a.link))
    if a.coin:
        print(r.coin())
    if a.d12:
        print(f"d12 \u2192 {r.d12()}")
    if a.shuffle_names:
        print("Suggested order:\n\n" + "\n".join(r.shuffled_titles()))
    d = r.dashboard()
    print("\n".join(d["chips"] + [" ".join(x for x in (row["name"], f"{row['bar_pct']}%", row["cohesion"],
                                                             row["top"], row["suggested"])) for row in d["rows"]]))
    return 0


def cmd_serve(a) -> int:
    """`mikmeans serve`: the room board and model serving over HTTP (mikmeans/serve.py)."""
    from .serve import serve

    session = None
    if a.found is not None or a.join:
        session = {"store_host": a.store_host, "store_port": a.store_port,
                   "found": a.found if a.found is not None else None, "member": a.member, "user": a.user}
    serve(a.room, a.model, host=a.host, port=a.port, device=a.device, session=session)
    return 0


def cmd_session(a) -> int:
    """A scripted participant of a live room session (parallel/elastic.py): ``--found ROOM``
    hosts the rendezvous store and starts the session, otherwise ``--join`` enters it; the
    edits given on the command line are submitted in the first round, every round prints one
    JSON status line, and all participants stop together at ``--until-round`` (the round
    counter is replicated)."""
    import datetime
    import os
    import socket
    import time

    import torch.distributed as dist

    from .parallel.elastic import ElasticRoomReplica

    store = dist.TCPStore(a.host, a.port, is_master=a.found is not None, wait_for_workers=False,
                          timeout=datetime.timedelta(seconds=a.timeout))
    member = a.member or f"{socket.gethostname()}-{os.getpid()}"
    kw = dict(user=a.user, seed=a.seed, timeout_s=a.timeout)
    if a.found is not None:
        state = Path(a.load).read_text() if a.load else None
        rep = ElasticRoomReplica.found(store, member, a.found or None, state_json=state, **kw)
    else:
        rep = ElasticRoomReplica.join(store, member, **kw)
    first = True
    while rep.round < a.until_round and not rep.left:
        if first:
            if a.populate:
                rep.populate_test_data()
            for name in a.centroid or []:
                rep.add_centroid(name)
            for spec in a.card or []:
                title, _, traits = spec.partition(":")
                rep.add_card(title, [t for t in traits.split(",") if t] or ["", ""])
            if a.auto:
                rep.auto_assign(seed=a.seed)
            first = False
        if a.leave_at is not None and rep.round >= a.leave_at:
            rep.leave()
        rep.sync()
        print(json.dumps({"member": member, "round": rep.round, "epoch": rep.epoch, "peers": rep.peers,
                          "roster": rep.roster, "left": rep.left, "digest": rep.digest()[:16]}), flush=True)
        time.sleep(a.interval)
    if a.export:
        Path(a.export).write_text(rep.room.export_json())
    return 0


def cmd_export(a) -> int:
    """Checkpoint -> flat-float centroid JSON, or a room-export JSON whose centroids
    are the model's clusters (named by their top features when a vocabulary exists)."""
    from .utils.checkpoint import load_checkpoint
    from .utils.jsjson import centroids_to_json

    ck = load_checkpoint(a.model)
    C = ck["centers"]
    if a.format == "flat":
        Path(a.output).write_text(centroids_to_json(C))
    else:
        from .models.room import Room

        r = Room(a.room or ck.get("config", {}).get("run_id"), seed_jessica=False, seed=0)
        vocab = ck.get("vocab")
        names = None
        if vocab:
            from .utils.traits import label_clusters

            names = label_clusters(C.numpy(), [1] * C.shape[0], vocab)
        r.max_centroids = max(r.max_centroids, C.shape[0])
        for k in range(C.shape[0]):
            r.add_centroid((names[k] if names and names[k] else None) or f"Centroid {k + 1}",
                           cid=f"c:{k}")
        r.set_iteration(int(ck["iteration"]))
        Path(a.output).write_text(r.export_json())
    print(json.dumps({"output": a.output, "format": a.format, "k": int(C.shape[0])}))
    return 0


def cmd_import(a) -> int:
    """Room-export JSON -> numeric model: cards become multi-hot trait vectors, the
    room's centroids seed k-means (auto_assign), the result is saved as a checkpoint."""
    from .models.room import Room
    from .utils.checkpoint import save_checkpoint
    from .utils.traits import encode_traits

    r = Room.from_json(Path(a.room).read_text())
    dash = r.auto_assign(seed=a.seed) if a.assign else r.dashboard()
    X, vocab = encode_traits(r.cards)
    cents = []
    for c in r.centroids:
        members = [i for i, card in enumerate(r.cards) if card.get("assignedTo") == c["id"]]
        cents.append(X[members].mean(0) if members else np.zeros(X.shape[1], dtype=np.float32))
    C = torch.from_numpy(np.stack(cents).astype(np.float32)) if cents else torch.zeros(0, X.shape[1])
    save_checkpoint(a.output, C, int(r.meta.get("iteration") or 0), {"run_id": r.room, "mode": r.meta.get("mode")},
                    extra={"vocab": vocab, "centroid_ids": [c["id"] for c in r.centroids],
                           "centroid_names": [c["name"] for c in r.centroids]})
    if a.save_room:
        Path(a.save_room).write_text(r.export_json())
    print("\n".join(dash["chips"]))
    return 0


def cmd_launch(a, rest) -> int:
    """``mikmeans launch --nproc N [--max-restarts R] -- <command> ...``: run a mikmeans
    command as an N-rank job (one process per GPU, RCCL) and restart it as a FRESH process
    tree when it fails; with ``--checkpoint-dir`` the restart resumes from the last
    checkpoint (``--resume auto`` is added).  This process never touches the GPU."""
    from .parallel.launch import launch_self

    if rest and rest[0] == "--":
        rest = rest[1:]
    if not rest:
        raise SystemExit("usage: mikmeans launch --nproc N [--max-restarts R] -- <command> [args]")
    if "--checkpoint-dir" in rest and "--resume" not in rest:
        rest = [*rest, "--resume", "auto"]
    return launch_self(a.nproc, ["-m", "mikmeans", *rest], max_restarts=a.max_restarts)


def cmd_bench(a, rest) -> int:
    root = Path(__file__).resolve().parent.parent
    sys.path.insert(0, str(root))
    import bench  # noqa: E402

    bench.main(rest)
    return 0


def cmd_plan(a) -> int:
    """HBM plan of a fit (parallel/memplan.py) for N rows over W ranks: resident or
    streamed, the chunk, every buffer's bytes.  Budget: --budget-gb, MIKMEANS_HBM_BYTES,
    this GPU's free memory, or else an idle MI355X (98 % of 288 GB)."""
    import os

    from .parallel import memplan, shard_sizes

    n_local = max(shard_sizes(a.n, a.world))
    if a.budget_gb:
        budget = int(a.budget_gb * 1e9)
    elif os.environ.get("MIKMEANS_HBM_BYTES") or torch.cuda.is_available():
        budget = memplan.hbm_budget()
    else:
        budget = int(memplan.HBM_BYTES * 0.98)
    try:
        if a.batch_size > 0:
            pl = memplan.plan_minibatch(n_local, a.d, a.k, a.dtype, batch_rows=a.batch_size, resident=True)
            pl.budget = budget
            if not pl.fits:
                pl = memplan.plan_minibatch(n_local, a.d, a.k, a.dtype, batch_rows=a.batch_size, resident=False)
                pl.budget = budget
        else:
            fkw = dict(budget=budget, x_on_device=False, incremental=not a.full_mstep, init=a.init)
            pl = None
            if a.algorithm == "auto":   # (KMeans' default: the bounds when they fit beside a resident shard)
                try:
                    pl = memplan.plan_fit(n_local, a.d, a.k, a.dtype, bounded=True, **fkw)
                    pl = pl if pl.mode == "resident" else None
                except memplan.HBMCapacityError:
                    pl = None
            if pl is None:
                pl = memplan.plan_fit(n_local, a.d, a.k, a.dtype, bounded=a.algorithm in ("hamerly", "elkan"),
                                      **fkw)
    except memplan.HBMCapacityError as e:
        print(json.dumps({"error": str(e)}))
        return 1
    out = pl.as_dict()
    out["summary"] = pl.summary()
    out["world"] = a.world
    print(json.dumps(out, indent=None if a.compact else 1))
    return 0


def cmd_info(a) -> int:
    from .ops import native

    info = {"torch": torch.__version__, "hip": getattr(torch.version, "hip", None),
            "gpu": torch.cuda.is_available(), "native": native.available(), "native_path": native.loaded_path()}
    if torch.cuda.is_available():
        p = torch.cuda.get_device_properties(0)
        info.update(device=p.name, arch=getattr(p, "gcnArchName", None), cus=p.multi_processor_count,
                    hbm_gb=round(p.total_memory / 1e9, 1), n_gpus=torch.cuda.device_count())
    print(json.dumps(info))
    return 0


def build_parser():
    from .config import KMeansConfig

    ap = argparse.ArgumentParser(prog="mikmeans", description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    sub = ap.add_subparsers(dest="cmd", required=True)
    f = sub.add_parser("fit", help="fit k-means")
    src = f.add_mutually_exclusive_group(required=True)
    src.add_argument("--input", help=".npy / .safetensors / .csv point matrix")
    src.add_argument("--blobs", help="synthetic data N,D,CENTERS (generated on device, per rank)")
    f.add_argument("--output", help="checkpoint directory")
    f.add_argument("--save-labels", action="store_true")
    KMeansConfig.add_arguments(f)
    p = sub.add_parser("predict", help="assign points with a saved model")
    p.add_argument("--model", required=True)
    p.add_argument("--input", required=True)
    p.add_argument("--output")
    p.add_argument("--device")
    b = sub.add_parser("blobs", help="write a synthetic dataset")
    b.add_argument("--n", type=int, required=True)
    b.add_argument("--d", type=int, required=True)
    b.add_argument("--centers", type=int, required=True)
    b.add_argument("--std", type=float, default=1.0)
    b.add_argument("--seed", type=int, default=0)
    b.add_argument("--output", required=True)
    b.add_argument("--labels")
    r = sub.add_parser("room", help="headless trait-card room")
    r.add_argument("--room")
    r.add_argument("--load", help="import a room JSON export")
    r.add_argument("--populate", action="store_true", help="add the 11 test cards")
    r.add_argument("--centroid", action="append", help="add a centroid (repeatable, max 3)")
    r.add_argument("--auto", action="store_true", help="assign cards by numeric k-means")
    r.add_argument("--iteration", type=int)
    r.add_argument("--export", help="write kmeans-room JSON here")
    r.add_argument("--seed", type=int, default=0)
    r.add_argument("--link", nargs="?", const="", default=None, metavar="BASE_URL",
                   help="print the share link (?room=<code>)")
    r.add_argument("--coin", action="store_true", help="flip a coin (Heads/Tails)")
    r.add_argument("--d12", action="store_true", help="roll a twelve-sided die")
    r.add_argument("--shuffle-names", action="store_true", help="print a shuffled order of the card titles")
    sv = sub.add_parser("serve", help="HTTP service: the room board page + JSON API, and model serving")
    sv.add_argument("--room", default=None, help="room export JSON to start from")
    sv.add_argument("--model", default=None, help="fitted model directory (KMeans.save) to serve /api/predict")
    sv.add_argument("--host", default="127.0.0.1")
    sv.add_argument("--port", type=int, default=8000)
    sv.add_argument("--device", default=None)
    # serve one member of a live replicated room session (parallel/elastic.py)
    sg = sv.add_mutually_exclusive_group()
    sg.add_argument("--found", nargs="?", const="", metavar="ROOM",
                    help="start a live session (hosts its rendezvous store) and serve it")
    sg.add_argument("--join", action="store_true", help="join a running session and serve it")
    sv.add_argument("--store-host", default="127.0.0.1", help="session rendezvous (TCPStore) host")
    sv.add_argument("--store-port", type=int, default=29555, help="session rendezvous port")
    sv.add_argument("--member", help="unique member id (default host-pid)")
    sv.add_argument("--user", help="this member's display name")
    se = sub.add_parser("session", help="one participant of a live replicated room session")
    se.add_argument("--host", default="127.0.0.1", help="rendezvous (TCPStore) host")
    se.add_argument("--port", type=int, required=True)
    g = se.add_mutually_exclusive_group(required=True)
    g.add_argument("--found", nargs="?", const="", metavar="ROOM", help="start the session (hosts the store)")
    g.add_argument("--join", action="store_true", help="join a running session")
    se.add_argument("--member", help="unique member id (default host-pid)")
    se.add_argument("--user", help="display name (the reference's presence name)")
    se.add_argument("--load", help="--found: start from a room JSON export")
    se.add_argument("--populate", action="store_true")
    se.add_argument("--centroid", action="append")
    se.add_argument("--card", action="append", metavar="TITLE:TRAIT1,TRAIT2")
    se.add_argument("--auto", action="store_true")
    se.add_argument("--until-round", type=int, default=10)
    se.add_argument("--leave-at", type=int, help="leave once the session reaches this round")
    se.add_argument("--interval", type=float, default=0.1, help="seconds between rounds")
    se.add_argument("--seed", type=int, default=0)
    se.add_argument("--timeout", type=float, default=120.0)
    se.add_argument("--export", help="write the room JSON here at the end")
    e = sub.add_parser("export", help="checkpoint -> flat centroid JSON or room-export JSON")
    e.add_argument("--model", required=True)
    e.add_argument("--format", choices=["flat", "room"], default="flat")
    e.add_argument("--room", help="room code for --format room")
    e.add_argument("--output", required=True)
    i = sub.add_parser("import", help="room-export JSON -> numeric checkpoint (trait vectors)")
    i.add_argument("--room", required=True, help="kmeans-room-*.json")
    i.add_argument("--output", required=True, help="checkpoint directory")
    i.add_argument("--assign", action="store_true", help="re-assign cards by numeric k-means first")
    i.add_argument("--save-room", help="also write the (re-assigned) room JSON")
    i.add_argument("--seed", type=int, default=0)
    sub.add_parser("bench", help="headline benchmark (args forwarded to bench.py)", add_help=False)
    sub.add_parser("launch", help="N-rank job with restarts from the last checkpoint", add_help=False)
    sub.add_parser("info", help="environment / build info")
    pl = sub.add_parser("plan", help="HBM plan of a fit: resident / streamed, chunk rows, buffer bytes")
    pl.add_argument("--n", type=int, required=True, help="total rows (over all ranks)")
    pl.add_argument("--d", type=int, required=True)
    pl.add_argument("--k", type=int, required=True)
    pl.add_argument("--world", type=int, default=1)
    pl.add_argument("--dtype", default="bfloat16")
    pl.add_argument("--init", default="k-means++")
    pl.add_argument("--batch-size", type=int, default=0, help="> 0: plan a mini-batch fit")
    pl.add_argument("--full-mstep", action="store_true", help="no incremental M-step buffers")
    pl.add_argument("--algorithm", default="auto", choices=["auto", "lloyd", "hamerly", "elkan"],
                    help="hamerly: the bounded E-step's per-row bounds too; auto: them when they fit resident")
    pl.add_argument("--budget-gb", type=float, default=None)
    pl.add_argument("--compact", action="store_true")
    return ap


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    if argv and argv[0] == "bench":
        return cmd_bench(None, argv[1:])
    if argv and argv[0] == "launch":
        la = argparse.ArgumentParser(prog="mikmeans launch", description=cmd_launch.__doc__)
        la.add_argument("--nproc", type=int, default=1, help="ranks (one per GPU)")
        la.add_argument("--max-restarts", type=int, default=0, help="fresh-process restarts after a failure")
        a, rest = la.parse_known_args(argv[1:])
        return cmd_launch(a, rest)
    a = build_parser().parse_args(argv)
    return {"fit": cmd_fit, "predict": cmd_predict, "blobs": cmd_blobs, "room": cmd_room, "session": cmd_session,
            "export": cmd_export, "import": cmd_import, "info": cmd_info, "plan": cmd_plan,
            "serve": cmd_serve}[a.cmd](a)


if __name__ == "__main__":
    sys.exit(main())
