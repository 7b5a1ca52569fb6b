#!/usr/bin/env python3
"""Headline benchmark: Lloyd iterations/sec at N=1e8, D=128, K=1024, bf16 (BASELINE.json).

Driver contract: ``python bench.py --gpus N --steps K --warmup W``; for N>1 it runs
one rank per GPU (RCCL over xGMI): under ``torch.distributed.run`` it joins that job,
and started plainly it launches its own N-rank ``torch.distributed.run`` child (the
parent never touches the GPU).  By default even N=1 joins a real one-rank RCCL
process group, so every N runs the same collective path.  The
dataset is 1e8 synthetic Gaussian-blob points in total (1024 blobs, generated on
device, each rank its own contiguous row range; identical data for any world
size), centroids are K random data rows.  One timed step is one full Lloyd
iteration on every rank: MFMA assign + LDS scatter-add update + slab reduce +
f64 all-reduce + finalize.  Total work is fixed as N grows ("strong" scaling).
W untimed warmup iterations, then exactly K timed ones bracketed by a barrier and
``torch.cuda.synchronize()``; the max over ranks is reported by rank 0 as one
JSON line.  ``value`` is whole-job iterations/s; point-assignments/s and the
achieved MFMA TFLOP/s are included as extra fields.

Other BASELINE configs (own measurements, not the driver's): ``--config cfg2``
(N=1e6, D=128, K=256 fp32, one GPU), ``cfg4`` (N=1e7, D=64, K=4096: k-means++
seeding time + Lloyd it/s), ``cfg5`` (mini-batch, streamed blobs, D=256, K=512).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

METRIC = "Lloyd iterations/sec (and point-assignments/sec) at N=1e8, D=128, K=1024, 1/2/4/8 MI355X"

CONFIGS = {
    "cfg3": dict(n=100_000_000, d=128, k=1024, dtype="bfloat16", model="kmeans-lloyd N=1e8 D=128 K=1024"),
    "cfg2": dict(n=1_000_000, d=128, k=256, dtype="float32", model="kmeans-lloyd N=1e6 D=128 K=256"),
    "cfg4": dict(n=10_000_000, d=64, k=4096, dtype="bfloat16", model="kmeans-lloyd N=1e7 D=64 K=4096 k-means++"),
    "cfg5": dict(n=1_000_000_000, d=256, k=512, dtype="bfloat16", model="minibatch-kmeans N=1e9 D=256 K=512"),
}


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="cfg3", choices=sorted(CONFIGS))
    ap.add_argument("--points", "--n", dest="n", type=int, default=None, help="override total points")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--batch", type=int, default=1 << 24, help="cfg5 rows per rank per step")
    ap.add_argument("--resident", action="store_true",
                    help="cfg5: batches drawn on the device from an HBM-resident shard of stored rows")
    ap.add_argument("--shard-rows", type=int, default=None,
                    help="cfg5 --resident: rows per rank (default N/8: the W=8 shard of N=1e9, 64 GB)")
    ap.add_argument("--prefetch", action=argparse.BooleanOptionalAction, default=False,
                    help="cfg5: generate the next batch on a side stream, started between the "
                         "current batch's assign and its M-step (mikmeans/data/blobs.py kick); measured "
                         "no faster: the M-step's workgroups hold the CUs (profiles/r5_27_cfg5_*.log), and "
                         "kernel traces show no overlap even where the side stream has a hardware queue "
                         "of its own (profiles/r6_26_cfg5pf_overlap.json, r6_27_stream_probe.log)")
    ap.add_argument("--gen-norms", action=argparse.BooleanOptionalAction, default=False,
                    help="cfg5 streamed: the generator also writes the rows' |x|^2 (fused) and the "
                         "assign takes them (early prologue) instead of summing its fragments; "
                         "measured slower: assign -0.10 ms, generator +0.14 ms (profiles/r5_68_*)")
    ap.add_argument("--telemetry", action=argparse.BooleanOptionalAction, default=True,
                    help="sample the GFX clock and socket power (amdsmi, a background thread) over "
                         "the timed steps")
    ap.add_argument("--incremental", action="store_true",
                    help="incremental M-step (re-scatter changed rows only; not the headline mode)")
    ap.add_argument("--also-incremental", action=argparse.BooleanOptionalAction, default=True,
                    help="cfg3: after the timed full-M-step run, time the library default "
                         "(incremental M-step) from the same start and report it as an extra field")
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                    help="cpu: gloo rehearsal of the multi-rank path (tests; tiny --n)")
    ap.add_argument("--pg", default="force", choices=["force", "auto"],
                    help="force: even one rank joins a real process group (RCCL on GPU), so N=1 "
                         "runs the same collective path as N=8; auto: no group when WORLD_SIZE=1")
    ap.add_argument("--timeout", type=float, default=120.0,
                    help="collective timeout in seconds (a dead rank fails the job after this long)")
    ap.add_argument("--graph", default="auto", choices=["auto", "on", "off"],
                    help="replay each Lloyd iteration as one captured hipGraph (the same kernels and the RCCL "
                         "all-reduce, one launch; eager fallback if capture fails).  auto: on for one rank "
                         "(cfg2's 0.7 ms steps gain ~1 %%); off for N > 1, where the host already runs "
                         "far ahead of ~3 ms steps")
    ap.add_argument("--also-bounded", action=argparse.BooleanOptionalAction, default=True,
                    help="cfg3: also time KMeans(algorithm='hamerly')'s bounded E-step from the same start "
                         "(an extra field)")
    ap.add_argument("--kpp-sampling", default="exact", choices=["exact", "two-stage"],
                    help="cfg4 multi-rank k-means++: exact (2 collectives per centre) or two-stage (1)")
    ap.add_argument("--comm", default="rccl", choices=["rccl", "host"],
                    help="host: host-staged gloo collectives, rank r on GPU r %% device_count -- a "
                         "rehearsal of the N-rank job on fewer GPUs (N ranks may share one GPU; the "
                         "value then measures ranks, not GPUs).  rccl (default): RCCL, one rank per GPU")
    args = ap.parse_args(argv)
    if args.comm == "host":
        os.environ["MIKMEANS_COMM"] = "host"      # children of the self-launch inherit it

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # Self-launch: this parent has not touched the GPU (no HIP call yet); it starts
        # one rank per GPU as a torch.distributed.run child and exits with its code.
        from mikmeans.parallel.launch import launch_self

        return launch_self(args.gpus, [os.path.abspath(__file__), *(sys.argv[1:] if argv is None else argv)])
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if world_env != args.gpus:
        print(f"[bench] error: --gpus {args.gpus} but WORLD_SIZE={world_env}", file=sys.stderr)
        return 2
    if args.pg == "force" and world_env == 1:
        from mikmeans.parallel.launch import free_port

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(free_port()))
        os.environ.update(RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", MIKMEANS_FORCE_PG="1")

    import mikmeans
    from mikmeans.data.blobs import make_blobs, blob_centers
    from mikmeans.models.init import init_random, init_kmeanspp
    from mikmeans.models.lloyd import LloydEngine
    from mikmeans.parallel import Comm, shard_range

    cfg = dict(CONFIGS[args.config])
    if args.n and args.n != cfg["n"]:
        # (a rehearsal size: the model label says so, not the config's own N)
        m, e = f"{args.n:.0e}".split("e")
        cfg["model"] = cfg["model"].replace(cfg["model"].split()[1], f"N={m}e{int(e)}", 1)
        cfg["n"] = args.n
    comm = Comm.from_env(args.device, timeout_s=args.timeout)
    world = comm.world
    assert world == args.gpus, (world, args.gpus)
    dev = comm.device
    sync = torch.cuda.synchronize if dev.type == "cuda" else (lambda: None)
    dtype = torch.bfloat16 if cfg["dtype"] == "bfloat16" else torch.float32
    N, D, K = cfg["n"], cfg["d"], cfg["k"]
    extra = {}

    if args.config == "cfg5":
        value, ms, extra = _bench_minibatch(args, cfg, comm, dtype)
        unit = "points/s"
    else:
        s, e = shard_range(N, comm.rank, world)
        t0 = time.perf_counter()
        centers = blob_centers(K, D, 10.0, args.seed, device=dev)
        X = make_blobs(e - s, D, K, seed=args.seed, i0=s, dtype=dtype, device=dev, centers=centers)
        sync()
        extra["datagen_s"] = round(time.perf_counter() - t0, 3)
        t0 = time.perf_counter()
        if args.config == "cfg4":
            C0 = init_kmeanspp(X, D, K, N, s, comm, args.seed, sampling=args.kpp_sampling)
            extra["init_sampling"] = args.kpp_sampling
        else:
            C0 = init_random(X, D, K, N, s, comm, args.seed)
        sync()
        extra["init_s"] = round(time.perf_counter() - t0, 3)
        if args.config == "cfg4" and dev.type == "cuda":
            # k-means|| (init='k-means||'): ~2 collectives per round instead of per centre;
            # its seeding time and the potential of both seedings, reported beside the bench
            from mikmeans.models.init import init_kmeans_parallel

            # first call (kernel code objects and torch allocations loaded lazily), then the
            # seeding itself, warm
            for key in ("init_kmeans_parallel_first_call_s", "init_kmeans_parallel_s"):
                t0 = time.perf_counter()
                Ck = init_kmeans_parallel(X, D, K, N, s, comm, args.seed)
                sync()
                extra[key] = round(time.perf_counter() - t0, 3)
            pots = torch.zeros(2, dtype=torch.float64, device=dev)
            for j, Cj in enumerate((C0, Ck)):
                pots[j] = mikmeans.ops.assign(X, Cj, with_dist=True)[1].sum(dtype=torch.float64)
            comm.allreduce_(pots)
            extra["init_potential_kpp_vs_kpar"] = [float(pots[0]), float(pots[1])]
            del Ck
        if args.config == "cfg4" and world == 1 and comm.grouped and dev.type == "cuda":
            # the multi-rank owner path (all-gather of the potentials + owner sampling +
            # all-reduce of the drawn row per step) on the 1-rank RCCL group: its collective
            # overhead against the local path above, same centres
            t0 = time.perf_counter()
            C1 = init_kmeanspp(X, D, K, N, s, comm, args.seed, owner_path=True)
            sync()
            extra["init_owner_path_s"] = round(time.perf_counter() - t0, 3)
            extra["init_owner_path_same_centres"] = bool(torch.equal(C0, C1))
            # the one-all-gather-per-centre draw through the same group (same centres at W=1)
            t0 = time.perf_counter()
            C2 = init_kmeanspp(X, D, K, N, s, comm, args.seed, owner_path=True, sampling="two-stage")
            sync()
            extra["init_two_stage_s"] = round(time.perf_counter() - t0, 3)
            extra["init_two_stage_same_centres"] = bool(torch.equal(C0, C2))
        from mikmeans.parallel import memplan

        mp = memplan.plan_resident(e - s, D, K, dtype, incremental=args.incremental,
                                   init="k-means++" if args.config == "cfg4" else "random")
        extra["memory_plan"] = {"mode": mp.mode, "peak_GB": round(mp.peak / 1e9, 3),
                                "HBM_GB": round(torch.cuda.get_device_properties(dev).total_memory / 1e9, 1)
                                if dev.type == "cuda" else None}
        eng = LloydEngine(X, K, comm=comm, incremental=args.incremental).set_centers(C0)
        use_graph = args.graph == "on" or (args.graph == "auto" and world == 1)
        extra["graph"] = _capture(eng, use_graph)
        tel = {} if args.telemetry else None
        elapsed = _timed_steps(eng, comm, args.warmup, args.steps, sync, telemetry=tel)
        tel = tel or {}
        # the timed steps' mean GFX clock and socket power on rank 0 (null without amdsmi):
        # value / clock_mhz separates a kernel change from a slower box
        extra["clock_mhz"] = tel.get("clock_mhz")
        extra["power_w"] = tel.get("power_w")
        extra["telemetry"] = tel or None
        ms = elapsed * 1e3 / args.steps
        value = args.steps / elapsed
        unit = "iter/s"
        st = eng.last_stats()
        extra.update(
            assignments_per_s=value * N,
            mfma_tflops=2.0 * N * K * D * value / 1e12,
            inertia=st.inertia,
            n_changed=st.n_changed,
            # one extra, untimed, event-instrumented iteration
            phase_ms=_phase_breakdown(eng) if (eng.gpu and not args.incremental) else None,
        )
        if args.config == "cfg3" and args.also_incremental and not args.incremental and eng.gpu:
            # extras from the same start (untimed for the headline): a failure there is recorded
            # in the line instead of costing the headline its JSON
            try:
                _headline_extras(args, eng, X, K, C0, comm, sync, use_graph, N, extra)
            except Exception as exc:   # noqa: BLE001
                extra["extras_error"] = f"{type(exc).__name__}: {exc}"[:300]
    if comm.rank == 0:
        out = {
            "metric": METRIC if args.config == "cfg3" else f"{cfg['model']} ({unit})",
            "value": value,
            "unit": unit,
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,  # the reference publishes no number
            "dtype": "bf16" if dtype == torch.bfloat16 else "fp32",
            "data": "synthetic gaussian blobs (on-device Philox), random-init centroids",
            "config": {
                "model": cfg["model"],
                "global_batch": N,
                "seq_len": D,
                "n_points": N,
                "n_features": D,
                "n_clusters": K,
                "parallelism": f"dp{world}",
                **({"mstep": "incremental"} if args.incremental else {}),
            },
            "comm": {"backend": comm.backend, "world_size": comm.world, "process_group": comm.grouped,
                     **({"host_staged": True,
                         "physical_gpus": min(world, torch.cuda.device_count()) if dev.type == "cuda" else 0}
                        if comm.staged else {})},
            **extra,
        }
        print(json.dumps(out), flush=True)
    comm.close()
    return 0


def _capture(eng, want: bool):
    """hipGraph-capture the device work of a Lloyd iteration (bitwise the eager step:
    tests/test_gpu_rccl.py).  The collective stays eager between the graphs, so a rank
    may replay while another runs eagerly; a failed capture leaves the engine eager
    (``capture_error``) and is reported, never fatal."""
    if not (want and eng.gpu):
        return False
    eng.capture()
    if getattr(eng, "_graphs", None) is None:
        err = getattr(eng, "capture_error", None)
        if err:
            print(f"[bench] graph capture failed ({err}); eager steps", file=sys.stderr, flush=True)
        return {"captured": False, "error": err} if err else False
    return True



def _headline_extras(args, eng, X, K, C0, comm, sync, use_graph, N, extra):
    """The incremental M-step and bounded E-step runs reported beside the headline."""
    from mikmeans.models.lloyd import LloydEngine

    # The library default (KMeans(incremental=True)) from the same start: identical
    # E-step, the M-step re-scatters only rows whose label changed into exact int64
    # running totals.  Reported beside the headline, which stays the full M-step.
    C_full = eng.centers.clone()
    del eng
    inc = LloydEngine(X, K, comm=comm, incremental=True).set_centers(C0)
    _capture(inc, use_graph)
    el_inc = _timed_steps(inc, comm, args.warmup, args.steps, sync)
    extra["incremental_mstep"] = {
        "value": args.steps / el_inc,
        "ms_per_step": el_inc * 1e3 / args.steps,
        "assignments_per_s": args.steps / el_inc * N,
        "centres_bitwise_equal_to_full": bool(torch.equal(inc.centers, C_full)),
    }
    if args.also_bounded:
        # KMeans(algorithm="hamerly"): the bounded E-step re-assigns only the rows its
        # bounds cannot vouch for -- bitwise the full E-step's iterates.  From the same
        # start, same warm-up and step count; an extra field, not the headline.
        C_inc = inc.centers.clone()
        del inc
        bnd = LloydEngine(X, K, comm=comm, incremental=True, bounded=True).set_centers(C0)
        _capture(bnd, use_graph)
        el_b = _timed_steps(bnd, comm, args.warmup, args.steps, sync)
        extra["bounded_estep"] = {
            "value": args.steps / el_b,
            "ms_per_step": el_b * 1e3 / args.steps,
            "rows_reassigned_last_step": bnd.reassigned,
            "centres_bitwise_equal_to_full": bool(torch.equal(bnd.centers, C_inc)),
            "max_centre_diff_vs_full": float((bnd.centers - C_inc).abs().max()),
        }
        del bnd


def _timed_steps(eng, comm, warmup: int, steps: int, sync, telemetry: dict | None = None) -> float:
    """W untimed iterations, then exactly ``steps`` bracketed by barrier + device sync on
    both sides; returns the max elapsed seconds over ranks.  ``telemetry``: filled with this
    rank's mean GFX clock / socket power over the timed steps (utils/telemetry.py; a
    background amdsmi reader, no HIP calls, nothing inside the step loop)."""
    from mikmeans.utils.telemetry import ClockSampler

    for _ in range(warmup):
        eng.step()
    comm.barrier()
    sync()
    sampler = ClockSampler(comm.device.index or 0) if (telemetry is not None and comm.device.type == "cuda") else None
    if sampler is not None:
        # (outside the clock: entering takes the first amdsmi sample synchronously, ~1 ms --
        # 8 % of cfg2's timed region when it sat inside, profiles/r5_60_cfg2_*.log)
        sampler.__enter__()
    t0 = time.perf_counter()
    for _ in range(steps):
        eng.step()
    sync()
    t1 = time.perf_counter()
    if sampler is not None:
        sampler.__exit__(None, None, None)
        telemetry.update(sampler.summary() or {"error": sampler.error or "no samples"})
    comm.barrier()
    el = torch.tensor([t1 - t0], dtype=torch.float64, device=comm.device)
    comm.allreduce_max_(el)
    return float(el.item())


def _phase_breakdown(eng, reps: int = 3) -> dict:
    """Per-phase device time of a Lloyd iteration (rank-local; after the timed region): the
    median of ``reps`` event-instrumented eager iterations, each phase bracketed alone."""
    import statistics

    C = eng._C
    names = ["assign", "update", "reduce", "allreduce", "finalize"]
    runs = {n: [] for n in names}
    for _ in range(reps):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(6)]
        ev[0].record()
        eng.pk.assign(eng.X, eng.xn, eng.labels, eng.mind, eng.slots, True)
        ev[1].record()
        C.update(eng.X, eng.labels, eng.K, eng.slab, eng.cnt_slab, eng.n_chunks, eng.weights, eng.col_exp,
                 eng.cnt_exp, False)
        ev[2].record()
        C.reduce(eng.slab, eng.cnt_slab, eng.n_chunks, eng.K, eng.Dp, eng.slots, eng.packed, eng.col_exp,
                 eng.cnt_exp)
        ev[3].record()
        eng.comm.allreduce_(eng.packed)
        ev[4].record()
        eng.pk.finalize(1, eng.packed, eng.C, eng.Cnew, eng.frozen, None, eng.shift, eng.counts)
        ev[5].record()
        torch.cuda.synchronize()
        for i, n in enumerate(names):
            runs[n].append(ev[i].elapsed_time(ev[i + 1]))
    return {n: round(statistics.median(v), 4) for n, v in runs.items()}


def _bench_minibatch(args, cfg, comm, dtype):
    """cfg5: mini-batch k-means, D=256, K=512, 2^24 rows per rank per step.

    Default: every batch is a fresh slice of the N=1e9-row blob dataset generated on the
    device (the stream covers distinct rows).  ``--resident``: every rank holds its shard of
    a stored dataset in HBM (``--shard-rows``, default the W=8 shard of N=1e9: 1.25e8 rows,
    64 GB -- at W<8 a rehearsal of one W=8 rank) and each step draws its batch on the device
    (Philox keyed by (seed, rank, step), csrc/rows.hip).  Both report the whole step's
    points/s and, split by device events inside the timed steps, ``gen_ms`` (generating /
    gathering the batch) and ``kmeans_ms`` (assign + M-step + reduce + all-reduce + finalize)."""
    from mikmeans.data.blobs import BlobStream, blob_centers, make_blobs
    from mikmeans.models.init import init_random
    from mikmeans.models.minibatch import MiniBatchEngine
    from mikmeans.ops import col_stats, native
    from mikmeans.parallel import memplan

    N, D, K = cfg["n"], cfg["d"], cfg["k"]
    b = args.batch
    dev = comm.device
    extra = {"batch_per_rank": b}
    if args.resident:
        S = args.shard_rows or -(-N // 8)
        plan = memplan.plan_minibatch(S, D, K, dtype, batch_rows=b, resident=True)
        plan.budget = memplan.hbm_budget(dev)
        extra["memory_plan"] = {"mode": plan.mode, "peak_GB": round(plan.peak / 1e9, 3),
                                "budget_GB": round(plan.budget / 1e9, 3), "shard_rows": S}
        if not plan.fits:
            raise SystemExit(f"[bench] resident shard does not fit: {plan.summary()}")
        centers = blob_centers(K, D, 10.0, args.seed, device=dev)
        X = torch.empty((S, D), dtype=dtype, device=dev)
        step_rows = 1 << 24
        for i in range(0, S, step_rows):   # rank r holds global rows [r*S, (r+1)*S)
            make_blobs(min(step_rows, S - i), D, K, seed=args.seed, i0=comm.rank * S + i, dtype=dtype,
                       device=dev, centers=centers, out=X[i : i + step_rows])
        C = native.require()
        rows = torch.empty(b, dtype=torch.int64, device=dev)
        eng = MiniBatchEngine(K, D, b, dtype=dtype, device=dev, comm=comm)
        eng.set_bound(col_stats(X, stats=False).absmax)
        state = {"step": 0}

        def gen():   # the step's Philox row draws; the assign / M-step read X[rows] in place
            C.sample_index(S, b, args.seed, comm.rank, state["step"], rows)
            state["step"] += 1
            return X, rows
        extra["data_bytes_per_rank"] = S * D * X.element_size()
    else:
        stream = BlobStream(N, D, K, b, seed=args.seed, dtype=dtype, device=dev, rank=comm.rank,
                            world=comm.world, with_norms=args.gen_norms,  # (fused |x|^2 for the assign)
                            prefetch=args.prefetch)  # batch j+1 generated on a side stream during step j
        # the generator's value bound fixes the fixed-point scales up front (no per-step clamp check)
        eng = MiniBatchEngine(K, D, b, dtype=dtype, device=dev, comm=comm, value_bound=stream.value_bound)
        if args.prefetch:
            eng.after_assign = stream.kick   # batch j+1's generator overlaps batch j's M-step

        extra["gen_norms"] = bool(args.gen_norms)

        def gen():
            Xb = next(stream)
            return Xb, stream.last_norms
    step = eng.partial_fit_rows if args.resident else eng.partial_fit
    first, r0 = gen()
    first = first[r0] if args.resident else first
    eng.set_centers(init_random(first, D, K, b * comm.world, comm.rank * b, comm, args.seed))
    del first
    for _ in range(args.warmup):
        step(*gen())
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True),
           torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    comm.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        ev[i][0].record()
        Xb, nb = gen()
        ev[i][1].record()
        step(Xb, nb)
        ev[i][2].record()
    torch.cuda.synchronize()
    comm.barrier()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    comm.allreduce_max_(el)
    elapsed = float(el.item())
    gen_ms = sum(a.elapsed_time(m) for a, m, _ in ev) / args.steps
    km_ms = sum(m.elapsed_time(z) for _, m, z in ev) / args.steps
    t = torch.tensor([gen_ms, km_ms], dtype=torch.float64, device=dev)
    comm.allreduce_max_(t)
    gen_ms, km_ms = float(t[0]), float(t[1])
    pts = args.steps * b * comm.world
    extra.update(mode="resident" if args.resident else "stream", steps_cover_points=pts,
                 gen_ms=round(gen_ms, 4), kmeans_ms=round(km_ms, 4),
                 kmeans_points_per_s=b * comm.world / (km_ms * 1e-3),
                 batch_inertia=eng.last_batch_inertia())
    return pts / elapsed, elapsed * 1e3 / args.steps, extra


if __name__ == "__main__":
    sys.exit(main())
