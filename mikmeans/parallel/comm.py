"""Process-group wrapper: one process per GPU, RCCL over xGMI (backend "nccl" on ROCm).

This is the MI355X-native replacement of the reference's transport + replication
layers (P2PT/WebRTC gossip of Yjs CRDT updates, app.mjs:35-121): instead of
flooding state deltas to peers, every Lloyd iteration performs ONE bulk-synchronous
all-reduce of the packed f64 message ``[sums | counts | inertia | changed]``
(SURVEY.md §2.4 C1), which leaves every replica of the centroids bit-identical.
Rendezvous is env:// (MASTER_ADDR/PORT, a TCPStore) -- the analogue of the
reference's WebTorrent trackers (app.mjs:39-45); the run id plays the room code
(app.mjs:15-19).

The same code runs on CPU with the gloo backend (world_size > 1 in tests).

Host-staged mode (``staged=True``, or ``MIKMEANS_COMM=host`` in the environment): the
ranks compute on GPUs but the group is gloo, and every collective on a device tensor
goes device -> host -> gloo -> host -> device.  RCCL refuses two ranks on one GPU, so
this is how 2-4 processes share one MI355X and run the real HIP kernels through every
multi-rank code path (k-means++ owner selection, memory-plan agreement, per-rank
samplers, empty-cluster relocation) -- tests/test_gpu_multirank.py.  It is a correctness
rehearsal, not a production transport: each collective synchronises the stream, and a
host-staged step cannot be captured into a hipGraph (``capturable`` is False).
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class Comm:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    backend: str | None = None
    device: torch.device = torch.device("cpu")
    owns_group: bool = False
    staged: bool = False      # device tensors cross a gloo group through host memory

    # ---------------------------------------------------------------- setup
    @staticmethod
    def local(device=None) -> "Comm":
        dev = torch.device(device) if device is not None else torch.device("cpu")
        return Comm(device=dev)

    @staticmethod
    def from_env(device: str | None = None, timeout_s: float = 600.0, staged: bool | None = None) -> "Comm":
        """Join (or create) the default process group described by torchrun's env vars.

        ``device`` "cuda" binds LOCAL_RANK's GPU and uses RCCL; "cpu" uses gloo.
        Without WORLD_SIZE>1 in the environment this returns a single-rank Comm without a
        process group, unless ``MIKMEANS_FORCE_PG=1``: then even one rank joins a real group
        and every collective below is issued (a one-GPU rehearsal of the RCCL path).
        ``staged`` (default: ``MIKMEANS_COMM=host``): GPU ranks over a host-staged gloo group,
        rank r on GPU ``r % device_count`` -- several ranks may share one GPU.
        """
        world = int(os.environ.get("WORLD_SIZE", "1"))
        rank = int(os.environ.get("RANK", "0"))
        local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        if device is None:
            device = "cuda" if torch.cuda.is_available() else "cpu"
        if staged is None:
            staged = os.environ.get("MIKMEANS_COMM", "").lower() == "host"
        staged = bool(staged) and device.startswith("cuda")
        if staged:
            # (device_count does not initialise HIP on this image)
            idx = local_rank % max(1, torch.cuda.device_count())
            torch.cuda.set_device(idx)
            dev = torch.device("cuda", idx)
            backend = "gloo"
        elif device.startswith("cuda"):
            torch.cuda.set_device(local_rank)
            dev = torch.device("cuda", local_rank)
            backend = "nccl"
        else:
            dev = torch.device("cpu")
            backend = "gloo"
        force = os.environ.get("MIKMEANS_FORCE_PG", "0") not in ("", "0")
        if world <= 1 and not dist.is_initialized() and not force:
            return Comm(device=dev, backend=None)
        owns = False
        if not dist.is_initialized():
            kw = dict(backend=backend, timeout=datetime.timedelta(seconds=timeout_s))
            if backend == "nccl":
                kw["device_id"] = dev
            dist.init_process_group(**kw)
            owns = True
        return Comm(
            rank=dist.get_rank(),
            world=dist.get_world_size(),
            local_rank=local_rank,
            backend=dist.get_backend(),
            device=dev,
            owns_group=owns,
            staged=staged,
        )

    def close(self):
        if self.owns_group and dist.is_initialized():
            dist.destroy_process_group()
            self.owns_group = False

    def identity(self) -> dict:
        """Who this rank is (the reference's presence name + roster, app.mjs:22-27, :95)."""
        import socket

        dev = str(self.device)
        if self.device.type == "cuda" and torch.cuda.is_available():
            dev = f"{dev} ({torch.cuda.get_device_name(self.device)})"
        return {"host": socket.gethostname(), "pid": os.getpid(), "rank": self.rank, "world": self.world,
                "local_rank": self.local_rank, "backend": self.backend, "device": dev,
                "staged": self.staged}

    @property
    def distributed(self) -> bool:
        return self.world > 1

    @property
    def grouped(self) -> bool:
        """A process group exists: collectives are issued (also on a forced 1-rank group)."""
        return self.backend is not None and dist.is_initialized()

    @property
    def capturable(self) -> bool:
        """Collectives may be recorded into a hipGraph (device-side RCCL, or none at all).
        A host-staged collective copies through host memory: never capturable."""
        return not (self.staged and self.grouped)

    # ---------------------------------------------------------- collectives
    def _run(self, t: torch.Tensor, op) -> torch.Tensor:
        """``op(buffer)`` in place on ``t``: directly, or through a host copy when staged."""
        if self.staged and t.is_cuda:
            h = t.detach().to("cpu").contiguous()
            op(h)
            t.copy_(h)
        else:
            op(t)
        return t

    def allreduce_(self, t: torch.Tensor) -> torch.Tensor:
        """In-place SUM across ranks (no-op on one rank without a group)."""
        if self.grouped:
            self._run(t, lambda b: dist.all_reduce(b, op=dist.ReduceOp.SUM))
        return t

    def allreduce_max_(self, t: torch.Tensor) -> torch.Tensor:
        if self.grouped:
            self._run(t, lambda b: dist.all_reduce(b, op=dist.ReduceOp.MAX))
        return t

    def broadcast_(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        if self.grouped:
            self._run(t, lambda b: dist.broadcast(b, src=src))
        return t

    def all_gather(self, t: torch.Tensor) -> torch.Tensor:
        """Stack ``t`` from every rank: shape ``[world, *t.shape]``."""
        if not self.grouped:
            return t.unsqueeze(0).clone()
        src = t.contiguous().reshape(-1)
        host = self.staged and t.is_cuda
        if host:
            src = src.to("cpu")
        flat = torch.empty(self.world * t.numel(), dtype=t.dtype, device=src.device)
        dist.all_gather_into_tensor(flat, src)  # gloo wants flat buffers
        if host:
            flat = flat.to(t.device)
        return flat.view(self.world, *t.shape)

    def all_gather_object(self, obj):
        if self.world == 1:
            return [obj]
        out = [None] * self.world
        dist.all_gather_object(out, obj)
        return out

    def broadcast_object(self, obj, src: int = 0):
        if self.world == 1:
            return obj
        box = [obj]
        dist.broadcast_object_list(box, src=src)
        return box[0]

    def all_gather_bytes(self, data: bytes) -> list[bytes]:
        """Variable-length byte strings from every rank, as two tensor collectives
        (lengths, then a padded uint8 gather) -- no pickling of peer payloads."""
        if self.world == 1:
            return [bytes(data)]
        n = torch.tensor([len(data)], dtype=torch.int64, device=self.device)
        lens = self.all_gather(n).reshape(-1).tolist()
        buf = torch.zeros(max(max(lens), 1), dtype=torch.uint8)
        if data:
            buf[: len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8)
        allb = self.all_gather(buf.to(self.device)).cpu()
        return [allb[r, : lens[r]].numpy().tobytes() for r in range(self.world)]

    def broadcast_bytes(self, data: bytes | None, src: int = 0) -> bytes:
        if self.world == 1:
            return bytes(data or b"")
        n = torch.tensor([len(data) if self.rank == src else 0], dtype=torch.int64, device=self.device)
        self.broadcast_(n, src)
        buf = torch.zeros(max(int(n.item()), 1), dtype=torch.uint8)
        if self.rank == src and data:
            buf[: len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8)
        buf = buf.to(self.device)
        self.broadcast_(buf, src)
        return buf.cpu()[: int(n.item())].numpy().tobytes()

    def barrier(self):
        if self.grouped:
            if self.backend == "nccl":
                dist.barrier(device_ids=[self.device.index])
            else:
                dist.barrier()


_default: Comm | None = None


def get_comm() -> Comm:
    global _default
    if _default is None:
        _default = Comm.local()
    return _default


def set_comm(c: Comm) -> None:
    global _default
    _default = c
