"""Data-parallel shard planning for 288 GB-HBM3E GPUs.

Points are split into contiguous, balanced row ranges (rank r owns
``[start_r, end_r)``); centroids are replicated.  :func:`plan` sizes the
per-rank resident set (points + labels + norms + kernel workspace) against the
HBM budget and tells the caller whether a full-batch Lloyd fit fits or whether
the run must stream mini-batches (BASELINE config 5: N=1e9, D=256 bf16 is 512 GB,
over one GPU's 288 GB but 64 GB per rank at W=8).
"""
from __future__ import annotations

from dataclasses import asdict, dataclass

HBM_BYTES = 288 * 10**9          # MI355X HBM3E per GPU (spec)
HBM_USABLE_FRACTION = 0.90       # leave room for the runtime / RCCL buffers


# Shard boundaries fall on multiples of this many rows: the bf16 assign kernel folds one
# seed offset per workgroup of 128..512 points into its keys (csrc/assign16.hip; every
# workgroup size divides 1536), so aligned shards give every point the same workgroup --
# and the same near-tie resolution -- on any world size.
ROW_ALIGN = 1536


def shard_range(n: int, rank: int, world: int, align: int = ROW_ALIGN) -> tuple[int, int]:
    """Balanced contiguous split in units of ``align`` rows (the first ranks get one unit
    more; only the last shard may end off the grid)."""
    units = -(-n // align)
    base, rem = divmod(units, world)
    u0 = rank * base + min(rank, rem)
    u1 = u0 + base + (1 if rank < rem else 0)
    return min(n, u0 * align), min(n, u1 * align)


def shard_sizes(n: int, world: int, align: int = ROW_ALIGN) -> list[int]:
    return [shard_range(n, r, world, align)[1] - shard_range(n, r, world, align)[0] for r in range(world)]


@dataclass
class ShardPlan:
    n_global: int
    world: int
    rows_per_rank: int
    bytes_points: int
    bytes_aux: int
    bytes_workspace: int
    bytes_total: int
    hbm_budget: int
    fits: bool
    batch_rows: int  # rows per streamed mini-batch when it does not fit (0 = full batch)

    def as_dict(self):
        return asdict(self)


def plan(n: int, d: int, k: int, world: int = 1, itemsize: int = 2,
         hbm_bytes: int = HBM_BYTES, usable: float = HBM_USABLE_FRACTION,
         update_chunks: int = 64) -> ShardPlan:
    rows = -(-n // world)
    pts = rows * d * itemsize
    aux = rows * (4 + 4 + 4)                      # labels + |x|^2 + distance
    ws = update_chunks * k * d * 4 + k * d * 8 * 3 + (1 << 20)   # slabs + packed + centroids
    total = pts + aux + ws
    budget = int(hbm_bytes * usable)
    fits = total <= budget
    batch = 0
    if not fits:
        per_row = d * itemsize + 12
        batch = max(1, (budget - ws) // (4 * per_row))   # 4 batches in flight worth of headroom
    return ShardPlan(n, world, rows, pts, aux, ws, total, budget, fits, int(batch))
