"""Distributed layer: process groups (RCCL over xGMI / gloo), shard planning, replication."""
from .comm import Comm, get_comm, set_comm
from .replica import RoomReplica
from .shard import ShardPlan, plan, shard_range, shard_sizes

__all__ = ["Comm", "get_comm", "set_comm", "ShardPlan", "plan", "shard_range", "shard_sizes", "RoomReplica"]
