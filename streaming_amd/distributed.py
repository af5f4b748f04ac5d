"""One process per GPU, per-GPU shard ownership, no data-path collectives.

The environment contract mirrors the reference's (``streaming/base/distributed.py:23-56``:
``RANK`` / ``WORLD_SIZE`` / ``LOCAL_RANK``). Decoding needs no exchange: a rank decodes the shards
it owns (:func:`owned_shards`); the only collectives are the benchmark's barrier and its
max-over-ranks timing reduction.
"""

from __future__ import annotations

import os
from dataclasses import dataclass

import torch
import torch.distributed as dist

__all__ = ['RankInfo', 'rank_info', 'owned_shards', 'max_over_ranks', 'sum_over_ranks']


@dataclass(frozen=True)
class RankInfo:
    rank: int
    world_size: int
    local_rank: int


def rank_info() -> RankInfo:
    return RankInfo(int(os.environ.get('RANK', 0)), int(os.environ.get('WORLD_SIZE', 1)),
                    int(os.environ.get('LOCAL_RANK', 0)))


def owned_shards(num_shards: int, rank: int, world_size: int) -> list[int]:
    """Round-robin shard ownership: shard s -> rank s % world_size (imbalance <= 1 shard)."""
    if not (0 <= rank < world_size):
        raise ValueError(f'rank {rank} outside world of {world_size}')
    return list(range(rank, num_shards, world_size))


def _reduce(value: float, op, device) -> float:
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=op)
    return float(t.item())


def max_over_ranks(value: float, device=None) -> float:
    return _reduce(value, dist.ReduceOp.MAX, device)


def sum_over_ranks(value: float, device=None) -> float:
    return _reduce(value, dist.ReduceOp.SUM, device)
