"""Instance sharding across GPUs: one process per GPU, each
rank owns a contiguous block of instance ids and generates its inputs on its
own device, so the data path has no collective.  The only collectives are the
bench's barrier and max-over-ranks wall time (and a sum of per-rank rates)."""
from __future__ import annotations

import torch
import torch.distributed as dist


def instance_block(rank: int, world: int, per_rank: int) -> range:
    """Global instance ids owned by `rank` (weak scaling: per_rank fixed)."""
    if not 0 <= rank < world:
        raise ValueError("rank out of range")
    return range(rank * per_rank, (rank + 1) * per_rank)


def partition(n_total: int, rank: int, world: int) -> range:
    """Strong-scaling split of n_total instances: instance i -> rank floor(i*world/n)."""
    lo = (rank * n_total + world - 1) // world
    hi = ((rank + 1) * n_total + world - 1) // world
    return range(lo, hi)


def max_over_ranks(x: float, device=None) -> float:
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(x: float, device=None) -> float:
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t)
    return float(t.item())
