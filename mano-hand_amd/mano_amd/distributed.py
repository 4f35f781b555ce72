"""Data-parallel sharding of a hand batch over the GPUs of one node.

The reference has no parallelism; hands are independent
(mano_np.py:79-115 has no cross-hand term), so the batch splits into
contiguous shards with NO collective on the hot path.  One process drives one
GPU (torch.distributed, backend "nccl" = RCCL on ROCm).  A collective runs only
when the caller asks for every vertex assembled on one device (`gather_to_root`,
SURVEY.md §8e config C4): RCCL gather over xGMI, or all-gather when every rank
wants the whole batch.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
import torch.distributed as dist


def shard_range(n_total: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous [start, stop) of global hand indices owned by `rank` (ceil split)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank/world {rank}/{world}")
    per = -(-n_total // world)
    start = min(rank * per, n_total)
    return start, min(start + per, n_total)


def _world(group):
    if not dist.is_available() or not dist.is_initialized():
        return 1, 0
    return dist.get_world_size(group), dist.get_rank(group)


def gather_to_root(shard: torch.Tensor, n_total: int, root: int = 0,
                   group=None) -> Optional[torch.Tensor]:
    """Assemble the per-rank shards (dim 0, `shard_range` split) on `root`.

    Every rank passes its own shard; `root` receives the (n_total, ...) tensor,
    the other ranks get None.  Shards are padded to the common ceil size so one
    fixed-size collective serves ragged splits.
    """
    world, rank = _world(group)
    if world == 1:
        return shard
    per = -(-n_total // world)
    start, stop = shard_range(n_total, rank, world)
    if shard.shape[0] != stop - start:
        raise ValueError(f"rank {rank} shard has {shard.shape[0]} rows, expected {stop - start}")
    if shard.shape[0] == per:
        send = shard.contiguous()
    else:
        send = shard.new_zeros((per,) + tuple(shard.shape[1:]))
        send[: shard.shape[0]] = shard
    if rank == root:
        full = shard.new_empty((per * world,) + tuple(shard.shape[1:]))
        dist.gather(send, gather_list=list(full.chunk(world, 0)), dst=root, group=group)
        return full[:n_total]
    dist.gather(send, gather_list=None, dst=root, group=group)
    return None


def all_gather(shard: torch.Tensor, n_total: int, group=None) -> torch.Tensor:
    """Every rank receives the (n_total, ...) concatenation of all shards."""
    world, rank = _world(group)
    if world == 1:
        return shard
    per = -(-n_total // world)
    send = shard.new_zeros((per,) + tuple(shard.shape[1:]))
    send[: shard.shape[0]] = shard
    full = shard.new_empty((per * world,) + tuple(shard.shape[1:]))
    dist.all_gather_into_tensor(full, send, group=group)
    return full[:n_total]
