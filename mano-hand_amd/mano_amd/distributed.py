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

import ctypes
import math
from typing import Optional, Tuple

import torch
import torch.distributed as dist

from . import _abi


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
    # `root` is a rank of `group`; torch's gather takes a global rank.
    dst = root if group is None else dist.get_global_rank(group, root)
    if shard.shape[0] != stop - start:
        raise ValueError(f"rank {rank} shard has {shard.shape[0]} rows, expected {stop - start}")
    if shard.shape[0] == per:
        send = shard.contiguous()
    else:
        send = shard.new_zeros((per,) + tuple(shard.shape[1:]))
        send[: shard.shape[0]] = shard
    if rank == root:
        full = shard.new_empty((per * world,) + tuple(shard.shape[1:]))
        dist.gather(send, gather_list=list(full.chunk(world, 0)), dst=dst, group=group)
        return full[:n_total]
    dist.gather(send, gather_list=None, dst=dst, group=group)
    return None


def gather_rows_to_root(shard: torch.Tensor, n_total: int, out: Optional[torch.Tensor] = None,
                        root: int = 0, chunk_rows: int = 32768, group=None,
                        progress=None) -> Optional[torch.Tensor]:
    """`gather_to_root` in bounded pieces, for a host-backend (gloo) group and
    shards of many GB: every rank sends its shard in chunks of `chunk_rows`
    rows through host memory (the last chunk zero-padded; every rank runs
    the same ceil(ceil(n_total / world) / chunk_rows) collectives), and root
    writes rank r's rows at shard_range(n_total, r)[0] + offset of `out` (any
    device; allocated on the shard's device when None).  Host memory per
    collective: world x chunk_rows rows on root, one chunk elsewhere.
    `progress(rows_done, rows_per_rank)` is called after each chunk."""
    world, rank = _world(group)
    start, stop = shard_range(n_total, rank, world)
    if shard.shape[0] != stop - start:
        raise ValueError(f"rank {rank} shard has {shard.shape[0]} rows, expected {stop - start}")
    if chunk_rows < 1:
        raise ValueError("chunk_rows must be positive")
    if rank == root and out is None:
        out = shard.new_empty((n_total,) + tuple(shard.shape[1:]))
    if world == 1:
        if out.data_ptr() != shard.data_ptr():
            out[start:stop].copy_(shard)
        return out
    dst = root if group is None else dist.get_global_rank(group, root)
    per = -(-n_total // world)
    ranges = [shard_range(n_total, r, world) for r in range(world)]
    row_shape = tuple(shard.shape[1:])
    for off in range(0, per, chunk_rows):
        c = min(chunk_rows, per - off)
        piece = torch.zeros((c,) + row_shape, dtype=shard.dtype)
        have = max(0, min(c, shard.shape[0] - off))
        if have:
            piece[:have].copy_(shard[off:off + have])
        if rank == root:
            got = [torch.empty_like(piece) for _ in range(world)]
            dist.gather(piece, gather_list=got, dst=dst, group=group)
            for r, (a, b) in enumerate(ranges):
                n = max(0, min(c, (b - a) - off))
                if n and not (r == rank and out[a + off].data_ptr() == shard[off].data_ptr()):
                    out[a + off:a + off + n].copy_(got[r][:n])
        else:
            dist.gather(piece, gather_list=None, dst=dst, group=group)
        if progress is not None:
            progress(off + c, per)
    return out if rank == root else None


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


class AbiGather:
    """The C-ABI gather (include/mano_hip.h mano_comm_* / mano_gather): one
    RCCL group of direct peer -> root sends over xGMI, ragged shards landing
    contiguously on root (no padding, no ring).  torch.distributed is used only
    to hand rank 0's RCCL id to the other ranks."""

    def __init__(self, device: int, group=None):
        world, rank = _world(group)
        self.world, self.rank, self.device = world, rank, device
        lib = _abi.lib()
        uid = ctypes.create_string_buffer(_abi.MANO_COMM_ID_BYTES)
        if rank == 0:
            _abi.check(lib.mano_comm_unique_id(uid))
        if dist.is_available() and dist.is_initialized():  # also a 1-rank group (bench --force-pg)
            box = [uid.raw]
            dist.broadcast_object_list(box, src=0 if group is None else dist.get_global_rank(group, 0),
                                       group=group)
            uid = ctypes.create_string_buffer(box[0], _abi.MANO_COMM_ID_BYTES)
        self._c = ctypes.c_void_p()
        _abi.check(lib.mano_comm_create(device, world, rank, uid, ctypes.byref(self._c)))

    def info(self):
        """(n_ranks, rank, device) as the RCCL communicator holds them
        (mano_comm_info): what a multi-GPU run asserts RCCL actually saw."""
        n, r, d = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        _abi.check(_abi.lib().mano_comm_info(self._c, ctypes.byref(n), ctypes.byref(r), ctypes.byref(d)))
        return n.value, r.value, d.value

    def gather(self, shard: torch.Tensor, n_total: int, root: int = 0, out: Optional[torch.Tensor] = None,
               stream=None) -> Optional[torch.Tensor]:
        """Every rank passes its `shard_range` shard (dim 0); `root` gets the
        (n_total, ...) tensor (into `out` when given), the others None."""
        start, stop = shard_range(n_total, self.rank, self.world)
        if shard.shape[0] != stop - start or not shard.is_contiguous():
            raise ValueError(f"rank {self.rank} shard must be contiguous with {stop - start} rows")
        row = math.prod(shard.shape[1:]) * shard.element_size()  # bytes per hand
        sizes = (ctypes.c_size_t * self.world)(
            *[(b - a) * row for a, b in (shard_range(n_total, r, self.world) for r in range(self.world))])
        s = stream if stream is not None else torch.cuda.current_stream(shard.device)
        full = None
        if self.rank == root:
            if out is None:
                with torch.cuda.stream(s):  # reuse ordered after the recv on `s`
                    out = torch.empty((n_total,) + tuple(shard.shape[1:]), dtype=shard.dtype,
                                      device=shard.device)
            full = out
        _abi.check(_abi.lib().mano_gather(
            self._c, ctypes.c_void_p(shard.data_ptr()), shard.shape[0] * row,
            None if full is None else ctypes.c_void_p(full.data_ptr()), sizes, root,
            ctypes.c_void_p(s.cuda_stream)))
        return full

    def allgather(self, shard: torch.Tensor, out: Optional[torch.Tensor] = None,
                  stream=None) -> torch.Tensor:
        """Every rank gets the (world * rows, ...) concatenation of all shards
        (RCCL's ring all-gather, mano_allgather; equal shards only) -- the
        comparison form for `gather`."""
        if not shard.is_contiguous():
            raise ValueError("shard must be contiguous")
        shape = (self.world * shard.shape[0],) + tuple(shard.shape[1:])
        s = stream if stream is not None else torch.cuda.current_stream(shard.device)
        if out is None:
            with torch.cuda.stream(s):
                out = torch.empty(shape, dtype=shard.dtype, device=shard.device)
        elif tuple(out.shape) != shape or not out.is_contiguous() or out.dtype != shard.dtype:
            raise ValueError(f"out must be contiguous {shard.dtype} of shape {shape}")
        _abi.check(_abi.lib().mano_allgather(
            self._c, ctypes.c_void_p(shard.data_ptr()), shard.numel() * shard.element_size(),
            ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(s.cuda_stream)))
        return out

    def close(self):
        if getattr(self, "_c", None) is not None and self._c.value:
            _abi.check(_abi.lib().mano_comm_destroy(self._c))
            self._c = None
