"""Data-parallel sharding and the optional gather, on CPU with gloo (world size 2)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from mano_amd.distributed import all_gather, gather_to_root, shard_range


@pytest.mark.parametrize("n,world", [(0, 2), (1, 2), (7, 2), (64, 8), (65536, 8), (1000, 3)])
def test_shard_range_partitions(n, world):
    seen = []
    for r in range(world):
        a, b = shard_range(n, r, world)
        assert 0 <= a <= b <= n
        seen.extend(range(a, b))
    assert seen == list(range(n))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, n_total, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        a, b = shard_range(n_total, rank, world)
        # Per-hand values depend only on the global index (shard invariance).
        shard = torch.arange(a, b, dtype=torch.float32)[:, None, None].expand(b - a, 4, 3).contiguous()
        shard = shard + torch.tensor([0.0, 0.25, 0.5])
        full = gather_to_root(shard, n_total, root=0)
        everyone = all_gather(shard, n_total)
        q.put((rank, None if full is None else full.numpy(), everyone.numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n_total", [10, 9])
def test_gather_world2(n_total):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_total, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict()
    for _ in range(world):
        rank, full, everyone = q.get(timeout=120)
        results[rank] = (full, everyone)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    expect = np.arange(n_total, dtype=np.float32)[:, None, None] + np.array([0.0, 0.25, 0.5])
    expect = np.broadcast_to(expect, (n_total, 4, 3))
    assert results[1][0] is None
    assert np.array_equal(results[0][0], expect)
    for r in range(world):
        assert np.array_equal(results[r][1], expect)


def _subgroup_worker(rank, world, port, q):
    """Ranks 1 and 2 form a subgroup; its rank 0 (global rank 1) is the root."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        group = dist.new_group([1, 2])
        res = None
        if rank in (1, 2):
            g_rank = rank - 1
            a, b = shard_range(5, g_rank, 2)
            shard = torch.arange(a, b, dtype=torch.float32)[:, None]
            full = gather_to_root(shard, 5, root=0, group=group)
            res = None if full is None else full.numpy()
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


def test_gather_root_is_a_group_rank():
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_subgroup_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got[0] is None and got[2] is None
    assert np.array_equal(got[1][:, 0], np.arange(5, dtype=np.float32))


def _chunked_worker(rank, world, port, n_total, chunk, q):
    from mano_amd.distributed import gather_rows_to_root
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        a, b = shard_range(n_total, rank, world)
        if rank == 0:
            # root's shard computed in place in its rows of the assembled buffer
            out = torch.full((n_total, 4, 3), -1.0)
            shard = out[a:b]
            shard.copy_(torch.arange(a, b, dtype=torch.float32)[:, None, None] + torch.tensor([0.0, 0.25, 0.5]))
        else:
            out = None
            shard = torch.arange(a, b, dtype=torch.float32)[:, None, None].expand(b - a, 4, 3) + \
                torch.tensor([0.0, 0.25, 0.5])
        full = gather_rows_to_root(shard.contiguous() if rank else shard, n_total, out=out, root=0,
                                   chunk_rows=chunk)
        q.put((rank, None if full is None else full.numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n_total,world,chunk", [(10, 2, 3), (1000, 3, 64), (7, 3, 1), (16, 2, 100)])
def test_chunked_gather_rows(n_total, world, chunk):
    """bench.py's multi-GPU legs assemble C4's 40-GB batch on GPU 0 through
    gloo in bounded pieces (gather_rows_to_root): ragged shards, chunks that
    do not divide a shard, and the root's shard already in place all land
    every row where the contiguous mano_gather layout puts it."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_chunked_worker, args=(r, world, port, n_total, chunk, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    expect = np.broadcast_to(np.arange(n_total, dtype=np.float32)[:, None, None] + np.array([0.0, 0.25, 0.5]),
                             (n_total, 4, 3))
    assert all(got[r] is None for r in range(1, world))
    assert np.array_equal(got[0], expect)
