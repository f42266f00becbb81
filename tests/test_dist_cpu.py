"""CPU, world_size 2 over gloo: the sharding / gather / gradient-average logic of the N>1 path."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from toycrystals_amd.dist import allreduce_grads_, gather_shards, rank_seed, shard_range


@pytest.mark.parametrize("n,world", [(128, 1), (128, 2), (128, 8), (37, 4), (3, 8), (0, 2)])
def test_shard_range_partitions(n, world):
    seen = []
    for r in range(world):
        s, e = shard_range(n, r, world)
        assert 0 <= s <= e <= n
        seen.extend(range(s, e))
    assert seen == list(range(n))
    sizes = [shard_range(n, r, world)[1] - shard_range(n, r, world)[0] for r in range(world)]
    assert max(sizes) - min(sizes) <= 1


def test_rank_seeds_distinct():
    assert len({rank_seed(7, r) for r in range(64)}) == 64


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        s, e = shard_range(n, rank, world)
        full = torch.arange(n * 6, dtype=torch.float32).reshape(n, 1, 2, 3)
        got = gather_shards(full[s:e].clone(), n)
        ok_gather = torch.equal(got, full)
        # gradient average: rank r holds grad = r+1 -> mean = (world+1)/2
        p = torch.nn.Parameter(torch.zeros(5, 3))
        p.grad = torch.full((5, 3), float(rank + 1))
        allreduce_grads_([p])
        ok_grad = torch.allclose(p.grad, torch.full((5, 3), (world + 1) / 2))
        # max-over-ranks timing reduction used by bench.py
        t = torch.tensor([float(rank)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        q.put((rank, ok_gather, ok_grad, float(t.item())))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n", [128, 37])
def test_gloo_world2_gather_and_grad_average(n):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ok_gather, ok_grad, tmax in res:
        assert ok_gather and ok_grad and tmax == world - 1
