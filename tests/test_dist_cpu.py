"""CPU, world_size 2 over gloo: the sharding / gather / gradient-average logic of the N>1 path."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from toycrystals_amd.dist import BucketedGradAllReduce, allreduce_grads_, gather_shards, rank_seed, shard_range


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


def _bucket_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.manual_seed(0)
        model = torch.nn.Sequential(torch.nn.Linear(16, 64), torch.nn.SiLU(), torch.nn.Linear(64, 64),
                                    torch.nn.SiLU(), torch.nn.Linear(64, 4))
        ref = [p.detach().clone() for p in model.parameters()]
        ar = BucketedGradAllReduce(model.parameters(), bucket_mb=0.0005)  # three buckets
        assert len(ar.buckets) >= 3, len(ar.buckets)
        res = []
        for step in range(2):
            g = torch.Generator().manual_seed(100 * step + rank)
            x = torch.randn(8, 16, generator=g)
            if step == 0:  # a step begun without zero_grad(): the hooks adopt the fresh gradients
                for p in model.parameters():
                    p.grad = None
            else:  # gradient-as-bucket-view: autograd accumulates straight into the buckets
                ar.zero_grad()
                flats = [f for _, f, _ in ar.buckets]
                in_bucket = all(any(f.data_ptr() <= p.grad.data_ptr() < f.data_ptr() + f.numel() * 4 for f in flats)
                                for p in model.parameters())
                if not in_bucket:
                    raise AssertionError("zero_grad() did not point the gradients into the buckets")
            model(x).square().mean().backward()
            ar.finish()
            got = [p.grad.clone() for p in model.parameters()]
            # the same step with the flat post-backward all-reduce
            for p in model.parameters():
                p.grad = None
            ar.remove()
            model(x).square().mean().backward()
            allreduce_grads_(list(model.parameters()))
            want = [p.grad.clone() for p in model.parameters()]
            ar = BucketedGradAllReduce(model.parameters(), bucket_mb=0.0005)
            res.append(all(torch.allclose(a, b, atol=1e-7, rtol=1e-6) for a, b in zip(got, want)))
        unchanged = all(torch.equal(a, b.detach()) for a, b in zip(ref, model.parameters()))
        q.put((rank, all(res), unchanged))
    except Exception as e:  # report instead of leaving the parent waiting on the queue
        q.put((rank, False, repr(e)))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_bucketed_grad_allreduce_matches_flat():
    """BucketedGradAllReduce (hooks launch each bucket's all-reduce during backward) averages the
    gradients exactly as the flat post-backward all-reduce does, over two steps."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bucket_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ok, unchanged in res:
        assert ok and unchanged is True, (rank, ok, unchanged)


def _presence_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        used = torch.nn.Parameter(torch.ones(4))
        some = torch.nn.Parameter(torch.ones(3))    # gets a gradient on rank 0 only
        never = torch.nn.Parameter(torch.ones(5))   # no rank produces a gradient
        ar = BucketedGradAllReduce([used, some, never], bucket_mb=1e-6)  # one bucket per parameter
        ok = True
        # step 0 from grad None, step 1 from zero_grad()'s bucket views, step 2 from grads set to
        # None again WITHOUT zero_grad() (opt.zero_grad(set_to_none=True)): the buckets still hold
        # step 1's averages, which must not leak into the slot of a parameter this rank skipped
        for step in range(3):
            if step == 1:
                ar.zero_grad()
            elif step == 2:
                for p in (used, some, never):
                    p.grad = None
            loss = (used * (rank + 1)).sum()
            if rank == 0:
                loss = loss + (some * 4.0).sum()
            loss.backward()
            ar.finish()
            ok = ok and (torch.allclose(used.grad, torch.full((4,), (1 + world) / 2))
                         and torch.allclose(some.grad, torch.full((3,), 4.0 / world)) and never.grad is None)
        q.put((rank, ok, ""))
    except Exception as e:  # report instead of leaving the parent waiting on the queue
        q.put((rank, False, repr(e)))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_grad_presence():
    """A parameter no rank produced a gradient for keeps grad None (Adam skips it, as in one
    process); one produced on some ranks only is averaged with zeros (the global-batch mean)."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_presence_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ok, err in res:
        assert ok, (rank, err)
