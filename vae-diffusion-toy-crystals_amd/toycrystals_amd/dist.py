"""Data-parallel helpers (one process per GPU, torch.distributed; backend "nccl" is RCCL on ROCm).

Sampling shards over independent images (GroupNorm is per sample, CFG pairs stay on one rank),
so the data path has no collective: each rank samples a contiguous slice of the batch with its
own noise stream; `gather_shards` optionally collects the images (a B*16 KB all-gather at the
end).  SURVEY.md §8(e).
"""
from __future__ import annotations

import os
from typing import Optional, Tuple

import torch
import torch.distributed as dist


def rank_world() -> Tuple[int, int]:
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1"))


def shard_range(n: int, rank: int, world: int) -> Tuple[int, int]:
    """Balanced contiguous split of [0, n): the first n % world ranks get one extra item."""
    if world <= 0 or not (0 <= rank < world):
        raise ValueError(f"bad rank/world {rank}/{world}")
    q, r = divmod(n, world)
    start = rank * q + min(rank, r)
    return start, start + q + (1 if rank < r else 0)


def rank_seed(base_seed: int, rank: int) -> int:
    """Distinct Philox key per rank (64-bit golden-ratio stride)."""
    return (base_seed + 0x9E3779B97F4A7C15 * (rank + 1)) & ((1 << 63) - 1)


def gather_shards(local: torch.Tensor, n_total: int, group=None) -> torch.Tensor:
    """All-gather variable-size leading-dim shards (ranks hold shard_range slices in rank order)."""
    world = dist.get_world_size(group)
    per = -(-n_total // world)
    pad = torch.zeros((per,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    pad[: local.shape[0]] = local
    bufs = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(bufs, pad, group=group)
    parts = []
    for r in range(world):
        s, e = shard_range(n_total, r, world)
        parts.append(bufs[r][: e - s])
    return torch.cat(parts, 0)


def sample_sharded(sampler, model, sde, y_cat: torch.Tensor, y_cont: torch.Tensor, img_shape, *,
                   base_seed: int = 0, gather: bool = True, **kw) -> torch.Tensor:
    """Run `sampler` (e.g. sample_reverse_sde_euler_maruyama) on this rank's slice of the batch."""
    rank, world = rank_world()
    B = img_shape[0]
    s, e = shard_range(B, rank, world)
    local = sampler(model, sde, y_cat[s:e], y_cont[s:e], (e - s,) + tuple(img_shape[1:]),
                    seed=rank_seed(base_seed, rank), **kw)
    if gather and world > 1:
        return gather_shards(local, B)
    return local


def allreduce_grads_(params, group=None) -> None:
    """Average gradients across ranks with one flat bucket (batch-DP training step)."""
    grads = [p.grad for p in params if p.grad is not None]
    if not grads or not (dist.is_available() and dist.is_initialized()):
        return
    world = dist.get_world_size(group)
    flat = torch.cat([g.reshape(-1) for g in grads])
    dist.all_reduce(flat, group=group)
    flat.div_(world)
    off = 0
    for g in grads:
        n = g.numel()
        g.copy_(flat[off:off + n].view_as(g))
        off += n
