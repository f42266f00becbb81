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


class BucketedGradAllReduce:
    """Gradient averaging overlapped with the backward pass (batch-DP training).

    Parameters are grouped, in reverse registration order (roughly the order backward produces
    their gradients), into buckets of about `bucket_mb` MB.  A post-accumulate-grad hook per
    parameter copies the fresh gradient into its bucket's flat buffer; once a bucket is complete
    AND every bucket before it has been launched, its all-reduce is launched asynchronously (RCCL
    runs it on its own stream, ordered after the producing kernels) while the rest of the backward
    pass is still being computed.  Launching strictly in bucket order keeps every rank's sequence
    of collectives identical even if the ranks' graphs produce gradients in different orders.
    `finish()` launches what is left, waits, divides by the world size and points every `p.grad`
    at its slice of the averaged buffer.  Same result as `allreduce_grads_` (one flat bucket after
    backward); the 412 MB of FiLM-prior gradients no longer serialise behind the backward pass.

    Gradient presence: each bucket carries one extra slot per parameter (1 if this rank produced
    a gradient for it, summed by the same all-reduce).  A parameter no rank produced a gradient for
    keeps `p.grad = None` — as in a single-process run, where torch.optim.Adam (and the fused Adam)
    then skips it; one that only some ranks produced is averaged with zeros from the others (the
    global-batch mean).

    Usage per step: ``opt.zero_grad(set_to_none=True); loss.backward(); ar.finish(); opt.step()``.
    """

    def __init__(self, params, bucket_mb: float = 25.0, group=None) -> None:
        self.group = group
        self.params = [p for p in params if p.requires_grad]
        self.world = dist.get_world_size(group) if (dist.is_available() and dist.is_initialized()) else 1
        self.buckets = []  # (params, flat buffer incl. presence slots, n data elements)
        self.where = {}  # id(param) -> (bucket index, offset, index within the bucket)
        cur, cur_bytes = [], 0
        for p in reversed(self.params):
            cur.append(p)
            cur_bytes += p.numel() * p.element_size()
            if cur_bytes >= bucket_mb * 1e6:
                self._add_bucket(cur)
                cur, cur_bytes = [], 0
        if cur:
            self._add_bucket(cur)
        self.pending = [0] * len(self.buckets)
        self.works = [None] * len(self.buckets)
        self.next_launch = 0
        self.hooks = []
        if self.world > 1:
            for p in self.params:
                self.hooks.append(p.register_post_accumulate_grad_hook(self._on_grad))

    def _add_bucket(self, ps) -> None:
        n = sum(p.numel() for p in ps)
        flat = torch.zeros(n + len(ps), dtype=ps[0].dtype, device=ps[0].device)
        off = 0
        bi = len(self.buckets)
        for j, p in enumerate(ps):
            self.where[id(p)] = (bi, off, j)
            off += p.numel()
        self.buckets.append((ps, flat, n))

    def _launch(self, bi) -> None:
        self.works[bi] = dist.all_reduce(self.buckets[bi][1], group=self.group, async_op=True)

    def _launch_ready(self) -> None:
        while (self.next_launch < len(self.buckets)
               and self.pending[self.next_launch] == len(self.buckets[self.next_launch][0])):
            self._launch(self.next_launch)
            self.next_launch += 1

    def _on_grad(self, p) -> None:
        bi, off, j = self.where[id(p)]
        ps, flat, n = self.buckets[bi]
        flat[off:off + p.numel()].copy_(p.grad.reshape(-1))
        flat[n + j] = 1.0
        self.pending[bi] += 1
        self._launch_ready()

    def finish(self) -> None:
        if self.world <= 1:
            return
        missing = set()
        for bi in range(self.next_launch, len(self.buckets)):
            ps, flat, n = self.buckets[bi]
            for j, p in enumerate(ps):
                if p.grad is None:  # no gradient on this rank: zeros in its slot, presence 0
                    _, off, _ = self.where[id(p)]
                    flat[off:off + p.numel()].zero_()
                    flat[n + j] = 0.0
                    missing.add(id(p))
            self._launch(bi)
        for bi, (ps, flat, n) in enumerate(self.buckets):
            self.works[bi].wait()
            flat[:n].div_(self.world)
        # Only a parameter without a local gradient needs the global count (one host read, and
        # none at all in the common step where every parameter got a gradient on this rank).
        counts = {}
        if missing:
            for ps, flat, n in self.buckets:
                c = flat[n:].cpu().tolist()
                counts.update({id(p): c[j] for j, p in enumerate(ps) if id(p) in missing})
        for bi, (ps, flat, n) in enumerate(self.buckets):
            for p in ps:
                _, off, _ = self.where[id(p)]
                keep = id(p) not in missing or counts[id(p)] > 0
                p.grad = flat[off:off + p.numel()].view_as(p) if keep else None
            self.pending[bi] = 0
            self.works[bi] = None
        self.next_launch = 0

    def remove(self) -> None:
        for h in self.hooks:
            h.remove()
        self.hooks = []
