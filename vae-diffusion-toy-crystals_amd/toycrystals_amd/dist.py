"""Data-parallel helpers (one process per GPU, torch.distributed; backend "nccl" is RCCL on ROCm).

Sampling shards over independent images (GroupNorm is per sample, CFG pairs stay on one rank),
so the data path has no collective: each rank samples a contiguous slice of the batch, with the
ONE seed of the whole batch and its slice's Philox element offset, so an N-rank run produces the
1-rank images bit for bit; `gather_shards` optionally collects them (a B*16 KB all-gather at the
end).  Training is batch-DP with bucketed gradient all-reduces (`BucketedGradAllReduce`).
SURVEY.md §8(e).

Backend: "nccl" (RCCL over xGMI) unless TCX_DIST_BACKEND overrides it.  "gloo" lets several ranks
share ONE GPU (RCCL refuses two ranks per device), which is how the world-2 tests run the real
training scripts on a one-GPU box; gloo collectives on device tensors are staged through host
memory here (`all_reduce_`, `broadcast_`, `all_gather_`), so the data path is the same code.
"""
from __future__ import annotations

import os
from typing import Optional, Tuple

import torch
import torch.distributed as dist


def dist_backend() -> str:
    """The process-group backend of this job: TCX_DIST_BACKEND, default "nccl" (RCCL)."""
    b = os.environ.get("TCX_DIST_BACKEND", "nccl").strip().lower()
    if b not in ("nccl", "gloo"):
        raise ValueError(f"TCX_DIST_BACKEND must be nccl or gloo, got {b!r}")
    return b


def dp_forced() -> bool:
    """TCX_DP_FORCE=1: run the data-parallel machinery (process group, bucketed collectives) even at
    world size 1, so a one-GPU box executes the RCCL path the 8-GPU run takes (communicator init with
    device_id, async device-bucket collectives, Work.wait) and can compare it bit for bit with the
    non-DP run."""
    return os.environ.get("TCX_DP_FORCE", "0") == "1"


def dp_active(group=None) -> bool:
    """True when gradient collectives must run: an initialised process group of world > 1, or any
    initialised group under TCX_DP_FORCE=1."""
    if not (dist.is_available() and dist.is_initialized()):
        return False
    return dist.get_world_size(group) > 1 or dp_forced()


def local_device(local_rank: int) -> torch.device:
    """This rank's GPU.  Under gloo several ranks may share one device (ranks map round-robin onto
    the visible GPUs); RCCL needs one GPU per rank."""
    n = torch.cuda.device_count()
    if n < 1:
        raise SystemExit("no GPU visible: this build runs on the MI355X only")
    if dist_backend() == "nccl" and local_rank >= n:
        raise SystemExit(f"LOCAL_RANK {local_rank} but only {n} GPU(s): RCCL needs one GPU per rank "
                         f"(TCX_DIST_BACKEND=gloo shares a GPU between ranks)")
    return torch.device("cuda", local_rank % n)


def _host_staged(t: torch.Tensor, group=None) -> bool:
    return t.is_cuda and dist.get_backend(group) == "gloo"


class _Done:
    """Completed-work handle for a collective that ran synchronously."""

    def wait(self) -> bool:
        return True


def all_reduce_(t: torch.Tensor, op=None, group=None, async_op: bool = False):
    """In-place all-reduce (sum by default) of a device tensor on either backend."""
    op = dist.ReduceOp.SUM if op is None else op
    if _host_staged(t, group):
        h = t.detach().cpu()
        dist.all_reduce(h, op=op, group=group)
        t.copy_(h)
        return _Done() if async_op else None
    return dist.all_reduce(t, op=op, group=group, async_op=async_op)


def broadcast_(t: torch.Tensor, src: int = 0, group=None) -> None:
    if _host_staged(t, group):
        h = t.detach().cpu()
        dist.broadcast(h, src=src, group=group)
        t.copy_(h)
        return
    dist.broadcast(t, src=src, group=group)


def all_gather_(bufs, t: torch.Tensor, group=None) -> None:
    if _host_staged(t, group):
        hs = [torch.empty(b.shape, dtype=b.dtype) for b in bufs]
        dist.all_gather(hs, t.detach().cpu(), group=group)
        for b, h in zip(bufs, hs):
            b.copy_(h)
        return
    dist.all_gather(bufs, t, group=group)


def reduce_scatter_(out: torch.Tensor, t: torch.Tensor, group=None, async_op: bool = False):
    """out = this rank's 1/world slice of the element-wise sum of `t` over ranks (t.numel() =
    world * out.numel()); gloo stages device tensors through host memory (synchronous handle)."""
    if _host_staged(t, group):
        h = torch.empty(out.shape, dtype=out.dtype)
        dist.reduce_scatter_tensor(h, t.detach().cpu(), group=group)
        out.copy_(h)
        return _Done() if async_op else None
    return dist.reduce_scatter_tensor(out, t, group=group, async_op=async_op)


def all_gather_into_(out: torch.Tensor, t: torch.Tensor, group=None, async_op: bool = False):
    """out = concat over ranks of each rank's `t` (rank order); `t` may be this rank's slice of `out`."""
    if _host_staged(t, group):
        h = torch.empty(out.shape, dtype=out.dtype)
        dist.all_gather_into_tensor(h, t.detach().cpu(), group=group)
        out.copy_(h)
        return _Done() if async_op else None
    return dist.all_gather_into_tensor(out, t, group=group, async_op=async_op)


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
    """Distinct Philox key per rank (64-bit golden-ratio stride), for per-rank streams that are not
    meant to reproduce a one-GPU run (e.g. --global-draws 0 training draws)."""
    return (base_seed + 0x9E3779B97F4A7C15 * (rank + 1)) & ((1 << 63) - 1)


def gather_shards(local: torch.Tensor, n_total: int, group=None) -> torch.Tensor:
    """All-gather variable-size leading-dim shards (ranks hold shard_range slices in rank order)."""
    world = dist.get_world_size(group)
    per = -(-n_total // world)
    pad = torch.zeros((per,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    pad[: local.shape[0]] = local
    bufs = [torch.empty_like(pad) for _ in range(world)]
    all_gather_(bufs, pad, group=group)
    parts = []
    for r in range(world):
        s, e = shard_range(n_total, r, world)
        parts.append(bufs[r][: e - s])
    return torch.cat(parts, 0)


def sample_sharded(sampler, model, sde, y_cat: torch.Tensor, y_cont: torch.Tensor, img_shape, *,
                   base_seed: int = 0, gather: bool = True, **kw) -> torch.Tensor:
    """Run `sampler` (sample_reverse_sde_euler_maruyama / sample_probability_flow_ode) on this
    rank's slice [s, e) of the batch with the batch's one seed and Philox element offset s*H*W:
    the gathered images equal a one-GPU run of the whole batch with the same seed bit for bit
    (the reference draws one noise stream for the whole batch, sde_score_model.py:537,557)."""
    rank, world = rank_world()
    B = img_shape[0]
    s, e = shard_range(B, rank, world)
    per_img = 1
    for d in img_shape[1:]:
        per_img *= int(d)
    local = sampler(model, sde, y_cat[s:e], y_cont[s:e], (e - s,) + tuple(img_shape[1:]),
                    seed=int(base_seed), elem_offset=s * per_img, **kw)
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
    all_reduce_(flat, group=group)
    flat.div_(world)
    off = 0
    for g in grads:
        n = g.numel()
        g.copy_(flat[off:off + n].view_as(g))
        off += n


class BucketedGradAllReduce:
    """Gradient averaging overlapped with the backward pass (batch-DP training).

    Parameters are grouped, in reverse registration order (roughly the order backward produces
    their gradients), into buckets of about `bucket_mb` MB, each ONE flat device buffer.  Gradients
    live in the buckets: `zero_grad()` zeroes the buffers and points every `p.grad` at its slice
    (gradient-as-bucket-view), so autograd accumulates each fresh gradient straight into the bucket
    (`grad += new` in place) and nothing is copied.  A post-accumulate-grad hook per parameter
    counts arrivals; once a bucket is complete AND every bucket before it has been launched, its
    all-reduce is launched asynchronously (RCCL runs it on its own stream, ordered after the
    producing kernels) while the rest of the backward pass is still being computed.  Launching
    strictly in bucket order keeps every rank's sequence of collectives identical even if the
    ranks' graphs produce gradients in different orders.  `finish()` launches what is left, waits
    and divides by the world size; the averaged gradients are then already in `p.grad`.

    Gradient presence: each bucket carries one extra slot per parameter (1 if this rank produced
    a gradient for it, summed by the same all-reduce).  A parameter no rank produced a gradient for
    gets `p.grad = None` — as in a single-process run, where torch.optim.Adam (and the fused Adam)
    then skips it; one that only some ranks produced is averaged with zeros from the others (the
    global-batch mean).

    Usage per step: ``ar.zero_grad(); loss.backward(); ar.finish(); opt.step()``.  At world 1 it
    is a plain ``zero_grad(set_to_none=True)`` and `finish()` does nothing.
    """

    def __init__(self, params, bucket_mb: float = 25.0, group=None) -> None:
        self.group = group
        self.params = [p for p in params if p.requires_grad]
        self.world = dist.get_world_size(group) if (dist.is_available() and dist.is_initialized()) else 1
        self.active = dp_active(group)  # world > 1, or world 1 under TCX_DP_FORCE=1 (RCCL rehearsal)
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
        self.arrived = [set() for _ in self.buckets]
        self.works = [None] * len(self.buckets)
        self.next_launch = 0
        self.hooks = []
        if self.active:
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

    def _view(self, p) -> torch.Tensor:
        bi, off, _ = self.where[id(p)]
        return self.buckets[bi][1][off:off + p.numel()].view_as(p)

    def zero_grad(self) -> None:
        """Start a step: every gradient a zeroed view into its bucket (world 1: grads set to None)."""
        if not self.active:
            for p in self.params:
                p.grad = None
            return
        for bi, (ps, flat, n) in enumerate(self.buckets):
            flat.zero_()
            for p in ps:
                p.grad = self._view(p)
            self.arrived[bi] = set()
            self.works[bi] = None
        self.next_launch = 0

    def _launch(self, bi) -> None:
        ps, flat, n = self.buckets[bi]
        if len(self.arrived[bi]) == len(ps):
            flat[n:].fill_(1.0)
        else:  # some parameter got no gradient on this rank: presence 0 in its slot, zeros in its data
            pres = torch.tensor([1.0 if id(p) in self.arrived[bi] else 0.0 for p in ps], dtype=flat.dtype)
            flat[n:].copy_(pres)
            # A step not begun with zero_grad() (e.g. opt.zero_grad(set_to_none=True)) leaves the
            # previous step's averaged gradient in the slice: it must not enter this sum.
            for p in ps:
                if id(p) not in self.arrived[bi]:
                    self._view(p).zero_()
        self.works[bi] = all_reduce_(flat, group=self.group, async_op=True)

    def _launch_ready(self) -> None:
        while (self.next_launch < len(self.buckets)
               and len(self.arrived[self.next_launch]) == len(self.buckets[self.next_launch][0])):
            self._launch(self.next_launch)
            self.next_launch += 1

    def _on_grad(self, p) -> None:
        bi, _, _ = self.where[id(p)]
        g = p.grad
        view = self._view(p)
        if g is not None and g.data_ptr() != view.data_ptr():
            # the step was not started by zero_grad() (grad was None): adopt the fresh gradient
            view.copy_(g)
            p.grad = view
        self.arrived[bi].add(id(p))
        self._launch_ready()

    def finish(self) -> None:
        if not self.active:
            return
        missing = set()
        for bi in range(self.next_launch, len(self.buckets)):
            for p in self.buckets[bi][0]:
                if id(p) not in self.arrived[bi]:
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
                keep = id(p) not in missing or counts[id(p)] > 0
                p.grad = self._view(p) if keep else None
            self.arrived[bi] = set()
            self.works[bi] = None
        self.next_launch = 0

    def remove(self) -> None:
        for h in self.hooks:
            h.remove()
        self.hooks = []


class ZeroAdam:
    """ZeRO stage 1 for batch-DP training (config 4's prior): the gradient average and
    the Adam update of torch.optim.Adam (the reference's optimiser, train_diffusion_prior.py:248-277),
    with the optimiser state and the update sharded over the ranks.

    Parameters are grouped, in reverse registration order (the order backward produces their
    gradients), into buckets of about `bucket_mb` MB.  Each bucket owns two flat device buffers, its
    parameters and its gradients, both padded to a multiple of the world size; every parameter's
    `.data` and `.grad` are views into them (parameter- and gradient-as-bucket-view), so nothing is
    copied between the model and the collectives.  Per step:

      * backward accumulates into the gradient buckets; a post-accumulate-grad hook launches each
        complete bucket's REDUCE-SCATTER (async, in bucket order) while backward continues: rank r
        receives the summed slice r of every bucket (1/world of the bytes an all-reduce would
        deliver to it);
      * `step()` waits for them, divides by the world size and runs ONE fused Adam launch
        (tcx_adam) over this rank's slices only: exp_avg / exp_avg_sq exist for 1/world of the
        parameters, and the update streams 1/world of the 28 B per parameter;
      * the updated slices are ALL-GATHERED back into every rank's parameter buckets (async per
        bucket, waited before `step()` returns).

    Adam is element-wise, so a rank's slice update is the same arithmetic as the whole-tensor
    update: world N equals world 1 up to the gradient sum's rounding (the mean of N shard means),
    as for `BucketedGradAllReduce` + Adam.  Every parameter must receive a gradient on every rank in
    every step (the prior's graph uses them all); a missing one is an error, not a silent skip.  At
    world 1 without TCX_DP_FORCE there are no collectives: a fused Adam over the whole buckets.

    Usage per step: ``zo.zero_grad(); loss.backward(); zo.step()``.  `state_dict()` / `load_state_dict()`
    carry this rank's shard of the moments (not the reference's per-parameter layout; the prior's
    checkpoint holds only the model, train_diffusion_prior.py:272)."""

    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0,
                 bucket_mb: float = 25.0, group=None) -> None:
        from ._lib import TcxAdamTensor  # noqa: F401  (fail early without libtcx)
        self.group = group
        self.lr, self.betas, self.eps, self.weight_decay = float(lr), tuple(betas), float(eps), float(weight_decay)
        self.params = [p for p in params if p.requires_grad]
        if not self.params:
            raise ValueError("ZeroAdam: no trainable parameters")
        for p in self.params:
            if not (p.is_cuda and p.dtype == torch.float32):
                raise RuntimeError("ZeroAdam: fp32 parameters on the MI355X only")
        self.active = dp_active(group)
        self.world = dist.get_world_size(group) if self.active else 1
        self.rank = dist.get_rank(group) if self.active else 0
        self.buckets = []  # dicts: params, pflat, gflat, n (data elements), shard (elements per rank)
        cur, cur_bytes = [], 0
        for p in reversed(self.params):
            cur.append(p)
            cur_bytes += p.numel() * 4
            if cur_bytes >= bucket_mb * 1e6:
                self._add_bucket(cur)
                cur, cur_bytes = [], 0
        if cur:
            self._add_bucket(cur)
        self.where = {id(p): bi for bi, b in enumerate(self.buckets) for p in b["params"]}
        self.arrived = [set() for _ in self.buckets]
        self.works = [None] * len(self.buckets)
        self.next_launch = 0
        self.step_count = 0
        self.hooks = []
        if self.active:
            for p in self.params:
                self.hooks.append(p.register_post_accumulate_grad_hook(self._on_grad))

    def _add_bucket(self, ps) -> None:
        n = sum(p.numel() for p in ps)
        shard = -(-n // self.world)
        dev = ps[0].device
        pflat = torch.zeros(shard * self.world, dtype=torch.float32, device=dev)
        gflat = torch.zeros(shard * self.world, dtype=torch.float32, device=dev)
        off = 0
        for p in ps:
            k = p.numel()
            pflat[off:off + k].copy_(p.data.reshape(-1))
            p.data = pflat[off:off + k].view_as(p)
            off += k
        lo = self.rank * shard
        self.buckets.append(dict(params=ps, pflat=pflat, gflat=gflat, n=n, shard=shard,
                                 # world 1 without collectives: the whole gradient bucket is the shard
                                 gshard=torch.zeros(shard, dtype=torch.float32, device=dev) if self.active else gflat,
                                 m=torch.zeros(shard, dtype=torch.float32, device=dev),
                                 v=torch.zeros(shard, dtype=torch.float32, device=dev),
                                 live=max(0, min(shard, n - lo))))  # this rank's real (unpadded) elements

    def _gview(self, b, p) -> torch.Tensor:
        off = 0
        for q in b["params"]:
            if q is p:
                return b["gflat"][off:off + p.numel()].view_as(p)
            off += q.numel()
        raise KeyError("parameter not in bucket")

    def zero_grad(self) -> None:
        """Start a step: every gradient a zeroed view into its bucket."""
        for bi, b in enumerate(self.buckets):
            b["gflat"].zero_()
            off = 0
            for p in b["params"]:
                p.grad = b["gflat"][off:off + p.numel()].view_as(p)
                off += p.numel()
            self.arrived[bi] = set()
            self.works[bi] = None
        self.next_launch = 0

    def _launch(self, bi) -> None:
        b = self.buckets[bi]
        self.works[bi] = reduce_scatter_(b["gshard"], b["gflat"], group=self.group, async_op=True)

    def _launch_ready(self) -> None:
        while (self.next_launch < len(self.buckets)
               and len(self.arrived[self.next_launch]) == len(self.buckets[self.next_launch]["params"])):
            self._launch(self.next_launch)
            self.next_launch += 1

    def _on_grad(self, p) -> None:
        bi = self.where[id(p)]
        b = self.buckets[bi]
        view = self._gview(b, p)
        if p.grad is not None and p.grad.data_ptr() != view.data_ptr():
            view.copy_(p.grad)  # the step was not started by zero_grad(): adopt the fresh gradient
            p.grad = view
        self.arrived[bi].add(id(p))
        self._launch_ready()

    @torch.no_grad()
    def step(self) -> None:
        from ._lib import TcxAdamTensor, check, lib, stream_ptr
        if self.active:
            for bi in range(self.next_launch, len(self.buckets)):
                if len(self.arrived[bi]) != len(self.buckets[bi]["params"]):
                    raise RuntimeError("ZeroAdam: a parameter received no gradient on this rank this step")
                self._launch(bi)
            self.next_launch = len(self.buckets)
            for bi, b in enumerate(self.buckets):
                self.works[bi].wait()
                b["gshard"].div_(self.world)
        else:
            for b in self.buckets:
                if any(p.grad is None for p in b["params"]):
                    raise RuntimeError("ZeroAdam: a parameter received no gradient this step")
                for p in b["params"]:  # a step not begun with zero_grad(): gather the gradients
                    v = self._gview(b, p)
                    if p.grad.data_ptr() != v.data_ptr():
                        v.copy_(p.grad)
                        p.grad = v
        self.step_count += 1
        entries = []
        for b in self.buckets:
            lo = self.rank * b["shard"]
            if b["live"] > 0:
                entries.append(TcxAdamTensor(b["pflat"][lo:].data_ptr(), b["gshard"].data_ptr(), b["m"].data_ptr(),
                                             b["v"].data_ptr(), b["live"]))
        if entries:
            dev = self.buckets[0]["pflat"].device
            table = (TcxAdamTensor * len(entries))(*entries)
            check(lib().tcx_adam(table, len(entries), max(e.n for e in entries), self.lr, float(self.betas[0]),
                                 float(self.betas[1]), self.eps, self.weight_decay, self.step_count,
                                 stream_ptr(dev)), "tcx_adam (ZeRO-1 shard)")
        if self.active:
            works = []
            for b in self.buckets:
                lo = self.rank * b["shard"]
                works.append(all_gather_into_(b["pflat"], b["pflat"][lo:lo + b["shard"]], group=self.group,
                                              async_op=True))
            for w in works:
                w.wait()
            for bi in range(len(self.buckets)):
                self.arrived[bi] = set()
                self.works[bi] = None
            self.next_launch = 0
        from .optim import mark_updated
        mark_updated(self.params)  # packed-weight caches see the new weights

    def state_dict(self) -> dict:
        return {"step": self.step_count, "rank": self.rank, "world": self.world,
                "m": [b["m"].clone() for b in self.buckets], "v": [b["v"].clone() for b in self.buckets]}

    def load_state_dict(self, sd: dict) -> None:
        if sd["world"] != self.world or sd["rank"] != self.rank or len(sd["m"]) != len(self.buckets):
            raise ValueError("ZeroAdam: state of a different sharding")
        self.step_count = int(sd["step"])
        for b, m, v in zip(self.buckets, sd["m"], sd["v"]):
            b["m"].copy_(m)
            b["v"].copy_(v)

    def remove(self) -> None:
        for h in self.hooks:
            h.remove()
        self.hooks = []
