"""Optimiser and EMA for the training scripts, one fused multi-tensor HIP launch per step.

`Adam` follows torch.optim.Adam (the reference's optimiser: scripts/train_sde_score_model.py:160,
train_vae.py, train_diffusion_prior.py): same constructor arguments, param groups, state keys
(`step`, `exp_avg`, `exp_avg_sq`) and update arithmetic (torch/optim/adam.py single-tensor path),
so `state_dict()` round-trips with the reference's checkpoints.  `amsgrad`, `maximize`,
`capturable`, `differentiable` and `fused` are not supported (the reference uses none of them).

`ema_update` is the reference's EMA (train_sde_score_model.py:236-240):
p_ema = p_ema * decay + (1 - decay) * p.
"""
from __future__ import annotations

from typing import Iterable

import torch

from torch.autograd.graph import increment_version

from ._lib import TcxAdamTensor, check, lib, stream_ptr


def mark_updated(tensors) -> None:
    """Bump the autograd version counter of tensors a libtcx kernel rewrote through raw pointers (the
    fused Adam / EMA / ZeRO all-gather).  The models' packed-weight caches key on (data_ptr, _version)
    (sde_score_model.CondUNetTiny.tcx_pack, diffusion_prior.DiffusionPriorFiLM._tcx); without the bump
    an eval-mode forward after an optimiser step would reuse the pack of the previous weights (a sample
    grid after epoch 2 drawn with epoch-1 weights), as torch's in-place optimiser updates bump it."""
    # one call for the whole list: per tensor the same call costs ~7 us each (0.7 ms per prior step), the list
    # form ~6 us in total
    ts = list(tensors)
    if ts:
        increment_version(ts)


def _host_table(entries):
    """ctypes array of tcx_adam_tensor; libtcx copies it into the kernel arguments."""
    return (TcxAdamTensor * len(entries))(*entries)


class Adam(torch.optim.Optimizer):
    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0,
                 amsgrad: bool = False, *, maximize: bool = False) -> None:
        if lr < 0.0 or eps < 0.0 or not (0.0 <= betas[0] < 1.0) or not (0.0 <= betas[1] < 1.0) or weight_decay < 0:
            raise ValueError("invalid Adam hyper-parameter")
        if amsgrad or maximize:
            raise NotImplementedError("amsgrad / maximize are not supported by the fused MI355X Adam")
        super().__init__(params, dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay, amsgrad=False,
                                      maximize=False, foreach=None, capturable=False, differentiable=False,
                                      fused=None, decoupled_weight_decay=False))

    @torch.no_grad()
    def step(self, closure=None):
        """One fused tcx_adam launch per (param group, step count, device).

        The host path is kept short (round 6): the prior's training step (100+ parameters) left the GPU idle
        0.5-0.8 ms per step between the last backward kernel and the Adam launch while this loop ran a CPU
        tensor add, an .item() and a ctypes struct per parameter (profiles/r06_d_*).  Now the per-parameter
        `step` tensors of a group are 0-dim views of ONE CPU tensor (so state_dict() still holds one `step`
        tensor per parameter, as torch.optim.Adam's) advanced by a single add, the counts are mirrored in a
        Python list, and the kernel-argument table is rebuilt only when a storage pointer changes."""
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        L = lib()
        if not hasattr(self, "_tcx_steps"):
            self._tcx_steps, self._tcx_counts, self._tcx_masks = {}, {}, {}
        for gi, group in enumerate(self.param_groups):
            beta1, beta2 = group["betas"]
            params = group["params"]
            stor = self._tcx_steps.get(gi)
            if stor is None or stor.numel() != len(params):
                stor = self._tcx_steps[gi] = torch.zeros(len(params), dtype=torch.float32)
                self._tcx_counts[gi] = [0] * len(params)
            counts = self._tcx_counts[gi]
            items, has = [], []
            for i, p in enumerate(params):
                g = p.grad
                st = self.state[p]
                if len(st) == 0 and g is not None:
                    if g.is_sparse:
                        raise RuntimeError("Adam does not support sparse gradients")
                    if not p.is_cuda:
                        raise RuntimeError("the fused Adam runs on the MI355X only (params must be on 'cuda')")
                    if p.dtype != torch.float32 or not p.is_contiguous():
                        raise RuntimeError("fused Adam is fp32-only and needs contiguous params")
                    stor[i] = 0.0
                    counts[i] = 0
                    st["step"] = stor[i]
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                elif "step" in st and st["step"]._base is not stor:  # state loaded from a checkpoint
                    v = float(st["step"])
                    stor[i] = v
                    counts[i] = int(v)
                    st["step"] = stor[i]
                has.append(g is not None)
                if g is not None:
                    items.append((p, g if g.is_contiguous() else g.contiguous(), st))
                    counts[i] += 1
            if not items:
                continue
            pattern = tuple(has)
            if all(has):
                stor.add_(1.0)
            else:
                mask = self._tcx_masks.get((gi, pattern))
                if mask is None:
                    mask = self._tcx_masks[(gi, pattern)] = torch.tensor(pattern, dtype=torch.float32)
                stor.add_(mask)
            steps = [counts[i] for i, h in enumerate(has) if h]
            by_step = {}
            if min(steps) == max(steps):
                by_step[(steps[0], items[0][0].device)] = items
            else:  # counts differ (a parameter skipped in some steps): one launch per count
                for it, c in zip(items, steps):
                    by_step.setdefault((c, it[0].device), []).append(it)
            for (step, device), its in by_step.items():
                table, n, max_n = self._table(gi, step, its)
                check(L.tcx_adam(table, n, max_n, float(group["lr"]), float(beta1),
                                 float(beta2), float(group["eps"]), float(group["weight_decay"]), step,
                                 stream_ptr(device)), "tcx_adam")
                mark_updated([p for p, _, _ in its])
        return loss

    def _table(self, gi, step, items):
        """The ctypes {p, g, m, v, n} table of these parameters, cached while every pointer is unchanged."""
        key = tuple((p.data_ptr(), g.data_ptr(), st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr())
                    for p, g, st in items)
        cache = getattr(self, "_tcx_tables", None)
        if cache is None:
            cache = self._tcx_tables = {}
        ck = (gi, id(items[0][0]), len(items))  # (the step count is a launch argument, not in the table)
        hit = cache.get(ck)
        if hit is None or hit[0] != key:
            for p, g, st in items:
                if not (p.is_contiguous() and st["exp_avg"].is_contiguous() and st["exp_avg_sq"].is_contiguous()):
                    raise RuntimeError("fused Adam needs contiguous params and state")
            entries = [TcxAdamTensor(p.data_ptr(), g.data_ptr(), st["exp_avg"].data_ptr(),
                                     st["exp_avg_sq"].data_ptr(), p.numel()) for p, g, st in items]
            hit = (key, _host_table(entries), len(entries), max(p.numel() for p, _, _ in items))
            if len(cache) > 64:
                cache.clear()
            cache[ck] = hit
        return hit[1], hit[2], hit[3]

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        self._tcx_tables = {}  # (the loaded `step` tensors are re-bound to the group views at the next step)


@torch.no_grad()
def ema_update(ema_model: torch.nn.Module, model: torch.nn.Module, decay: float) -> None:
    """p_ema.mul_(decay).add_(p, alpha=1 - decay) for every parameter pair, one launch."""
    pairs = [(pe, p) for pe, p in zip(ema_model.parameters(), model.parameters())]
    if not pairs:
        return
    device = pairs[0][1].device
    entries = [TcxAdamTensor(pe.data_ptr(), p.data_ptr(), None, None, p.numel()) for pe, p in pairs]
    check(lib().tcx_ema(_host_table(entries), len(entries), max(p.numel() for _, p in pairs), float(decay),
                        stream_ptr(device)), "tcx_ema")
    mark_updated(pe for pe, _ in pairs)


def params_to(params: Iterable[torch.nn.Parameter]):  # pragma: no cover - convenience
    return [p for p in params if p.requires_grad]
