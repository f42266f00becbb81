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
    for t in tensors:
        increment_version(t)


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
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        L = lib()
        for group in self.param_groups:
            beta1, beta2 = group["betas"]
            by_step = {}
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.grad.is_sparse:
                    raise RuntimeError("Adam does not support sparse gradients")
                if not p.is_cuda:
                    raise RuntimeError("the fused Adam runs on the MI355X only (params must be on 'cuda')")
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = torch.tensor(0.0, dtype=torch.float32)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["step"] += 1
                g = p.grad if p.grad.is_contiguous() else p.grad.contiguous()
                if not (p.is_contiguous() and st["exp_avg"].is_contiguous() and st["exp_avg_sq"].is_contiguous()):
                    raise RuntimeError("fused Adam needs contiguous params and state")
                if p.dtype != torch.float32:
                    raise RuntimeError("fused Adam is fp32-only")
                key = (int(st["step"].item()), p.device)
                by_step.setdefault(key, []).append((p, g, st))
            for (step, device), items in by_step.items():
                entries = [TcxAdamTensor(p.data_ptr(), g.data_ptr(), s["exp_avg"].data_ptr(),
                                         s["exp_avg_sq"].data_ptr(), p.numel()) for p, g, s in items]
                table = _host_table(entries)
                max_n = max(p.numel() for p, _, _ in items)
                check(L.tcx_adam(table, len(entries), max_n, float(group["lr"]), float(beta1),
                                 float(beta2), float(group["eps"]), float(group["weight_decay"]), step,
                                 stream_ptr(device)), "tcx_adam")
                mark_updated(p for p, _, _ in items)
        return loss


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
