"""MI355X-native drop-in for toycrystals.models.diffusion_prior (FiLM-MLP latent prior).

Mirrors /root/reference/src/toycrystals/models/diffusion_prior.py (names, signatures,
state_dict keys, seeded init).  The forward runs in libtcx as fp32-MFMA GEMMs:
  t_mlp / y_cont_mlp / y_fuse      Linear+SiLU epilogue, Linear          (:80-104)
  all n_blocks FiLM `cond` linears ONE [B,2W] x [2W, n_blocks*2W] GEMM  (:47, cond shared)
  per block LN+FiLM (tcx_layernorm_film), fc1+SiLU, fc2 + residual epilogue (:49-54)
  out LayerNorm, out_proj                                              (:125-126)
The integer-t sinusoid (:11-25), the y_cat row gather, q_sample and the DDIM update run in
libtcx kernels too (tcx_prior_temb / tcx_embedding_fwd / tcx_q_sample / tcx_ddim_step).
Training: with autograd on, the same forward runs as a chain of libtcx autograd Functions
(functional.py): GEMM linears, per-block LayerNorm+FiLM with its fused backward, residual
added in the fc2 GEMM (beta = 1).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import functional as TF
from .._lib import check, lib, ptr, require_gpu_tensor, stream_ptr

_FREQS = {}


def _temb_freqs(dim: int, device) -> torch.Tensor:
    """exp(-linspace(0, ln 1e4, half)) with the reference's fp32 torch arithmetic, cached on device."""
    key = (dim, torch.device(device))
    if key not in _FREQS:
        half = dim // 2
        f = torch.exp(torch.linspace(0, math.log(10_000), steps=half, dtype=torch.float32) * (-1.0))
        _FREQS[key] = f.to(device)
    return _FREQS[key]


def _temb_dev(t: torch.Tensor, dim: int) -> torch.Tensor:
    t = t.to(torch.int64).contiguous()
    B = t.shape[0]
    te = torch.empty((B, dim), device=t.device, dtype=torch.float32)
    check(lib().tcx_prior_temb(ptr(t), ptr(_temb_freqs(dim, t.device)), B, dim, ptr(te), stream_ptr(t.device)),
          "tcx_prior_temb")
    return te


def timestep_embedding(t: torch.Tensor, dim: int) -> torch.Tensor:
    """Integer-t sinusoid [sin, cos], no 2*pi (diffusion_prior.py:11-25)."""
    half = dim // 2
    freqs = torch.exp(torch.linspace(0, math.log(10_000), steps=half, device=t.device, dtype=torch.float32) * (-1.0))
    args = t.to(torch.float32)[:, None] * freqs[None, :]
    emb = torch.cat([torch.sin(args), torch.cos(args)], dim=1)
    if dim % 2 == 1:
        emb = torch.cat([emb, torch.zeros((emb.shape[0], 1), device=t.device)], dim=1)
    return emb


def y_vec(y_cat: torch.Tensor, y_cont: torch.Tensor, n_types: int) -> torch.Tensor:
    y_oh = F.one_hot(y_cat, num_classes=n_types).to(dtype=torch.float32)
    return torch.cat([y_oh, y_cont.to(dtype=torch.float32)], dim=1)


class FiLMResBlock(nn.Module):
    def __init__(self, width: int, cond_dim: int, mult: int = 4) -> None:
        super().__init__()
        self.norm = nn.LayerNorm(width)
        self.fc1 = nn.Linear(width, mult * width)
        self.fc2 = nn.Linear(mult * width, width)
        self.cond = nn.Linear(cond_dim, 2 * width)
        self.act = nn.SiLU()


def _round_up(v: int, a: int) -> int:
    return (v + a - 1) // a * a


class _PriorPack:
    def __init__(self, m: "DiffusionPriorFiLM", device) -> None:
        L = lib()
        st = stream_ptr(device)
        self.keep = []

        def dev(t):
            t = t.detach().to(device=device, dtype=torch.float32).contiguous()
            self.keep.append(t)
            return t

        def lin(w, b):
            w = dev(w)
            n, k = w.shape
            npad, kpad = _round_up(n, 32), _round_up(k, 32)
            wpk = torch.empty((npad, kpad), device=device, dtype=torch.float32)
            check(L.tcx_pack_conv_weight(ptr(w), ptr(wpk), n, k, 1, npad, kpad, st), "pack linear")
            self.keep.append(wpk)
            return (wpk, n, npad, kpad, k, dev(b))

        def seq(s):
            return lin(s[0].weight, s[0].bias), lin(s[2].weight, s[2].bias)

        self.t_mlp = seq(m.t_mlp)
        self.y_cont_mlp = seq(m.y_cont_mlp)
        self.y_fuse = seq(m.y_fuse)
        self.y_cat_emb = dev(m.y_cat_emb.weight)
        self.in_proj = lin(m.in_proj.weight, m.in_proj.bias)
        blocks = list(m.blocks)
        self.cond_all = lin(torch.cat([b.cond.weight for b in blocks], 0), torch.cat([b.cond.bias for b in blocks], 0))
        self.blocks = [(dev(b.norm.weight), dev(b.norm.bias), lin(b.fc1.weight, b.fc1.bias),
                        lin(b.fc2.weight, b.fc2.bias)) for b in blocks]
        self.out_norm = (dev(m.out_norm.weight), dev(m.out_norm.bias))
        self.out_proj = lin(m.out_proj.weight, m.out_proj.bias)


def _lin(x1, x2, packed, act, resid=None, out=None):
    wpk, n, npad, kpad, k, b = packed
    M, K1 = x1.shape
    K2 = x2.shape[1] if x2 is not None else 0
    assert K1 + K2 == k, (K1, K2, k)
    y = out if out is not None else torch.empty((M, n), device=x1.device, dtype=torch.float32)
    # skinny batches (DDIM over 36 samples) split K over the chip (tcx_linear_ws scratch)
    nb = int(lib().tcx_linear_workspace(M, n, K1, K2))
    ws = TF._ws(x1.device, nb) if nb else None
    check(lib().tcx_linear_ws(ptr(x1), K1, ptr(x2), K2, ptr(wpk), ptr(b), ptr(resid), ptr(y), M, n, npad, kpad, act,
                              ptr(ws), nb, stream_ptr(x1.device)), "tcx_linear")
    return y


class DiffusionPriorFiLM(nn.Module):
    """eps-prediction FiLM-MLP on z (diffusion_prior.py:57-127)."""

    def __init__(self, z_dim: int, n_types: int, y_cont_dim: int, t_emb_dim: int = 64, width: int = 256,
                 n_blocks: int = 6, y_cat_emb_dim: int = 64) -> None:
        super().__init__()
        self.z_dim = int(z_dim)
        self.n_types = int(n_types)
        self.y_cont_dim = int(y_cont_dim)
        self.t_emb_dim = int(t_emb_dim)
        self.width = int(width)
        self.y_cat_emb = nn.Embedding(self.n_types, y_cat_emb_dim)
        self.y_cont_mlp = nn.Sequential(nn.Linear(self.y_cont_dim, y_cat_emb_dim), nn.SiLU(),
                                        nn.Linear(y_cat_emb_dim, y_cat_emb_dim))
        self.y_fuse = nn.Sequential(nn.Linear(2 * y_cat_emb_dim, width), nn.SiLU(), nn.Linear(width, width))
        self.t_mlp = nn.Sequential(nn.Linear(self.t_emb_dim, width), nn.SiLU(), nn.Linear(width, width))
        self.in_proj = nn.Linear(self.z_dim, width)
        cond_dim = 2 * width
        self.blocks = nn.ModuleList([FiLMResBlock(width, cond_dim) for _ in range(n_blocks)])
        self.out_norm = nn.LayerNorm(width)
        self.out_proj = nn.Linear(width, self.z_dim)

    def _tcx(self, device):
        if device.type != "cuda":
            raise RuntimeError("DiffusionPriorFiLM runs on the MI355X only: move the model and inputs to 'cuda'")
        key = (device,) + tuple((p.data_ptr(), p._version) for p in self.parameters())
        if getattr(self, "_pk_key", None) != key:
            with torch.no_grad():
                self._pk = _PriorPack(self, device)
            self._pk_key = key
        return self._pk

    def forward(self, z_t: torch.Tensor, t: torch.Tensor, y_cat: torch.Tensor, y_cont: torch.Tensor) -> torch.Tensor:
        require_gpu_tensor(z_t, "z_t")
        if torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters()):
            return self._forward_train(z_t, t, y_cat, y_cont)
        with torch.no_grad():
            return self._forward_eval(z_t, t, y_cat, y_cont)

    def _forward_train(self, z_t, t, y_cat, y_cont):
        """Differentiable forward (diffusion_prior.py:108-127) on libtcx autograd Functions."""
        te = _temb_dev(t, self.t_emb_dim)
        t_feat = TF.linear(TF.act(TF.linear(te, self.t_mlp[0]), TF.ACT_SILU), self.t_mlp[2])
        ycf = TF.EmbeddingFn.apply(y_cat.to(torch.int64), self.y_cat_emb.weight)
        ycont = TF.linear(TF.act(TF.linear(y_cont.to(torch.float32), self.y_cont_mlp[0]), TF.ACT_SILU),
                          self.y_cont_mlp[2])
        y_feat = TF.linear(TF.act(TF.linear(TF.cat_cols(ycf, ycont), self.y_fuse[0]), TF.ACT_SILU), self.y_fuse[2])
        cond = TF.cat_cols(t_feat, y_feat)
        h = TF.linear(z_t.to(torch.float32), self.in_proj)
        for blk in self.blocks:
            gb = TF.linear(cond, blk.cond)  # [gamma | beta] = cond(cond).chunk(2)
            hn = TF.LayerNormFiLMFn.apply(h, blk.norm.weight, blk.norm.bias, gb, blk.norm.eps)
            h = TF.linear(TF.act(TF.linear(hn, blk.fc1), TF.ACT_SILU), blk.fc2, resid=h)
        hn = TF.LayerNormFiLMFn.apply(h, self.out_norm.weight, self.out_norm.bias, None, self.out_norm.eps)
        return TF.linear(hn, self.out_proj)

    def _forward_eval(self, z_t, t, y_cat, y_cont):
        pk = self._tcx(z_t.device)
        st = stream_ptr(z_t.device)
        W = self.width
        te = _temb_dev(t, self.t_emb_dim)
        t_feat = _lin(_lin(te, None, pk.t_mlp[0], act=3), None, pk.t_mlp[1], act=0)
        yc = _lin(_lin(y_cont.to(torch.float32).contiguous(), None, pk.y_cont_mlp[0], act=3), None,
                  pk.y_cont_mlp[1], act=0)
        yci = y_cat.to(torch.int64).contiguous()
        ycat_feat = torch.empty((yci.shape[0], pk.y_cat_emb.shape[1]), device=z_t.device, dtype=torch.float32)
        check(lib().tcx_embedding_fwd(ptr(yci), ptr(pk.y_cat_emb), yci.shape[0], pk.y_cat_emb.shape[1],
                                      ptr(ycat_feat), st), "tcx_embedding_fwd")
        y_feat = _lin(_lin(ycat_feat, yc, pk.y_fuse[0], act=3), None, pk.y_fuse[1], act=0)
        gb_all = _lin(t_feat, y_feat, pk.cond_all, act=0)  # [B, n_blocks*2W]
        h = _lin(z_t.to(torch.float32).contiguous(), None, pk.in_proj, act=0)
        B = h.shape[0]
        hn = torch.empty_like(h)
        L = lib()
        for i, (lw, lb, fc1, fc2) in enumerate(pk.blocks):
            gb = gb_all[:, i * 2 * W:]
            check(L.tcx_layernorm_film(ptr(h), ptr(hn), B, W, ptr(lw), ptr(lb), gb.data_ptr(), gb_all.shape[1],
                                       1e-5, st), "layernorm_film")
            a = _lin(hn, None, fc1, act=3)
            h = _lin(a, None, fc2, act=0, resid=h)
        check(L.tcx_layernorm_film(ptr(h), ptr(hn), B, W, ptr(pk.out_norm[0]), ptr(pk.out_norm[1]), None, 0, 1e-5,
                                   st), "layernorm")
        return _lin(hn, None, pk.out_proj, act=0)


@dataclass(frozen=True)
class DiffusionSchedule:
    """Linear-beta DDPM constants, q_sample and DDIM (eta=0) (diffusion_prior.py:167-252)."""
    betas: torch.Tensor
    alphas: torch.Tensor
    alpha_bars: torch.Tensor
    sqrt_alpha_bars: torch.Tensor
    sqrt_one_minus_alpha_bars: torch.Tensor

    @staticmethod
    def linear(T: int, beta_start: float, beta_end: float, device: torch.device) -> "DiffusionSchedule":
        # computed on the CPU (the reference's own device=cpu arithmetic) then moved
        betas = torch.linspace(beta_start, beta_end, steps=T, dtype=torch.float32)
        alphas = 1.0 - betas
        alpha_bars = torch.cumprod(alphas, dim=0)
        mv = lambda v: v.to(device)  # noqa: E731
        return DiffusionSchedule(betas=mv(betas), alphas=mv(alphas), alpha_bars=mv(alpha_bars),
                                 sqrt_alpha_bars=mv(torch.sqrt(alpha_bars)),
                                 sqrt_one_minus_alpha_bars=mv(torch.sqrt(1.0 - alpha_bars)))

    def q_sample(self, z0: torch.Tensor, t: torch.Tensor, eps: torch.Tensor) -> torch.Tensor:
        """z_t = sqrt(abar_t) z0 + sqrt(1 - abar_t) eps (diffusion_prior.py:194-201)."""
        z0 = z0.to(torch.float32).contiguous()
        eps = eps.to(device=z0.device, dtype=torch.float32).contiguous()
        t = t.to(device=z0.device, dtype=torch.int64).contiguous()
        out = torch.empty_like(z0)
        check(lib().tcx_q_sample(ptr(z0), ptr(t), ptr(eps), ptr(self.sqrt_alpha_bars),
                                 ptr(self.sqrt_one_minus_alpha_bars), z0.shape[0], z0.shape[1], ptr(out),
                                 stream_ptr(z0.device)), "tcx_q_sample")
        return out

    @torch.no_grad()
    def ddim_sample(self, model: nn.Module, y_cat: torch.Tensor, y_cont: torch.Tensor, n_steps: int = 50,
                    eta: float = 0.0, z_init: torch.Tensor | None = None) -> torch.Tensor:
        """DDIM (eta = 0) over the rounded, de-duplicated linspace grid (diffusion_prior.py:203-252)."""
        model.eval()
        device = self.betas.device
        B = int(y_cat.shape[0])
        z = torch.randn((B, model.z_dim), device=device) if z_init is None else z_init.to(device).float()
        z = z.contiguous().clone()
        T = int(self.betas.shape[0])
        ts = torch.round(torch.linspace(T - 1, 0, steps=n_steps)).to(torch.int64)
        ts = torch.unique_consecutive(ts).tolist()
        n = len(ts)
        abar = self.alpha_bars.detach().float().cpu()
        st = stream_ptr(device)
        for i in range(n):
            t = torch.full((B,), ts[i], device=device, dtype=torch.int64)
            eps_pred = model(z, t, y_cat, y_cont).contiguous()
            last = i == n - 1
            if not last and eta != 0.0:
                raise NotImplementedError("eta != 0 not implemented in this minimal version")
            a_prev = float(abar[ts[i + 1]]) if not last else 1.0
            check(lib().tcx_ddim_step(ptr(z), ptr(eps_pred), z.numel(), float(abar[ts[i]]), a_prev, 1 if last else 0,
                                      st), "tcx_ddim_step")
            if last:
                break
        return z
