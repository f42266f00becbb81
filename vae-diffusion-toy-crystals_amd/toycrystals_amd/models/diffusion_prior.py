"""MI355X-native drop-in for toycrystals.models.diffusion_prior (FiLM-MLP latent prior).

Mirrors /root/reference/src/toycrystals/models/diffusion_prior.py (names, signatures,
state_dict keys, seeded init).  The eval forward is ONE native call, tcx_prior_forward
(csrc/prior.hip), over fp32-MFMA linears:
  t_mlp / y_cont_mlp / y_fuse      Linear+SiLU epilogue, Linear          (:80-104)
  all n_blocks FiLM `cond` linears ONE [B,2W] x [2W, n_blocks*2W] GEMM  (:47, cond shared)
  per block LN+FiLM, fc1+SiLU, fc2 + residual                          (:49-54)
  out LayerNorm, out_proj                                              (:125-126)
At B <= 64 (the DDIM's latents) each weight is streamed once by the skinny kernels
(csrc/skinny.hip) and every LayerNorm+FiLM is fused into the preceding residual reduce.
DiffusionSchedule.ddim_sample on this model is ONE native call too (tcx_prior_ddim_sample),
with the step-invariant y branch and the FiLM projections of all timesteps hoisted out of the loop.
Training: with autograd on, the same forward runs as a chain of libtcx autograd Functions
(functional.py): fp32-MFMA GEMM linears, per-block LayerNorm+FiLM with its fused backward, residual
added in the fc2 GEMM (beta = 1).
"""
from __future__ import annotations

import ctypes
import math
import os
from dataclasses import dataclass

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import functional as TF
from .._lib import TcxLinearW, TcxPrior, c_fp, c_ll, check, lib, ptr, require_gpu_tensor, stream_ptr

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

        def lin(w, b, h2=False):
            """packed fp32 weight [npad][kpad]; h2: + the f16x3 pack (tcx_pack_linear_h2, K % 32 == 0)"""
            w = dev(w)
            n, k = w.shape
            npad, kpad = _round_up(n, 32), _round_up(k, 32)
            wpk = torch.empty((npad, kpad), device=device, dtype=torch.float32)
            check(L.tcx_pack_conv_weight(ptr(w), ptr(wpk), n, k, 1, npad, kpad, st), "pack linear")
            self.keep.append(wpk)
            wh = winv = None
            if h2 and k % 32 == 0:
                wh = torch.empty(int(L.tcx_linear_h2_bytes(n, k)), device=device, dtype=torch.uint8)
                winv = torch.empty((n + 15) // 16 * 16, device=device, dtype=torch.float32)
                check(L.tcx_pack_linear_h2(ptr(w), n, k, ptr(wh), ptr(winv), st), "pack linear h2")
                self.keep += [wh, winv]
            return (wpk, n, npad, kpad, k, dev(b), wh, winv)

        def seq(s):
            return lin(s[0].weight, s[0].bias), lin(s[2].weight, s[2].bias)

        self.t_mlp = seq(m.t_mlp)
        self.y_cont_mlp = seq(m.y_cont_mlp)
        self.y_fuse = seq(m.y_fuse)
        self.y_cat_emb = dev(m.y_cat_emb.weight)
        self.in_proj = lin(m.in_proj.weight, m.in_proj.bias)
        blocks = list(m.blocks)
        self.cond_all = lin(torch.cat([b.cond.weight for b in blocks], 0), torch.cat([b.cond.bias for b in blocks], 0))
        self.blocks = [(dev(b.norm.weight), dev(b.norm.bias), lin(b.fc1.weight, b.fc1.bias, h2=True),
                        lin(b.fc2.weight, b.fc2.bias, h2=True)) for b in blocks]
        self.out_norm = (dev(m.out_norm.weight), dev(m.out_norm.bias))
        self.out_proj = lin(m.out_proj.weight, m.out_proj.bias, h2=True)
        self.freqs = _temb_freqs(m.t_emb_dim, device)
        self.net = self._net(m)

    @staticmethod
    def _lw(packed) -> TcxLinearW:
        wpk, n, npad, kpad, k, b, wh, winv = packed
        return TcxLinearW(wpk.data_ptr(), b.data_ptr(), n, k, npad, kpad, ptr(wh), ptr(winv))

    def _net(self, m) -> TcxPrior:
        nb = len(self.blocks)
        self.fc1 = (TcxLinearW * nb)(*[self._lw(b[2]) for b in self.blocks])
        self.fc2 = (TcxLinearW * nb)(*[self._lw(b[3]) for b in self.blocks])
        self.norm_w = (c_fp * nb)(*[b[0].data_ptr() for b in self.blocks])
        self.norm_b = (c_fp * nb)(*[b[1].data_ptr() for b in self.blocks])
        return TcxPrior(
            z_dim=m.z_dim, n_types=m.n_types, y_cont_dim=m.y_cont_dim, t_emb_dim=m.t_emb_dim, width=m.width,
            n_blocks=nb, y_cat_emb_dim=self.y_cat_emb.shape[1], ln_eps=float(m.out_norm.eps),
            temb_freqs=self.freqs.data_ptr(), y_cat_emb=self.y_cat_emb.data_ptr(),
            t_mlp0=self._lw(self.t_mlp[0]), t_mlp2=self._lw(self.t_mlp[1]), y_cont0=self._lw(self.y_cont_mlp[0]),
            y_cont2=self._lw(self.y_cont_mlp[1]), y_fuse0=self._lw(self.y_fuse[0]), y_fuse2=self._lw(self.y_fuse[1]),
            in_proj=self._lw(self.in_proj), cond_all=self._lw(self.cond_all), out_proj=self._lw(self.out_proj),
            fc1=self.fc1, fc2=self.fc2, norm_w=self.norm_w, norm_b=self.norm_b,
            out_norm_w=self.out_norm[0].data_ptr(), out_norm_b=self.out_norm[1].data_ptr())


# "f16x3" (default): fc1 / fc2 / out_proj of the native eval forward and DDIM at B <= 64 on split-f16
# MFMA products (csrc/skinny.hip, ~2^-21 relative per product, fp32 accumulation); "fp32": f32 MFMA.
PRIOR_PRECISION = os.environ.get("TCX_PRIOR_PRECISION", "f16x3")


def _run_h2_or_fp32(run, device) -> None:
    """run(ovf) with an overflow word for the f16x3 path; if an activation left the f16 range (the
    word is set; one host read per call) run again in fp32 (ovf = None)."""
    if PRIOR_PRECISION != "f16x3":
        run(None)
        return
    ovf = torch.zeros(1, dtype=torch.int32, device=device)
    run(ovf)
    if int(ovf.item()) != 0:
        run(None)


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
        # fp32-MFMA GEMMs (an f16x3 GEMM measured slower on this step and was removed: DESIGN.md §3k)
        for blk in self.blocks:
            gb = TF.linear(cond, blk.cond)  # [gamma | beta] = cond(cond).chunk(2)
            hn = TF.LayerNormFiLMFn.apply(h, blk.norm.weight, blk.norm.bias, gb, blk.norm.eps)
            h = TF.linear(TF.act(TF.linear(hn, blk.fc1), TF.ACT_SILU), blk.fc2, resid=h)
        hn = TF.LayerNormFiLMFn.apply(h, self.out_norm.weight, self.out_norm.bias, None, self.out_norm.eps)
        return TF.linear(hn, self.out_proj)

    def _forward_eval(self, z_t, t, y_cat, y_cont):
        """tcx_prior_forward (csrc/prior.hip): the whole eval forward in one native call."""
        dev = z_t.device
        pk = self._tcx(dev)
        B = int(z_t.shape[0])
        out = torch.empty((B, self.z_dim), device=dev, dtype=torch.float32)
        if B == 0:
            return out
        z = z_t.to(torch.float32).contiguous()
        tt = t.to(device=dev, dtype=torch.int64).reshape(-1).expand(B).contiguous()
        yc = y_cat.to(device=dev, dtype=torch.int64).contiguous()
        yv = y_cont.to(device=dev, dtype=torch.float32).contiguous()
        L = lib()
        nb = int(L.tcx_prior_workspace(ctypes.byref(pk.net), B, 0))
        ws = TF._ws(dev, nb)

        def run(ovf):
            check(L.tcx_prior_forward(ctypes.byref(pk.net), ptr(z), ptr(tt), ptr(yc), ptr(yv), B, ptr(out), ptr(ovf),
                                      ptr(ws), nb, stream_ptr(dev)), "tcx_prior_forward")
        _run_h2_or_fp32(run, dev)
        return out


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
        if isinstance(model, DiffusionPriorFiLM) and z.is_cuda:
            if n > 1 and eta != 0.0:
                raise NotImplementedError("eta != 0 not implemented in this minimal version")
            # one native call: tcx_prior_ddim_sample (csrc/prior.hip)
            pk = model._tcx(device)
            a_t = [float(abar[ts[i]]) for i in range(n)]
            a_p = [float(abar[ts[i + 1]]) if i + 1 < n else 1.0 for i in range(n)]
            yci = y_cat.to(device=device, dtype=torch.int64).contiguous()
            ycv = y_cont.to(device=device, dtype=torch.float32).contiguous()
            L = lib()
            nb = int(L.tcx_prior_workspace(ctypes.byref(pk.net), B, n))
            ws = TF._ws(device, nb)
            z_init = z.clone()

            def run(ovf):
                z.copy_(z_init)
                check(L.tcx_prior_ddim_sample(ctypes.byref(pk.net), ptr(yci), ptr(ycv), B, (c_ll * n)(*ts),
                                              (ctypes.c_float * n)(*a_t), (ctypes.c_float * n)(*a_p), n, ptr(z),
                                              ptr(ovf), ptr(ws), nb, st), "tcx_prior_ddim_sample")
            _run_h2_or_fp32(run, device)
            return z
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
