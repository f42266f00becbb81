"""MI355X-native drop-in for toycrystals.models.sde_score_model.

Mirrors /root/reference/src/toycrystals/models/sde_score_model.py: same class and function
names, constructor signatures, attributes, submodule names (so `state_dict` keys and the seeded
default initialisation are identical: `torch.manual_seed(s); CondUNetTiny(...)` gives the same
weights as the reference) and the same error behaviour.  The arithmetic runs in libtcx (HIP,
gfx950): the nn.Modules here are parameter containers only.  Tensors must live on the GPU
(`device="cuda"` is the MI355X under PyTorch-ROCm); there is no CPU path.

Reference map:
  timestep_embedding :17-32, ConditionEmbedding :35-82, _gn_groups/_ConvBlock :89-111,
  SelfAttention2d :114-167, CondUNetTiny :170-266, VPSDE :273-298, save_sde_samples :301-355,
  diffusion_loss_eps :358-399, predict_eps_cfg :402-423, _probflow_drift :426-449,
  sample_probability_flow_ode :452-504, sample_reverse_sde_euler_maruyama :507-569.
"""
from __future__ import annotations

import ctypes
import math
import warnings
from dataclasses import dataclass
from typing import Optional, Tuple

import torch
import torch.nn as nn

from .. import _lib
from .. import functional as TF
from .._lib import (_CONV_NAMES, TCX_SAMPLE_X0_HAT, TCX_SCAL, TcxConv, TcxUnet, check, lib, ptr,
                    require_gpu_tensor, stream_ptr)


# =========================
# Embeddings (host-side helpers with the reference's semantics)
# =========================

def timestep_embedding(t: torch.Tensor, dim: int) -> torch.Tensor:
    """Continuous-time sinusoidal embedding [cos, sin] of 2*pi*t (sde_score_model.py:17-32).
    Kept as a plain tensor function for API parity; the U-Net computes it inside k_cond."""
    half = dim // 2
    freqs = torch.exp(-math.log(10_000.0) * torch.arange(half, device=t.device, dtype=torch.float32)
                      / max(half - 1, 1))
    args = (2.0 * math.pi) * t.float().unsqueeze(1) * freqs.unsqueeze(0)
    emb = torch.cat([torch.cos(args), torch.sin(args)], dim=1)
    if dim % 2 == 1:
        emb = torch.nn.functional.pad(emb, (0, 1))
    return emb


class ConditionEmbedding(nn.Module):
    """Parameter container of (y_cat, y_cont) -> emb (sde_score_model.py:35-82).
    Evaluated by libtcx k_cond (null token = n_types for CFG)."""

    def __init__(self, n_types: int, y_cont_dim: int, emb_dim: int) -> None:
        super().__init__()
        self.n_types = int(n_types)
        self.y_cont_dim = int(y_cont_dim)
        self.emb_dim = int(emb_dim)
        if self.y_cont_dim < 3:
            raise ValueError("theta_sincos requires y_cont_dim >= 3 (needs indices 1 and 2).")
        self.cat_emb = nn.Embedding(self.n_types + 1, emb_dim)
        self.cont_mlp = nn.Sequential(nn.Linear(self.y_cont_dim, emb_dim), nn.SiLU(), nn.Linear(emb_dim, emb_dim))
        self.out = nn.Sequential(nn.SiLU(), nn.Linear(emb_dim * 2, emb_dim))


def _gn_groups(ch: int) -> int:
    for g in (8, 4, 2):
        if ch % g == 0:
            return g
    return 1


class _ConvBlock(nn.Module):
    def __init__(self, in_ch: int, out_ch: int) -> None:
        super().__init__()
        g = _gn_groups(out_ch)
        self.net = nn.Sequential(
            nn.Conv2d(in_ch, out_ch, kernel_size=3, padding=1, padding_mode="circular"),
            nn.GroupNorm(num_groups=g, num_channels=out_ch),
            nn.SiLU(),
            nn.Conv2d(out_ch, out_ch, kernel_size=3, padding=1, padding_mode="circular"),
            nn.GroupNorm(num_groups=g, num_channels=out_ch),
            nn.SiLU(),
        )


class SelfAttention2d(nn.Module):
    def __init__(self, ch: int, num_heads: int = 4) -> None:
        super().__init__()
        if ch % num_heads != 0:
            raise ValueError(f"ch ({ch}) must be divisible by num_heads ({num_heads})")
        self.ch = int(ch)
        self.num_heads = int(num_heads)
        self.head_dim = self.ch // self.num_heads
        self.norm = nn.GroupNorm(num_groups=_gn_groups(self.ch), num_channels=self.ch)
        self.qkv = nn.Conv2d(self.ch, 3 * self.ch, kernel_size=1, padding=0)
        self.proj = nn.Conv2d(self.ch, self.ch, kernel_size=1, padding=0)


def _round_up(v: int, a: int) -> int:
    return (v + a - 1) // a * a


def _cout_pad(cout: int) -> int:
    return _round_up(cout, 32)


def _pack_frag(L, wh, cpad, kpad, cin, ks, st):
    """Fragment-ordered copy of a packed h2 / bf16 conv weight: 3x3 (tcx_pack_conv_weight_h2_frag) or
    4x4 stride-2 (tcx_pack_conv_weight_h2_frag4); None where no fragment kernel covers the shape."""
    if ks == 3 and kpad == 9 * cin:
        nfb, fn = int(L.tcx_conv_weight_h2_frag_bytes(cpad, cin)), L.tcx_pack_conv_weight_h2_frag
    elif ks == 4 and kpad == 16 * cin:
        nfb, fn = int(L.tcx_conv_weight_h2_frag4_bytes(cpad, cin)), L.tcx_pack_conv_weight_h2_frag4
    else:
        return None
    if not nfb:
        return None
    whf = torch.empty(nfb // 4, device=wh.device, dtype=torch.float32)
    check(fn(wh.data_ptr(), whf.data_ptr(), cpad, kpad, cin, st), "pack conv weight frag")
    return whf


class _UNetPack:
    """Device-resident packed weights + the tcx_unet descriptor for one CondUNetTiny."""

    def __init__(self, model: "CondUNetTiny", device: torch.device) -> None:
        self.device = device
        self.keep = []  # tensors referenced by raw pointers in the descriptor
        L = lib()
        st = stream_ptr(device)
        net = TcxUnet()
        net.base_ch = model.base_ch
        net.emb_dim = model.cond_emb.emb_dim
        net.cond_ch = model.cond_ch
        net.time_ch = model.time_ch
        net.n_types = model.n_types
        net.y_cont_dim = model.y_cont_dim
        net.heads = model.attn.num_heads
        # the f16x3 split convs need every conv source channel count % 32 (base_ch % 32 == 0)
        self.split_ok = model.base_ch % 32 == 0
        self._warned_bf16 = False
        self.ovf = torch.zeros(4, device=device, dtype=torch.int32)
        net.h2_ovf = self.ovf.data_ptr()
        net.precision = 0

        def dev(t: torch.Tensor) -> int:
            t = t.detach().to(device=device, dtype=torch.float32).contiguous()
            self.keep.append(t)
            return t.data_ptr()

        def lin_t(m: nn.Linear):
            return dev(m.weight.detach().t()), dev(m.bias)

        net.time_w1t, net.time_b1 = lin_t(model.time_mlp[0])
        net.time_w2t, net.time_b2 = lin_t(model.time_mlp[2])
        net.ttm_wt, net.ttm_b = lin_t(model.to_time_map)
        net.tcm_wt, net.tcm_b = lin_t(model.to_cond_map)
        ce = model.cond_emb
        net.cat_emb = dev(ce.cat_emb.weight)
        net.cmlp_w1t, net.cmlp_b1 = lin_t(ce.cont_mlp[0])
        net.cmlp_w2t, net.cmlp_b2 = lin_t(ce.cont_mlp[2])
        net.cout_wt, net.cout_b = lin_t(ce.out[1])

        def conv(m: nn.Conv2d, weight: Optional[torch.Tensor] = None) -> TcxConv:
            w = (m.weight if weight is None else weight).detach().to(device=device, dtype=torch.float32).contiguous()
            cout, cin, ks, _ = w.shape
            kpad = _round_up(ks * ks * cin, 32)
            cpad = _cout_pad(cout)
            wpk = torch.empty((cpad, kpad), device=device, dtype=torch.float32)
            check(L.tcx_pack_conv_weight(w.data_ptr(), wpk.data_ptr(), cout, cin, ks, cpad, kpad, st),
                  "pack conv weight")
            self.keep.extend([w, wpk])
            wh = whs = whf = None
            if self.split_ok:
                wh = torch.empty((cpad, kpad), device=device, dtype=torch.float32)  # h2: 4 B per element
                whs = torch.empty(4, device=device, dtype=torch.float32)
                check(L.tcx_pack_conv_weight_h2(wpk.data_ptr(), wh.data_ptr(), whs.data_ptr(), cpad, kpad, st),
                      "pack conv weight h2")
                self.keep.extend([wh, whs])
                # fragment-ordered copy for the 3x3 kernels (k_conv3g / k_conv3l*) and the 4x4/s2
                # downsample kernel k_conv4s2g (their B fragments are DMA'd / loaded straight from it)
                whf = _pack_frag(L, wh, cpad, kpad, cin, ks, st)
                if whf is not None:
                    self.keep.append(whf)
            return TcxConv(wpk.data_ptr(), dev(m.bias), cin, cout, ks, kpad, cpad, ptr(wh), ptr(whs), ptr(whf))

        w0 = model.down1.net[0].weight.detach()
        net.down1_0 = conv(model.down1.net[0], w0[:, :1])
        net.map_wsum = dev(w0[:, 1:].to(torch.float64).sum(dim=(2, 3)).to(torch.float32))
        net.down1_1 = conv(model.down1.net[3])
        net.ds1 = conv(model.ds1)
        net.down2_0 = conv(model.down2.net[0])
        net.down2_1 = conv(model.down2.net[3])
        net.ds2 = conv(model.ds2)
        net.mid_0 = conv(model.mid.net[0])
        net.mid_1 = conv(model.mid.net[3])
        net.qkv = conv(model.attn.qkv)
        net.proj = conv(model.attn.proj)
        net.us2 = conv(model.us2_conv)
        net.up2_0 = conv(model.up2.net[0])
        net.up2_1 = conv(model.up2.net[3])
        net.us1 = conv(model.us1_conv)
        net.up1_0 = conv(model.up1.net[0])
        net.up1_1 = conv(model.up1.net[3])
        wo = model.out.weight.detach()
        net.out_w = dev(wo[0].reshape(wo.shape[1], 9))
        net.out_b = float(model.out.bias.detach().float().cpu()[0])
        norms = [model.down1.net[1], model.down1.net[4], model.down2.net[1], model.down2.net[4], model.mid.net[1],
                 model.mid.net[4], model.attn.norm, model.up2.net[1], model.up2.net[4], model.up1.net[1],
                 model.up1.net[4]]
        for i, gnm in enumerate(norms):
            net.gn_w[i] = dev(gnm.weight)
            net.gn_b[i] = dev(gnm.bias)
        self.net = net
        self.ws = None
        self._st = st
        self._bf = None  # bf16 packs, built on first use

    def _bf16_packs(self):
        """{conv name: (wh, wscale, whf)} in the bf16 single-product layout (tcx_pack_conv_weight_bf16)."""
        if self._bf is None:
            L = lib()
            packs = {}
            for name in _CONV_NAMES:
                c = getattr(self.net, name)
                if not c.wh:
                    continue
                wh = torch.empty((c.cout_pad, c.kpad), device=self.device, dtype=torch.float32)
                ws = torch.empty(4, device=self.device, dtype=torch.float32)
                check(L.tcx_pack_conv_weight_bf16(c.w, wh.data_ptr(), ws.data_ptr(), c.cout_pad, c.kpad, self._st),
                      "pack conv weight bf16")
                whf = _pack_frag(L, wh, c.cout_pad, c.kpad, c.cin, c.ks, self._st) if c.whf else None
                packs[name] = (wh, ws, whf)
            self._bf = packs
        return self._bf

    def run(self, H: int, W: int, launch) -> None:
        """Run `launch()` (which must (re)initialise its outputs) with the configured conv
        precision; if an f16x3 run raised the range flag, re-run it in fp32 (one host sync).
        "bf16" (config 5's precision) runs where the split attention applies, else f16x3."""
        prec = _lib.conv_precision()
        split = prec in ("f16x3", "bf16") and self.split_ok and ((H // 4) * (W // 4)) % 32 == 0
        bf = split and prec == "bf16" and ((H // 4) * (W // 4)) % 256 == 0
        if prec == "bf16" and not bf and not self._warned_bf16:
            self._warned_bf16 = True
            warnings.warn(f"libtcx: bf16 precision needs (H/4)*(W/4) % 256 == 0 (the split attention); "
                          f"{H}x{W} runs in {'f16x3' if split else 'fp32'}")
        _lib.note_used_precision("bf16" if bf else ("f16x3" if split else "fp32"))
        if bf:
            saved = {}
            for name, (wh, ws, whf) in self._bf16_packs().items():
                c = getattr(self.net, name)
                saved[name] = (c.wh, c.wscale, c.whf)
                c.wh, c.wscale, c.whf = wh.data_ptr(), ws.data_ptr(), ptr(whf)
            try:
                self.net.precision = 2
                launch()
            finally:
                for name, (a, b, f) in saved.items():
                    c = getattr(self.net, name)
                    c.wh, c.wscale, c.whf = a, b, f
                self.net.precision = 0
            return
        self.net.precision = 1 if split else 0
        if split:
            self.ovf.zero_()
        launch()
        if split and int(self.ovf[0].item()) != 0:
            warnings.warn("libtcx: an activation left the f16 range of the split path; recomputed in fp32")
            _lib.note_used_precision("fp32")
            self.net.precision = 0
            launch()
        self.net.precision = 0

    def workspace(self, Bt: int, H: int, W: int, extra: int = 0, need: Optional[int] = None) -> Tuple[torch.Tensor, int]:
        """The caller-owned workspace of a libtcx call (grown, never shrunk): `need` bytes when the
        call has its own size query (tcx_sde/ode_workspace_size), else one U-Net evaluation's."""
        if need is None:
            need = int(lib().tcx_unet_workspace_size(ctypes.byref(self.net), Bt, H, W)) + extra
        if self.ws is None or self.ws.numel() < need:
            self.ws = torch.empty(need, dtype=torch.uint8, device=self.device)
        return self.ws, self.ws.numel()


class CondUNetTiny(nn.Module):
    """Tiny conditional U-Net predicting eps_hat = eps_theta(x_t, t, c) (sde_score_model.py:170-266)."""

    def __init__(self, n_types: int, y_cont_dim: int, base_ch: int = 32, emb_dim: int = 128, cond_ch: int = 8,
                 time_ch: int = 8) -> None:
        super().__init__()
        self.n_types = int(n_types)
        self.y_cont_dim = int(y_cont_dim)
        self.base_ch = int(base_ch)
        self.cond_ch = int(cond_ch)
        self.time_ch = int(time_ch)
        self.cond_emb = ConditionEmbedding(n_types=self.n_types, y_cont_dim=self.y_cont_dim, emb_dim=emb_dim)
        self.time_mlp = nn.Sequential(nn.Linear(emb_dim, emb_dim), nn.SiLU(), nn.Linear(emb_dim, emb_dim))
        self.to_cond_map = nn.Linear(emb_dim, cond_ch)
        self.to_time_map = nn.Linear(emb_dim, time_ch)
        in_ch = 1 + cond_ch + time_ch
        self.down1 = _ConvBlock(in_ch, base_ch)
        self.ds1 = nn.Conv2d(base_ch, base_ch, kernel_size=4, stride=2, padding=1, padding_mode="circular")
        self.down2 = _ConvBlock(base_ch, base_ch * 2)
        self.ds2 = nn.Conv2d(base_ch * 2, base_ch * 2, kernel_size=4, stride=2, padding=1, padding_mode="circular")
        self.mid = _ConvBlock(base_ch * 2, base_ch * 2)
        self.attn = SelfAttention2d(base_ch * 2, num_heads=4)
        self.us2 = nn.Upsample(scale_factor=2, mode="bilinear", align_corners=False)
        self.us2_conv = nn.Conv2d(base_ch * 2, base_ch * 2, kernel_size=3, padding=1, padding_mode="circular")
        self.up2 = _ConvBlock(base_ch * 4, base_ch)
        self.us1 = nn.Upsample(scale_factor=2, mode="bilinear", align_corners=False)
        self.us1_conv = nn.Conv2d(base_ch, base_ch, kernel_size=3, padding=1, padding_mode="circular")
        self.up1 = _ConvBlock(base_ch * 2, base_ch)
        self.out = nn.Conv2d(base_ch, 1, kernel_size=3, padding=1, padding_mode="circular")
        self._pack: Optional[_UNetPack] = None
        self._pack_key = None

    # ---------------------------------------------------------------- packing
    def _weights_key(self, device):
        return (device,) + tuple((p.data_ptr(), p._version) for p in self.parameters())

    def tcx_pack(self, device: Optional[torch.device] = None) -> _UNetPack:
        """(Re)pack the weights for libtcx when they changed (new storage or in-place update)."""
        device = torch.device(device) if device is not None else next(self.parameters()).device
        if device.type != "cuda":
            raise _lib.TcxError("CondUNetTiny runs on the MI355X only: move the model and inputs to 'cuda'")
        key = self._weights_key(device)
        if self._pack is None or self._pack_key != key:
            with torch.no_grad():
                self._pack = _UNetPack(self, device)
            self._pack_key = key
        return self._pack

    # ---------------------------------------------------------------- forward
    def _check_inputs(self, x_t, t, y_cat, y_cont):
        require_gpu_tensor(x_t, "x_t")
        if x_t.dim() != 4 or x_t.shape[1] != 1:
            raise ValueError(f"x_t must be [B,1,H,W], got {tuple(x_t.shape)}")
        B = x_t.shape[0]
        t = torch.as_tensor(t, device=x_t.device).float().expand(B).contiguous()
        y_cat = y_cat.to(device=x_t.device, dtype=torch.int64).contiguous()
        y_cont = y_cont.to(device=x_t.device, dtype=torch.float32).contiguous()
        return x_t.float().contiguous(), t, y_cat, y_cont

    def forward(self, x_t: torch.Tensor, t: torch.Tensor, y_cat: torch.Tensor, y_cont: torch.Tensor) -> torch.Tensor:
        x, t, y_cat, y_cont = self._check_inputs(x_t, t, y_cat, y_cont)
        if torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters()):
            return self._forward_train(x, t, y_cat, y_cont)
        return _eval_eps(self, x, t, 1, y_cat, y_cont, 0.0)

    # ---------------------------------------------------------------- training forward
    def _forward_train(self, x: torch.Tensor, t: torch.Tensor, y_cat: torch.Tensor,
                       y_cont: torch.Tensor) -> torch.Tensor:
        """Differentiable forward (sde_score_model.py:243-266) as a chain of libtcx autograd
        Functions (functional.py); activations NHWC.  Same arithmetic as the fused evaluator,
        with every intermediate kept for the backward."""
        B, _, H, W = x.shape
        E = self.cond_emb.emb_dim
        ce = self.cond_emb
        # conditioning (:195-202, :35-82, :227-241)
        te = torch.empty((B, E), device=x.device)
        yv = torch.empty((B, self.y_cont_dim), device=x.device)
        yc = torch.empty((B,), device=x.device, dtype=torch.int64)
        check(lib().tcx_cond_inputs(ptr(t), ptr(y_cat), ptr(y_cont), B, E, self.n_types, self.y_cont_dim, ptr(te),
                                    ptr(yv), ptr(yc), stream_ptr(x.device)), "tcx_cond_inputs")
        temb = TF.linear(TF.act(TF.linear(te, self.time_mlp[0]), TF.ACT_SILU), self.time_mlp[2])
        t_map = TF.linear(temb, self.to_time_map)
        e_cat = TF.EmbeddingFn.apply(yc, ce.cat_emb.weight)
        e_cont = TF.linear(TF.act(TF.linear(yv, ce.cont_mlp[0]), TF.ACT_SILU), ce.cont_mlp[2])
        cemb = TF.linear(TF.act(TF.cat_cols(e_cat, e_cont), TF.ACT_SILU), ce.out[1])
        c_map = TF.linear(cemb, self.to_cond_map)
        maps = TF.cat_cols(t_map, c_map)  # channel order of torch.cat([x_t, t_map, c_map]) (:246)

        def block(h, blk, x2=None):
            h = TF.group_norm_act(TF.conv2d(h, x2, blk.net[0]), blk.net[1], True)
            return TF.group_norm_act(TF.conv2d(h, None, blk.net[3]), blk.net[4], True)

        d1 = self.down1.net
        h = TF.FirstConvFn.apply(x.view(B, H, W, 1), maps, d1[0].weight, d1[0].bias)
        h = TF.group_norm_act(h, d1[1], True)
        h1 = TF.group_norm_act(TF.conv2d(h, None, d1[3]), d1[4], True)
        h = TF.conv2d(h1, None, self.ds1)
        h2 = block(h, self.down2)
        h = TF.conv2d(h2, None, self.ds2)
        h = block(h, self.mid)
        # attention (:140-167): x_in + proj(SDPA(qkv(GN(x_in))))
        at = self.attn
        Bq, Hq, Wq, Cq = h.shape
        qkv = TF.conv2d(TF.group_norm_act(h, at.norm, False), None, at.qkv)
        a = TF.AttentionFn.apply(qkv.view(Bq, Hq * Wq, 3 * Cq), at.num_heads)
        h = TF.conv2d(a.view(Bq, Hq, Wq, Cq), None, at.proj, resid=h)
        h = TF.conv2d(TF.Upsample2xFn.apply(h), None, self.us2_conv)
        h = block(h, self.up2, x2=h2)
        h = TF.conv2d(TF.Upsample2xFn.apply(h), None, self.us1_conv)
        h = block(h, self.up1, x2=h1)
        eps = TF.conv2d(h, None, self.out)  # [B, H, W, 1] == [B, 1, H, W]
        return eps.view(B, 1, H, W)


def _eval_eps(model: CondUNetTiny, x, t, t_per_sample, y_cat, y_cont, guidance: float) -> torch.Tensor:
    B, _, H, W = x.shape
    pk = model.tcx_pack(x.device)
    Bt = 2 * B if guidance > 0.0 else B
    ws, nbytes = pk.workspace(Bt, H, W)
    eps = torch.empty_like(x)
    pk.run(H, W, lambda: check(lib().tcx_unet_eval(ctypes.byref(pk.net), ptr(x), None, ptr(t), t_per_sample, ptr(y_cat),
                                                   ptr(y_cont), B, H, W, float(guidance), 0, None, None, 0, 0, None,
                                                   ptr(eps), ptr(ws), nbytes, stream_ptr(x.device)), "tcx_unet_eval"))
    return eps


# =========================
# OU/VP-SDE + loss + sampler
# =========================

@dataclass(frozen=True)
class VPSDE:
    """VP SDE dx = -0.5 beta(t) x dt + sqrt(beta(t)) dW with linear beta (sde_score_model.py:273-298)."""
    beta_min: float = 0.1
    beta_max: float = 20.0

    def beta(self, t: torch.Tensor) -> torch.Tensor:
        return self.beta_min + t * (self.beta_max - self.beta_min)

    def int_beta(self, t: torch.Tensor) -> torch.Tensor:
        return self.beta_min * t + 0.5 * (self.beta_max - self.beta_min) * (t ** 2)

    def alpha(self, t: torch.Tensor) -> torch.Tensor:
        return torch.exp(-0.5 * self.int_beta(t))

    def sigma(self, t: torch.Tensor) -> torch.Tensor:
        a = self.alpha(t)
        return torch.sqrt(torch.clamp(1.0 - a * a, min=1e-8))


def step_table(sde: VPSDE, n_steps: int, t_end: float) -> torch.Tensor:
    """Per-step scalars [n_steps+1, 8] = {t, t_next, dt, beta, sigma, sqrt(beta), sqrt|dt|, alpha},
    computed on the host with the reference's fp32 torch formulas (quadratic grid
    sde_score_model.py:540-541, per-step scalars :545-550, final projection :562-565), so the
    device update sees exactly the reference's scalar values."""
    u = torch.linspace(0.0, 1.0, n_steps + 1)
    ts = t_end + (1.0 - t_end) * (1.0 - u) ** 2
    t_next = torch.cat([ts[1:], ts[-1:]])
    dt = t_next - ts
    beta = sde.beta(ts)
    tab = torch.stack([ts, t_next, dt, beta, sde.sigma(ts), torch.sqrt(beta), torch.sqrt(torch.abs(dt)),
                       sde.alpha(ts)], dim=1).to(torch.float32)
    assert tab.shape[1] == TCX_SCAL
    return tab.contiguous()


@torch.no_grad()
def save_sde_samples(model: CondUNetTiny, sde: VPSDE, out_path: str, device: torch.device, n: int = 36,
                     theta_max: float = math.pi / 3.0, steps: int = 200, cfg: float = 0.0, t_end: float = 1e-3,
                     sampler: str = "ode") -> None:
    """Save a 6x6 grid: cycle lattice types, sweep theta in [0, pi/3] (sde_score_model.py:301-355)."""
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt

    model.eval()
    y_cat = torch.tensor([i % model.n_types for i in range(n)], device=device, dtype=torch.int64)
    thetas = torch.linspace(0.0, theta_max, steps=n, device=device)
    y_cont = torch.zeros((n, model.y_cont_dim), device=device)
    y_cont[:, 1] = thetas
    kw = dict(model=model, sde=sde, y_cat=y_cat, y_cont=y_cont, img_shape=(n, 1, 64, 64), n_steps=steps,
              guidance_scale=cfg, t_end=t_end)
    if sampler == "ode":
        x = sample_probability_flow_ode(**kw)
    elif sampler == "sde":
        x = sample_reverse_sde_euler_maruyama(**kw)
    else:
        raise ValueError(f"Unknown sampler='{sampler}'. Use 'ode' or 'sde'.")
    fig, axes = plt.subplots(6, 6, figsize=(6, 6))
    fig.suptitle(f"{sampler} | steps={steps} | cfg={cfg:.2f} | t_end={t_end:g}", fontsize=10)
    for i, ax in enumerate(axes.flat):
        ax.imshow(x[i, 0].cpu(), cmap="gray", vmin=0.0, vmax=1.0)
        ax.axis("off")
    fig.tight_layout()
    fig.savefig(out_path, dpi=200)
    plt.close(fig)


def diffusion_loss_eps(model: CondUNetTiny, sde: VPSDE, x0: torch.Tensor, y_cat: torch.Tensor,
                       y_cont: torch.Tensor, p_uncond: float = 0.1, t_power: float = 1.0, *,
                       draws: Optional[Tuple[torch.Tensor, torch.Tensor, Optional[torch.Tensor]]] = None
                       ) -> torch.Tensor:
    """Eps-prediction denoising loss with CFG condition dropout (sde_score_model.py:358-399).

    Same RNG draw order as the reference: u = rand(B), eps = randn_like(x0), then (p_uncond > 0)
    rand(B) for the dropout, from torch's generator on x0's device.  `draws=(u, eps, drop_u)`
    injects them instead (parity runs against the reference's CPU draws).  The data path
    (t = u^p, alpha/sigma, x_t, dropout, MSE and its gradient) runs in libtcx kernels."""
    require_gpu_tensor(x0, "x0")
    device = x0.device
    B = x0.shape[0]
    if draws is None:
        u = torch.rand((B,), device=device)
        eps = torch.randn_like(x0)
        drop_u = torch.rand((B,), device=device) if p_uncond > 0.0 else None
    else:
        u, eps, drop_u = draws
        u = u.to(device=device, dtype=torch.float32).contiguous()
        eps = eps.to(device=device, dtype=torch.float32).contiguous()
        drop_u = drop_u.to(device=device, dtype=torch.float32).contiguous() if (
            drop_u is not None and p_uncond > 0.0) else None
    x0 = x0.to(torch.float32).contiguous()
    eps = eps.contiguous()
    HW = x0[0].numel()
    st = stream_ptr(device)
    L = lib()
    t = torch.empty((B,), device=device)
    x_t = torch.empty_like(x0)
    check(L.tcx_qsample_vp(ptr(x0), ptr(eps), ptr(u), float(t_power), float(sde.beta_min),
                           float(0.5 * (sde.beta_max - sde.beta_min)), B, HW, ptr(t), ptr(x_t), st), "tcx_qsample_vp")
    yc = torch.empty((B,), device=device, dtype=torch.int64)
    yv = torch.empty((B, y_cont.shape[1]), device=device)
    y_cat = y_cat.to(device=device, dtype=torch.int64).contiguous()
    y_cont = y_cont.to(device=device, dtype=torch.float32).contiguous()
    check(L.tcx_cond_drop(ptr(y_cat), ptr(y_cont), ptr(drop_u), float(p_uncond), B, y_cont.shape[1], model.n_types,
                          ptr(yc), ptr(yv), st), "tcx_cond_drop")
    eps_hat = model(x_t, t, yc, yv)
    return TF.mse_loss(eps_hat, eps)


@torch.no_grad()
def predict_eps_cfg(model: CondUNetTiny, x_t: torch.Tensor, t: torch.Tensor, y_cat: torch.Tensor,
                    y_cont: torch.Tensor, guidance_scale: float) -> torch.Tensor:
    """eps = eps_u + s (eps_c - eps_u) (sde_score_model.py:402-423).  Both halves run as ONE
    2B-batch U-Net evaluation (null token n_types, y_cont = 0 first) combined in the head."""
    x, t, y_cat, y_cont = model._check_inputs(x_t, t, y_cat, y_cont)
    return _eval_eps(model, x, t, 1, y_cat, y_cont, float(guidance_scale) if guidance_scale > 0.0 else 0.0)


def _probflow_drift(model, sde, x, t, y_cat, y_cont, guidance_scale):
    """PF-ODE drift -0.5 beta x - 0.5 beta score, score = -eps/sigma (sde_score_model.py:426-449)."""
    B = x.shape[0]
    beta_t = sde.beta(t).view(B, 1, 1, 1)
    sigma_t = sde.sigma(t).view(B, 1, 1, 1)
    eps_hat = predict_eps_cfg(model, x, t, y_cat, y_cont, guidance_scale=guidance_scale)
    score = -eps_hat / sigma_t
    return -0.5 * beta_t * x - 0.5 * beta_t * score


def _sampler_prologue(model, y_cat, y_cont, img_shape, t_end):
    device = y_cat.device
    B, C, H, W = img_shape
    assert C == 1
    t_end = float(t_end)
    if not (0.0 < t_end < 1.0):
        raise ValueError(f"t_end must be in (0,1), got {t_end}")
    require_gpu_tensor(y_cat, "y_cat")
    return device, B, H, W, t_end, y_cat.to(torch.int64).contiguous(), y_cont.to(torch.float32).contiguous()


def host_noise(shape, n_draws: int, generator: Optional[torch.Generator] = None) -> torch.Tensor:
    """Noise in the reference's CPU draw order: x_T = randn(shape), then one randn_like per step
    (sde_score_model.py:537,557).  Parity mode: copy this to the device and pass as `noise`."""
    return torch.stack([torch.randn(shape, generator=generator) for _ in range(n_draws)])


@torch.no_grad()
def sample_reverse_sde_euler_maruyama(model: CondUNetTiny, sde: VPSDE, y_cat: torch.Tensor, y_cont: torch.Tensor,
                                      img_shape: Tuple[int, int, int, int], n_steps: int = 200,
                                      guidance_scale: float = 0.0, t_end: float = 1e-3, *,
                                      noise: Optional[torch.Tensor] = None,
                                      seed: Optional[int] = None,
                                      return_x0_hat: bool = False,
                                      elem_offset: int = 0) -> torch.Tensor:
    """Reverse-time SDE via Euler-Maruyama, t: 1 -> t_end (sde_score_model.py:507-569).

    The whole loop runs natively (tcx_sde_sample): per step ONE fused CFG-doubled U-Net
    evaluation whose head applies the EM update in place.
    Noise: `noise` [n_steps+1, B, 1, H, W] (x_T then one z per step, e.g. host_noise(...)) for
    bit-reproducible parity runs; otherwise x_T and z come from in-kernel Philox4x32-10 keyed by
    `seed` (default: drawn from torch's global CPU generator, so torch.manual_seed governs it).
    `return_x0_hat=True` returns the projection x0_hat = (x - sigma eps)/max(alpha, 1e-6) of :566
    itself, before the reference's (x0_hat + 1)/2 map and clamp (:568-569).
    `elem_offset`: Philox element offset of x[0] in a larger batch (a data-parallel shard, see
    dist.sample_sharded): rows [s, e) of a batch sampled with elem_offset = s*H*W equal those rows of
    the whole batch sampled in one call with the same seed.
    """
    device, B, H, W, t_end, y_cat, y_cont = _sampler_prologue(model, y_cat, y_cont, img_shape, t_end)
    pk = model.tcx_pack(device)
    tab = step_table(sde, n_steps, t_end).to(device)
    L = lib()
    st = stream_ptr(device)
    if seed is None:
        seed = int(torch.randint(0, 2 ** 62, (1,)).item())
    x = torch.empty((B, 1, H, W), device=device, dtype=torch.float32)
    zs = None
    if noise is not None:
        noise = noise.to(device=device, dtype=torch.float32).contiguous()
        if noise.shape[0] != n_steps + 1 or noise[0].numel() != x.numel():
            raise ValueError(f"noise must be [n_steps+1, B, 1, H, W], got {tuple(noise.shape)}")
        zs = noise[1:]
    g = float(guidance_scale) if guidance_scale > 0.0 else 0.0
    ws, nbytes = pk.workspace(2 * B if g > 0 else B, H, W,
                              need=int(L.tcx_sde_workspace_size(ctypes.byref(pk.net), B, H, W, int(n_steps), g)))
    flags = TCX_SAMPLE_X0_HAT if return_x0_hat else 0

    def launch():
        if noise is not None:
            x.copy_(noise[0].view_as(x))
        else:
            check(L.tcx_randn_at(ptr(x), x.numel(), seed, 0, int(elem_offset), st), "tcx_randn")
        check(L.tcx_sde_sample_shard(ctypes.byref(pk.net), ptr(x), ptr(y_cat), ptr(y_cont), B, H, W, int(n_steps), g,
                                     ptr(tab), ptr(zs) if zs is not None else None, seed, flags, int(elem_offset),
                                     ptr(ws), nbytes, st), "tcx_sde_sample")
    pk.run(H, W, launch)
    return x


@torch.no_grad()
def sample_probability_flow_ode(model: CondUNetTiny, sde: VPSDE, y_cat: torch.Tensor, y_cont: torch.Tensor,
                                img_shape: Tuple[int, int, int, int], n_steps: int = 200,
                                guidance_scale: float = 0.0, t_end: float = 1e-3, *,
                                x_init: Optional[torch.Tensor] = None,
                                seed: Optional[int] = None,
                                return_x0_hat: bool = False,
                                elem_offset: int = 0) -> torch.Tensor:
    """Deterministic probability-flow ODE with Heun steps (sde_score_model.py:452-504).
    `return_x0_hat=True`: the unclamped projection of :500 instead of the image of :503-504.
    `elem_offset`: Philox element offset of x_T[0] in a larger batch (as for the reverse SDE)."""
    device, B, H, W, t_end, y_cat, y_cont = _sampler_prologue(model, y_cat, y_cont, img_shape, t_end)
    pk = model.tcx_pack(device)
    tab = step_table(sde, n_steps, t_end).to(device)
    L = lib()
    st = stream_ptr(device)
    x = torch.empty((B, 1, H, W), device=device, dtype=torch.float32)
    if x_init is None and seed is None:
        seed = int(torch.randint(0, 2 ** 62, (1,)).item())
    g = float(guidance_scale) if guidance_scale > 0.0 else 0.0
    ws, nbytes = pk.workspace(2 * B if g > 0 else B, H, W,
                              need=int(L.tcx_ode_workspace_size(ctypes.byref(pk.net), B, H, W, int(n_steps), g)))

    def launch():
        if x_init is not None:
            x.copy_(x_init.to(device=device, dtype=torch.float32).view_as(x))
        else:
            check(L.tcx_randn_at(ptr(x), x.numel(), seed, 0, int(elem_offset), st), "tcx_randn")
        check(L.tcx_ode_sample_ex(ctypes.byref(pk.net), ptr(x), ptr(y_cat), ptr(y_cont), B, H, W, int(n_steps), g,
                                  ptr(tab), TCX_SAMPLE_X0_HAT if return_x0_hat else 0, ptr(ws), nbytes, st),
              "tcx_ode_sample")
    pk.run(H, W, launch)
    return x
