"""torch-CPU restatement of the VP-SDE score path — TEST INFRASTRUCTURE / CPU BASELINE ONLY.

The same arithmetic as the numpy oracle (oracle/score_model.py) written over torch's CPU ops
(`F.conv2d` on circularly padded inputs, `F.group_norm`, `F.silu`, bilinear `F.interpolate`,
`F.scaled_dot_product_attention`): these are the ATen kernels the reference's nn.Modules call
("Third-party arithmetic"), so this is the reference's CPU arithmetic without
the reference's source.  It serves `bench.py`'s `cpu_baseline` leg (B = 128,
2- and 4-step runs, per-forward fit) and is pinned to the reference goldens by
tests/test_oracle_goldens.py.  Nothing in the product package imports it.

Follows /root/reference/src/toycrystals/models/sde_score_model.py:
  timestep_embedding :17-32, ConditionEmbedding :35-82 (incl. the theta view quirk :75-78),
  _ConvBlock :97-111, SelfAttention2d :140-167, CondUNetTiny.forward :243-266,
  predict_eps_cfg :402-423, sample_reverse_sde_euler_maruyama :507-569.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F


def _groups(ch: int) -> int:
    for g in (8, 4, 2):
        if ch % g == 0:
            return g
    return 1


class TorchScoreUNet:
    """CondUNetTiny forward from a state dict of CPU tensors (the reference's keys)."""

    def __init__(self, sd: dict, n_types: int = 4, dtype=torch.float32):
        self.w = {k: (v.detach().to("cpu", dtype) if v.is_floating_point() else v.detach().cpu())
                  for k, v in sd.items()}
        self.n_types = n_types
        self.dtype = dtype
        self.emb_dim = self.w["time_mlp.0.weight"].shape[1]

    def _lin(self, name, x):
        return F.linear(x, self.w[name + ".weight"], self.w[name + ".bias"])

    def _conv(self, name, x, stride=1, pad=1):
        if pad:
            x = F.pad(x, (pad, pad, pad, pad), mode="circular")
        return F.conv2d(x, self.w[name + ".weight"], self.w[name + ".bias"], stride=stride)

    def _gn(self, name, x):
        return F.group_norm(x, _groups(x.shape[1]), self.w[name + ".weight"], self.w[name + ".bias"], 1e-5)

    def _block(self, name, x):
        h = F.silu(self._gn(name + ".net.1", self._conv(name + ".net.0", x)))
        return F.silu(self._gn(name + ".net.4", self._conv(name + ".net.3", h)))

    def maps(self, t, y_cat, y_cont):
        half = self.emb_dim // 2
        freqs = torch.exp(-math.log(10_000.0) * torch.arange(half, dtype=torch.float32) / max(half - 1, 1))
        args = (2.0 * math.pi) * t.float()[:, None] * freqs[None, :]
        te = torch.cat([torch.cos(args), torch.sin(args)], dim=1).to(self.dtype)
        te = self._lin("time_mlp.2", F.silu(self._lin("time_mlp.0", te)))
        yc = y_cat.long().clamp(0, self.n_types)
        y = y_cont.to(self.dtype).clone()
        theta = y[:, 1]          # a view, as in the reference: y[:,2] = cos(sin(theta))
        y[:, 1] = torch.sin(theta)
        y[:, 2] = torch.cos(theta)
        e_cat = self.w["cond_emb.cat_emb.weight"][yc]
        e_cont = self._lin("cond_emb.cont_mlp.2", F.silu(self._lin("cond_emb.cont_mlp.0", y)))
        ce = self._lin("cond_emb.out.1", F.silu(torch.cat([e_cat, e_cont], dim=1)))
        return torch.cat([self._lin("to_time_map", te), self._lin("to_cond_map", ce)], dim=1)

    def _attn(self, x, heads=4):
        B, C, H, W = x.shape
        d = C // heads
        qkv = self._conv("attn.qkv", self._gn("attn.norm", x), pad=0)
        q, k, v = (z.reshape(B, heads, d, H * W).transpose(2, 3) for z in qkv.chunk(3, dim=1))
        y = F.scaled_dot_product_attention(q, k, v).transpose(2, 3).reshape(B, C, H, W)
        return x + self._conv("attn.proj", y, pad=0)

    @torch.no_grad()
    def __call__(self, x_t, t, y_cat, y_cont):
        B, _, H, W = x_t.shape
        m = self.maps(t, y_cat, y_cont)
        x = torch.cat([x_t.to(self.dtype), m[:, :, None, None].expand(B, m.shape[1], H, W)], dim=1)
        h1 = self._block("down1", x)
        h2 = self._block("down2", self._conv("ds1", h1, stride=2))
        h = self._attn(self._block("mid", self._conv("ds2", h2, stride=2)))
        up = lambda z: F.interpolate(z, scale_factor=2, mode="bilinear", align_corners=False)  # noqa: E731
        h = self._block("up2", torch.cat([self._conv("us2_conv", up(h)), h2], dim=1))
        h = self._block("up1", torch.cat([self._conv("us1_conv", up(h)), h1], dim=1))
        return self._conv("out", h)


def predict_eps_cfg(model: TorchScoreUNet, x, t, y_cat, y_cont, s: float):
    if s <= 0.0:
        return model(x, t, y_cat, y_cont)
    eps_u = model(x, t, torch.full_like(y_cat, model.n_types), torch.zeros_like(y_cont))
    eps_c = model(x, t, y_cat, y_cont)
    return eps_u + s * (eps_c - eps_u)


@torch.no_grad()
def sample_reverse_sde(model: TorchScoreUNet, beta_min, beta_max, y_cat, y_cont, shape, n_steps, s, t_end,
                       generator=None, return_x0_hat=False, noise=None):
    """Reverse-SDE Euler-Maruyama + final projection, draws from `generator` in the reference's
    order (x_T, then one z per step), or taken from `noise` [n_steps+1, *shape]."""
    if noise is not None:
        draws = iter(noise)
        generator = None
    randn = (lambda: next(draws)) if noise is not None else (lambda: torch.randn(shape, generator=generator))  # noqa: E731
    B = shape[0]
    beta = lambda t: beta_min + t * (beta_max - beta_min)  # noqa: E731
    alpha = lambda t: torch.exp(-0.5 * (beta_min * t + 0.5 * (beta_max - beta_min) * t ** 2))  # noqa: E731
    sigma = lambda t: torch.sqrt(torch.clamp(1.0 - alpha(t) ** 2, min=1e-8))  # noqa: E731
    x = randn().to(model.dtype)
    u = torch.linspace(0.0, 1.0, n_steps + 1)
    ts = t_end + (1.0 - t_end) * (1.0 - u) ** 2
    for i in range(n_steps):
        t, tn = ts[i].expand(B), ts[i + 1].expand(B)
        dt = (tn - t).view(B, 1, 1, 1)
        b, sg = beta(t).view(B, 1, 1, 1), sigma(t).view(B, 1, 1, 1)
        score = -predict_eps_cfg(model, x, t, y_cat, y_cont, s) / sg
        drift = (-0.5 * b * x) - (b * score)
        z = randn().to(model.dtype)
        x = x + drift * dt + torch.sqrt(b) * torch.sqrt(torch.abs(dt)) * z
    tf = ts[-1].expand(B)
    a, sg = alpha(tf).view(B, 1, 1, 1), sigma(tf).view(B, 1, 1, 1)
    x0 = (x - sg * predict_eps_cfg(model, x, tf, y_cat, y_cont, s)) / torch.clamp(a, min=1e-6)
    return x0 if return_x0_hat else ((x0 + 1.0) * 0.5).clamp(0.0, 1.0)
