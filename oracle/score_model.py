"""Oracle restatement of the VP-SDE score path (test-only; see oracle/__init__.py).

Follows /root/reference/src/toycrystals/models/sde_score_model.py:
  timestep_embedding        :17-32
  ConditionEmbedding        :35-82
  _gn_groups / _ConvBlock   :89-111
  SelfAttention2d           :114-167
  CondUNetTiny.forward      :243-266 (+ _make_maps :227-241)
  VPSDE                     :273-298
  diffusion_loss_eps        :358-399 (forward value, noise injected)
  predict_eps_cfg           :402-423
  _probflow_drift           :426-449
  sample_probability_flow_ode        :452-504 (noise injected)
  sample_reverse_sde_euler_maruyama  :507-569 (noise injected)

`sd` is a state dict of numpy arrays with the reference's keys.  Noise is passed in
explicitly (the reference draws it from the global torch RNG; the goldens record the
draws), so the restatement itself is deterministic.
"""
from __future__ import annotations

import math

import numpy as np

from . import nn_np as F


def gn_groups(ch: int) -> int:
    for g in (8, 4, 2):
        if ch % g == 0:
            return g
    return 1


def timestep_embedding(t, dim: int, dt=np.float32):
    """Continuous-t sinusoid: freqs = exp(-ln(1e4) k/(half-1)), args = 2*pi*t*freqs, [cos, sin]."""
    half = dim // 2
    k = np.arange(half, dtype=dt)
    freqs = np.exp(dt(-math.log(10_000.0)) * k / dt(max(half - 1, 1)))
    args = (dt(2.0 * math.pi) * t.astype(dt))[:, None] * freqs[None, :]
    emb = np.concatenate([np.cos(args), np.sin(args)], axis=1)
    if dim % 2 == 1:
        emb = np.pad(emb, ((0, 0), (0, 1)))
    return emb


class ScoreUNet:
    """numpy CondUNetTiny(n_types, y_cont_dim, base_ch, emb_dim, cond_ch, time_ch)."""

    def __init__(self, sd: dict, n_types: int = 4, dt=np.float32):
        self.w = {k: np.asarray(v).astype(dt) if np.asarray(v).dtype.kind == "f" else np.asarray(v)
                  for k, v in sd.items()}
        self.n_types = n_types
        self.dt = dt
        self.emb_dim = self.w["time_mlp.0.weight"].shape[1]

    # --- conditioning (sde_score_model.py:35-82, 195-202, 227-241)
    def cond_emb(self, y_cat, y_cont):
        w = self.w
        y_cat = np.clip(y_cat.astype(np.int64), 0, self.n_types)
        y = y_cont.astype(self.dt).copy()
        # theta = y[:, 1] is a VIEW in the reference (:75-78): after y[:,1] = sin(theta) the
        # cos reads the replaced value, so y[:,2] = cos(sin(theta)).
        theta = y[:, 1]
        y[:, 1] = np.sin(theta)
        y[:, 2] = np.cos(theta)
        e_cat = w["cond_emb.cat_emb.weight"][y_cat]
        h = F.silu(F.linear(y, w["cond_emb.cont_mlp.0.weight"], w["cond_emb.cont_mlp.0.bias"]))
        e_cont = F.linear(h, w["cond_emb.cont_mlp.2.weight"], w["cond_emb.cont_mlp.2.bias"])
        return F.linear(F.silu(np.concatenate([e_cat, e_cont], axis=1)),
                        w["cond_emb.out.1.weight"], w["cond_emb.out.1.bias"])

    def maps(self, t, y_cat, y_cont):
        """[B, time_ch + cond_ch] spatially-constant map values ([t_map, c_map] order)."""
        w = self.w
        te = timestep_embedding(t, self.emb_dim, self.dt)
        te = F.linear(F.silu(F.linear(te, w["time_mlp.0.weight"], w["time_mlp.0.bias"])),
                      w["time_mlp.2.weight"], w["time_mlp.2.bias"])
        ce = self.cond_emb(y_cat, y_cont)
        t_map = F.linear(te, w["to_time_map.weight"], w["to_time_map.bias"])
        c_map = F.linear(ce, w["to_cond_map.weight"], w["to_cond_map.bias"])
        return np.concatenate([t_map, c_map], axis=1)

    # --- blocks
    def conv(self, name, x, stride=1, padding=1):
        return F.conv2d(x, self.w[name + ".weight"], self.w[name + ".bias"], stride=stride,
                        padding=padding, mode="circular")

    def gn(self, name, x):
        C = x.shape[1]
        return F.group_norm(x, gn_groups(C), self.w[name + ".weight"], self.w[name + ".bias"])

    def conv_block(self, name, x):
        h = F.silu(self.gn(name + ".net.1", self.conv(name + ".net.0", x)))
        return F.silu(self.gn(name + ".net.4", self.conv(name + ".net.3", h)))

    def attn(self, x, heads: int = 4):
        B, C, H, W = x.shape
        N = H * W
        d = C // heads
        h = self.gn("attn.norm", x)
        qkv = F.conv2d(h, self.w["attn.qkv.weight"], self.w["attn.qkv.bias"])
        q, k, v = np.split(qkv, 3, axis=1)
        q = q.reshape(B, heads, d, N).transpose(0, 1, 3, 2)
        k = k.reshape(B, heads, d, N).transpose(0, 1, 3, 2)
        v = v.reshape(B, heads, d, N).transpose(0, 1, 3, 2)
        y = F.sdpa(q, k, v)
        y = y.transpose(0, 1, 3, 2).reshape(B, C, H, W)
        y = F.conv2d(y, self.w["attn.proj.weight"], self.w["attn.proj.bias"])
        return x + y

    def forward(self, x_t, t, y_cat, y_cont):
        B, _, H, W = x_t.shape
        m = self.maps(np.asarray(t), np.asarray(y_cat), np.asarray(y_cont))
        maps = np.broadcast_to(m[:, :, None, None], (B, m.shape[1], H, W))
        x = np.concatenate([x_t.astype(self.dt), maps], axis=1)
        h1 = self.conv_block("down1", x)
        h = self.conv("ds1", h1, stride=2, padding=1)
        h2 = self.conv_block("down2", h)
        h = self.conv("ds2", h2, stride=2, padding=1)
        h = self.conv_block("mid", h)
        h = self.attn(h)
        h = self.conv("us2_conv", F.upsample_bilinear2x(h))
        h = self.conv_block("up2", np.concatenate([h, h2], axis=1))
        h = self.conv("us1_conv", F.upsample_bilinear2x(h))
        h = self.conv_block("up1", np.concatenate([h, h1], axis=1))
        return self.conv("out", h)

    __call__ = forward


class VPSDE:
    """VPSDE(beta_min, beta_max) — sde_score_model.py:273-298 (fp32 scalar arithmetic)."""

    def __init__(self, beta_min=0.1, beta_max=20.0, dt=np.float32):
        self.beta_min, self.beta_max, self.dt = beta_min, beta_max, dt

    def beta(self, t):
        return self.dt(self.beta_min) + t * self.dt(self.beta_max - self.beta_min)

    def int_beta(self, t):
        return self.dt(self.beta_min) * t + self.dt(0.5 * (self.beta_max - self.beta_min)) * (t ** 2)

    def alpha(self, t):
        return np.exp(self.dt(-0.5) * self.int_beta(t))

    def sigma(self, t):
        a = self.alpha(t)
        return np.sqrt(np.maximum(self.dt(1.0) - a * a, self.dt(1e-8)))


def time_grid(n_steps: int, t_end: float, dt=np.float32):
    """ts = t_end + (1 - t_end) (1 - linspace(0,1,N+1))^2  (sde_score_model.py:486-487,540-541).
    torch.linspace(0,1,N+1) in fp32 computes step*i for i < N/2 and 1 - step*(N-i) above."""
    n = n_steps + 1
    step = dt(1.0) / dt(n - 1) if n > 1 else dt(0)
    i = np.arange(n)
    u = np.where(i < n // 2, dt(0.0) + step * i.astype(dt), dt(1.0) - step * (n - 1 - i).astype(dt)).astype(dt)
    return (dt(t_end) + dt(1.0 - t_end) * (dt(1.0) - u) ** 2).astype(dt)


def predict_eps_cfg(model: ScoreUNet, x_t, t, y_cat, y_cont, guidance_scale: float):
    if guidance_scale <= 0.0:
        return model(x_t, t, y_cat, y_cont)
    y_cat_u = np.full_like(y_cat, model.n_types)
    y_cont_u = np.zeros_like(y_cont)
    eps_u = model(x_t, t, y_cat_u, y_cont_u)
    eps_c = model(x_t, t, y_cat, y_cont)
    return eps_u + model.dt(guidance_scale) * (eps_c - eps_u)


def _probflow_drift(model, sde, x, t, y_cat, y_cont, guidance_scale):
    B = x.shape[0]
    beta_t = sde.beta(t).reshape(B, 1, 1, 1)
    sigma_t = sde.sigma(t).reshape(B, 1, 1, 1)
    eps_hat = predict_eps_cfg(model, x, t, y_cat, y_cont, guidance_scale)
    score = -eps_hat / sigma_t
    return model.dt(-0.5) * beta_t * x - model.dt(0.5) * beta_t * score


def final_projection(model, sde, x, t_final, y_cat, y_cont, guidance_scale, clamp=True):
    B = x.shape[0]
    a = sde.alpha(t_final).reshape(B, 1, 1, 1)
    s = sde.sigma(t_final).reshape(B, 1, 1, 1)
    eps_hat = predict_eps_cfg(model, x, t_final, y_cat, y_cont, guidance_scale)
    x0_hat = (x - s * eps_hat) / np.maximum(a, model.dt(1e-6))
    if not clamp:
        return x0_hat
    return np.clip((x0_hat + model.dt(1.0)) * model.dt(0.5), 0.0, 1.0)


def sample_reverse_sde_euler_maruyama(model, sde, y_cat, y_cont, noise, n_steps, guidance_scale, t_end,
                                      clamp=True):
    """noise: [n_steps+1, B, 1, H, W]; noise[0] is x_T, noise[i+1] the z of step i."""
    dt_ = model.dt
    B = noise.shape[1]
    x = noise[0].astype(dt_)
    ts = time_grid(n_steps, t_end, dt_)
    for i in range(n_steps):
        t = np.full(B, ts[i], dtype=dt_)
        t_next = np.full(B, ts[i + 1], dtype=dt_)
        dtt = (t_next - t).reshape(B, 1, 1, 1)
        beta_t = sde.beta(t).reshape(B, 1, 1, 1)
        sigma_t = sde.sigma(t).reshape(B, 1, 1, 1)
        g = np.sqrt(beta_t)
        eps_hat = predict_eps_cfg(model, x, t, y_cat, y_cont, guidance_scale)
        score = -eps_hat / sigma_t
        drift = (dt_(-0.5) * beta_t * x) - (beta_t * score)
        x = x + drift * dtt + g * np.sqrt(np.abs(dtt)) * noise[i + 1].astype(dt_)
    t_final = np.full(B, ts[-1], dtype=dt_)
    return final_projection(model, sde, x, t_final, y_cat, y_cont, guidance_scale, clamp)


def sample_probability_flow_ode(model, sde, y_cat, y_cont, x_init, n_steps, guidance_scale, t_end,
                                clamp=True):
    dt_ = model.dt
    B = x_init.shape[0]
    x = x_init.astype(dt_)
    ts = time_grid(n_steps, t_end, dt_)
    for i in range(n_steps):
        t = np.full(B, ts[i], dtype=dt_)
        t_next = np.full(B, ts[i + 1], dtype=dt_)
        dtt = (t_next - t).reshape(B, 1, 1, 1)
        drift = _probflow_drift(model, sde, x, t, y_cat, y_cont, guidance_scale)
        x_e = x + drift * dtt
        drift_n = _probflow_drift(model, sde, x_e, t_next, y_cat, y_cont, guidance_scale)
        x = x + dt_(0.5) * (drift + drift_n) * dtt
    t_final = np.full(B, ts[-1], dtype=dt_)
    return final_projection(model, sde, x, t_final, y_cat, y_cont, guidance_scale, clamp)


def diffusion_loss_eps(model, sde, x0, y_cat, y_cont, u, eps, drop_u, p_uncond=0.1, t_power=1.0):
    """Forward value of the ε-MSE loss with the three RNG draws injected (u, eps, drop_u)."""
    dt_ = model.dt
    B = x0.shape[0]
    x0 = x0.astype(dt_) * dt_(2.0) - dt_(1.0)
    t = u.astype(dt_) ** dt_(t_power)
    a = sde.alpha(t).reshape(B, 1, 1, 1)
    s = sde.sigma(t).reshape(B, 1, 1, 1)
    x_t = a * x0 + s * eps.astype(dt_)
    y_cat = y_cat.copy()
    y_cont = y_cont.copy()
    if p_uncond > 0.0:
        drop = drop_u < p_uncond
        y_cat[drop] = model.n_types
        y_cont[drop] = 0.0
    eps_hat = model(x_t, t, y_cat, y_cont)
    return np.mean((eps_hat - eps) ** 2)
