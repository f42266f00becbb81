"""Oracle restatement of the VAE and the latent-prior path (test-only; see oracle/__init__.py).

Follows /root/reference:
  CondVAE encode/decode/forward   src/toycrystals/models/vae.py:8-78
  VAE (unconditional)             vae.py:81-134
  kl_stats + loss                 scripts/train_vae.py:17-36, 309-312
  prior timestep_embedding        src/toycrystals/models/diffusion_prior.py:11-25
  FiLMResBlock                    diffusion_prior.py:39-54
  DiffusionPriorFiLM.forward      diffusion_prior.py:112-127
  DiffusionSchedule               diffusion_prior.py:167-252 (linear, q_sample, ddim eta=0)
"""
from __future__ import annotations

import math

import numpy as np

from . import nn_np as F


def _f(sd, dt):
    return {k: (np.asarray(v).astype(dt) if np.asarray(v).dtype.kind == "f" else np.asarray(v))
            for k, v in sd.items()}


class VAE:
    """Both CondVAE (cond=True) and VAE (cond=False)."""

    def __init__(self, sd, cond=True, n_types=4, dt=np.float32):
        self.w = _f(sd, dt)
        self.cond, self.n_types, self.dt = cond, n_types, dt

    def y_vec(self, y_cat, y_cont):
        oh = np.eye(self.n_types, dtype=self.dt)[y_cat]
        return np.concatenate([oh, y_cont.astype(self.dt)], axis=1)

    def encode(self, x, y_cat=None, y_cont=None):
        w = self.w
        h = x.astype(self.dt)
        for i in (0, 2, 4, 6):
            h = F.relu(F.conv2d(h, w[f"enc.{i}.weight"], w[f"enc.{i}.bias"], stride=2, padding=1))
        h = h.reshape(h.shape[0], -1)
        if self.cond:
            h = np.concatenate([h, self.y_vec(y_cat, y_cont)], axis=1)
        h = F.relu(F.linear(h, w["enc_fc.weight"], w["enc_fc.bias"]))
        return F.linear(h, w["mu.weight"], w["mu.bias"]), F.linear(h, w["logvar.weight"], w["logvar.bias"])

    def decode(self, z, y_cat=None, y_cont=None):
        w = self.w
        if self.cond:
            z = np.concatenate([z, self.y_vec(y_cat, y_cont)], axis=1)
        h = F.linear(z.astype(self.dt), w["dec_fc.weight"], w["dec_fc.bias"]).reshape(-1, 256, 4, 4)
        for i in (0, 2, 4):
            h = F.relu(F.conv_transpose2d(h, w[f"dec.{i}.weight"], w[f"dec.{i}.bias"]))
        return F.sigmoid(F.conv_transpose2d(h, w["dec.6.weight"], w["dec.6.bias"]))

    def forward(self, x, y_cat, y_cont, rep_eps):
        mu, logvar = self.encode(x, y_cat, y_cont)
        z = mu + np.exp(self.dt(0.5) * logvar) * rep_eps.astype(self.dt)
        return self.decode(z, y_cat, y_cont), mu, logvar


def kl_stats(mu, logvar, free_bits=0.0):
    kl_dim = 0.5 * (mu ** 2 + np.exp(logvar) - 1.0 - logvar)
    kl_raw = kl_dim.sum(axis=1).mean()
    kl_used = np.maximum(kl_dim, free_bits).sum(axis=1).mean() if free_bits > 0 else kl_raw
    return kl_used, kl_raw


def vae_loss(x_hat, x, mu, logvar, beta, epoch, free_bits):
    recon = np.mean((x_hat - x) ** 2)
    kl_used, kl_raw = kl_stats(mu, logvar, free_bits)
    b = beta * min(1.0, (epoch + 1) / 5.0)
    return recon + b * kl_used, recon, kl_used, kl_raw


def prior_timestep_embedding(t, dim, dt=np.float32):
    """Integer-t sinusoid WITHOUT 2*pi, [sin, cos] order (diffusion_prior.py:11-25)."""
    half = dim // 2
    # torch.linspace(0, ln 1e4, half) in fp32 (symmetric two-sided evaluation)
    end = dt(math.log(10_000))
    step = end / dt(half - 1)
    i = np.arange(half)
    lin = np.where(i < half // 2, step * i.astype(dt), end - step * (half - 1 - i).astype(dt)).astype(dt)
    freqs = np.exp(lin * dt(-1.0))
    args = t.astype(dt)[:, None] * freqs[None, :]
    emb = np.concatenate([np.sin(args), np.cos(args)], axis=1)
    if dim % 2 == 1:
        emb = np.pad(emb, ((0, 0), (0, 1)))
    return emb


class PriorFiLM:
    def __init__(self, sd, dt=np.float32):
        self.w = _f(sd, dt)
        self.dt = dt
        self.t_emb_dim = self.w["t_mlp.0.weight"].shape[1]
        self.n_blocks = len({k.split(".")[1] for k in sd if k.startswith("blocks.")})
        self.z_dim = self.w["in_proj.weight"].shape[1]

    def mlp(self, prefix, x):
        w = self.w
        return F.linear(F.silu(F.linear(x, w[prefix + ".0.weight"], w[prefix + ".0.bias"])),
                        w[prefix + ".2.weight"], w[prefix + ".2.bias"])

    def forward(self, z_t, t, y_cat, y_cont):
        w = self.w
        te = prior_timestep_embedding(np.asarray(t), self.t_emb_dim, self.dt)
        t_feat = self.mlp("t_mlp", te)
        y_feat = self.mlp("y_fuse", np.concatenate(
            [w["y_cat_emb.weight"][y_cat], self.mlp("y_cont_mlp", y_cont.astype(self.dt))], axis=-1))
        cond = np.concatenate([t_feat, y_feat], axis=-1)
        h = F.linear(z_t.astype(self.dt), w["in_proj.weight"], w["in_proj.bias"])
        for i in range(self.n_blocks):
            p = f"blocks.{i}."
            hn = F.layer_norm(h, w[p + "norm.weight"], w[p + "norm.bias"])
            gb = F.linear(cond, w[p + "cond.weight"], w[p + "cond.bias"])
            gamma, beta = np.split(gb, 2, axis=-1)
            hn = hn * (self.dt(1.0) + gamma) + beta
            hn = F.linear(F.silu(F.linear(hn, w[p + "fc1.weight"], w[p + "fc1.bias"])),
                          w[p + "fc2.weight"], w[p + "fc2.bias"])
            h = h + hn
        h = F.layer_norm(h, w["out_norm.weight"], w["out_norm.bias"])
        return F.linear(h, w["out_proj.weight"], w["out_proj.bias"])

    __call__ = forward


class Schedule:
    """DiffusionSchedule.linear(T, beta_start, beta_end) (diffusion_prior.py:178-190)."""

    def __init__(self, T, beta_start, beta_end, dt=np.float32):
        n = T
        step = dt((beta_end - beta_start) / (n - 1))
        i = np.arange(n)
        self.betas = np.where(i < n // 2, dt(beta_start) + step * i.astype(dt),
                              dt(beta_end) - step * (n - 1 - i).astype(dt)).astype(dt)
        self.alphas = (dt(1.0) - self.betas).astype(dt)
        self.alpha_bars = np.cumprod(self.alphas, dtype=dt)
        self.sqrt_alpha_bars = np.sqrt(self.alpha_bars)
        self.sqrt_one_minus_alpha_bars = np.sqrt(dt(1.0) - self.alpha_bars)
        self.dt = dt

    def q_sample(self, z0, t, eps):
        return self.sqrt_alpha_bars[t][:, None] * z0 + self.sqrt_one_minus_alpha_bars[t][:, None] * eps

    def ddim_timesteps(self, n_steps):
        T = len(self.betas)
        ts = np.round(np.linspace(T - 1, 0, n_steps, dtype=np.float32)).astype(np.int64)
        keep = np.concatenate([[True], ts[1:] != ts[:-1]])
        return ts[keep]

    def ddim_sample(self, model, y_cat, y_cont, z_init, n_steps=50):
        dt = self.dt
        z = z_init.astype(dt)
        B = z.shape[0]
        ts = self.ddim_timesteps(n_steps)
        for i in range(len(ts)):
            t = np.full(B, ts[i])
            eps = model(z, t, y_cat, y_cont)
            ab = self.alpha_bars[t][:, None]
            z0 = (z - np.sqrt(dt(1.0) - ab) * eps) / (np.sqrt(ab) + dt(1e-8))
            if i == len(ts) - 1:
                return z0
            abp = self.alpha_bars[np.full(B, ts[i + 1])][:, None]
            z = np.sqrt(abp) * z0 + np.sqrt(dt(1.0) - abp) * eps
        return z
