#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ by importing the REFERENCE.

Run ONLY in the build container (the reference is not present on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 PYTHONPATH=/root/reference/src:/root/reference \
        python tests/golden/make_goldens.py

Every fixture is data only (inputs and the reference's outputs, as .npz with no
pickles).  Weights of the random-init models are NOT stored: they are rebuilt by
`torch.manual_seed(seed)` + module construction in the reference's parameter order
(verified bit-identical by the CPU tests through the stored per-parameter checksums).
Exceptions: the base_ch=16 U-Net fixture stores its full state (its GroupNorm affine
parameters are perturbed away from the 1/0 default init so the affine path is pinned),
and one short-trained base_ch=32 score model is stored (trajectory-level parity needs
a real score; random weights make the 300-step SDE diverge).

Reference call sites reproduced (file:line in /root/reference):
  CondUNetTiny.forward                 src/toycrystals/models/sde_score_model.py:243-266
  predict_eps_cfg                      sde_score_model.py:402-423
  sample_reverse_sde_euler_maruyama    sde_score_model.py:507-569
  sample_probability_flow_ode          sde_score_model.py:452-504
  diffusion_loss_eps                   sde_score_model.py:358-399
  CondVAE / VAE                        src/toycrystals/models/vae.py:8-134
  kl_stats + VAE loss                  scripts/train_vae.py:17-36,309-312
  DiffusionPriorFiLM / ddim_sample     src/toycrystals/models/diffusion_prior.py:57-252
  score / VAE / prior training steps   scripts/train_sde_score_model.py:217-240,
                                       scripts/train_vae.py:299-312, scripts/train_diffusion_prior.py:251-277
"""
from __future__ import annotations

import math
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))

from toycrystals.models import sde_score_model as ref_sde  # noqa: E402  (reference)
from toycrystals.models import vae as ref_vae  # noqa: E402
from toycrystals.models import diffusion_prior as ref_prior  # noqa: E402
from toycrystals.data import ToyCrystalsDataset  # noqa: E402


def sd_checksums(module: torch.nn.Module) -> dict:
    out = {}
    for k, v in module.state_dict().items():
        vv = v.detach().double()
        out["ck/" + k] = np.array([vv.sum().item(), vv.abs().sum().item(), float(vv.numel())])
    return out


def sd_arrays(module: torch.nn.Module, prefix: str = "w/") -> dict:
    return {prefix + k: v.detach().cpu().numpy() for k, v in module.state_dict().items()}


def save(name: str, **arrays) -> None:
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **{k: np.asarray(v) for k, v in arrays.items()})
    print(f"  wrote {name}.npz ({os.path.getsize(path) / 1e3:.1f} kB)")


def cond_inputs(B: int, n_types: int = 4, null_last: bool = True, seed: int = 7):
    g = torch.Generator().manual_seed(seed)
    y_cat = torch.tensor([i % n_types for i in range(B)], dtype=torch.int64)
    if null_last:
        y_cat[-1] = n_types  # CFG null token
    y_cont = torch.zeros(B, 4)
    y_cont[:, 1] = torch.rand(B, generator=g) * (math.pi / 3)
    y_cont[:, 0] = torch.rand(B, generator=g)  # exercises the non-rot-only slots too
    y_cont[:, 3] = torch.rand(B, generator=g)
    return y_cat, y_cont


def perturb_norms(model: torch.nn.Module, seed: int) -> None:
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for m in model.modules():
            if isinstance(m, (torch.nn.GroupNorm, torch.nn.LayerNorm)):
                m.weight.copy_(1.0 + 0.2 * torch.randn(m.weight.shape, generator=g))
                m.bias.copy_(0.2 * torch.randn(m.bias.shape, generator=g))


# ---------------------------------------------------------------- score U-Net
def gen_unet(base_ch: int, B: int, name: str, store_weights: bool, H: int = 64) -> None:
    torch.manual_seed(0)
    model = ref_sde.CondUNetTiny(n_types=4, y_cont_dim=4, base_ch=base_ch)
    ck = sd_checksums(model)
    if store_weights:
        perturb_norms(model, 11)
    model.eval()
    g = torch.Generator().manual_seed(3)
    x_t = torch.randn(B, 1, H, H, generator=g)
    t = torch.rand(B, generator=g) * 0.99 + 0.005
    y_cat, y_cont = cond_inputs(B)
    with torch.no_grad():
        eps = model(x_t, t, y_cat, y_cont)
        # intermediate taps for per-layer debugging
        maps = model._make_maps(t, y_cat, y_cont, H, H)
        temb = ref_sde.timestep_embedding(t, 128)
        cemb = model.cond_emb(y_cat, y_cont)
    extra = sd_arrays(model) if store_weights else {}
    save(name, x_t=x_t.numpy(), t=t.numpy(), y_cat=y_cat.numpy(), y_cont=y_cont.numpy(),
         eps=eps.numpy(), maps=maps[:, :, 0, 0].numpy(), temb=temb.numpy(), cemb=cemb.numpy(),
         base_ch=np.int64(base_ch), seed=np.int64(0), **ck, **extra)


def gen_cfg(name: str) -> None:
    torch.manual_seed(0)
    model = ref_sde.CondUNetTiny(n_types=4, y_cont_dim=4, base_ch=16).eval()
    g = torch.Generator().manual_seed(5)
    B = 3
    x_t = torch.randn(B, 1, 64, 64, generator=g)
    t = torch.full((B,), 0.37)
    y_cat, y_cont = cond_inputs(B, null_last=False)
    with torch.no_grad():
        eps = ref_sde.predict_eps_cfg(model, x_t, t, y_cat, y_cont, guidance_scale=1.5)
        eps0 = ref_sde.predict_eps_cfg(model, x_t, t, y_cat, y_cont, guidance_scale=0.0)
    save(name, x_t=x_t.numpy(), t=t.numpy(), y_cat=y_cat.numpy(), y_cont=y_cont.numpy(),
         eps=eps.numpy(), eps0=eps0.numpy(), base_ch=np.int64(16), guidance=np.float64(1.5))


def draw_noise(seed: int, shape, n: int):
    """The reference's draw order with the global CPU RNG seeded at `seed`:
    x_T = randn(shape) then one randn_like(x) per step (sde_score_model.py:537,557)."""
    torch.manual_seed(seed)
    return [torch.randn(shape) for _ in range(n)]


def gen_sampler(name: str, sampler: str, base_ch: int, B: int, steps: int, cfg: float, t_end: float,
                beta_max: float = 30.0, state_dict=None, store_noise: bool = True, H: int = 64) -> None:
    torch.manual_seed(0)
    model = ref_sde.CondUNetTiny(n_types=4, y_cont_dim=4, base_ch=base_ch)
    if state_dict is not None:
        model.load_state_dict(state_dict)
    model.eval()
    sde = ref_sde.VPSDE(beta_min=0.1, beta_max=beta_max)
    y_cat = torch.tensor([i % 4 for i in range(B)], dtype=torch.int64)
    y_cont = torch.zeros(B, 4)
    y_cont[:, 1] = torch.linspace(0.0, math.pi / 3, B)
    shape = (B, 1, H, H)
    seed = 1234
    n_draws = steps + 1 if sampler == "sde" else 1
    noise = draw_noise(seed, shape, n_draws)
    torch.manual_seed(seed)  # the reference sampler now consumes the identical stream
    fn = ref_sde.sample_reverse_sde_euler_maruyama if sampler == "sde" else ref_sde.sample_probability_flow_ode
    t0 = time.time()
    with torch.no_grad():
        out = fn(model=model, sde=sde, y_cat=y_cat, y_cont=y_cont, img_shape=shape,
                 n_steps=steps, guidance_scale=cfg, t_end=t_end)
    print(f"  {name}: reference sampler {time.time() - t0:.1f}s")
    # Also record the unclamped x0_hat (the clamp saturates most pixels for weak models).
    torch.manual_seed(seed)
    with torch.no_grad():
        x0_unclamped = _unclamped(model, sde, y_cat, y_cont, shape, steps, cfg, t_end, sampler)
    arrays = dict(y_cat=y_cat.numpy(), y_cont=y_cont.numpy(), out=out.numpy(),
                  x0_unclamped=x0_unclamped.numpy(), steps=np.int64(steps), cfg=np.float64(cfg),
                  t_end=np.float64(t_end), beta_min=np.float64(0.1), beta_max=np.float64(beta_max),
                  base_ch=np.int64(base_ch), noise_seed=np.int64(seed), B=np.int64(B))
    if store_noise:
        arrays["noise"] = torch.stack(noise).numpy()
    save(name, **arrays)


def _unclamped(model, sde, y_cat, y_cont, shape, steps, cfg, t_end, sampler):
    """Same arithmetic as the reference samplers (sde_score_model.py:452-569), returning
    x0_hat before the (x+1)/2 map and the clamp.  Calls the reference's own
    predict_eps_cfg / _probflow_drift so that only the final two lines differ."""
    B = shape[0]
    x = torch.randn(shape)
    u = torch.linspace(0.0, 1.0, steps + 1)
    ts = t_end + (1.0 - t_end) * (1.0 - u) ** 2
    for i in range(steps):
        t = ts[i].expand(B)
        t_next = ts[i + 1].expand(B)
        dt = (t_next - t).view(B, 1, 1, 1)
        if sampler == "sde":
            beta_t = sde.beta(t).view(B, 1, 1, 1)
            sigma_t = sde.sigma(t).view(B, 1, 1, 1)
            gg = torch.sqrt(beta_t)
            eps_hat = ref_sde.predict_eps_cfg(model, x, t, y_cat, y_cont, guidance_scale=cfg)
            score = -eps_hat / sigma_t
            drift = (-0.5 * beta_t * x) - (beta_t * score)
            z = torch.randn_like(x)
            x = x + drift * dt + gg * torch.sqrt(torch.abs(dt)) * z
        else:
            drift = ref_sde._probflow_drift(model, sde, x, t, y_cat, y_cont, cfg)
            x_e = x + drift * dt
            drift_n = ref_sde._probflow_drift(model, sde, x_e, t_next, y_cat, y_cont, cfg)
            x = x + 0.5 * (drift + drift_n) * dt
    t_final = ts[-1].expand(B)
    a = sde.alpha(t_final).view(B, 1, 1, 1)
    s = sde.sigma(t_final).view(B, 1, 1, 1)
    eps_hat = ref_sde.predict_eps_cfg(model, x, t_final, y_cat, y_cont, guidance_scale=cfg)
    return (x - s * eps_hat) / torch.clamp(a, min=1e-6)


def train_fixture_model(n_steps: int = 600, B: int = 32, base_ch: int = 32):
    """Short-train a base_ch=32 score model with the reference's own loss
    (sde_score_model.py:358-399) + Adam, on the reference's rot-only renderer."""
    torch.manual_seed(0)
    model = ref_sde.CondUNetTiny(n_types=4, y_cont_dim=4, base_ch=base_ch)
    sde = ref_sde.VPSDE(beta_min=0.1, beta_max=30.0)
    ds = ToyCrystalsDataset(n_samples=2048, img_size=64, seed=0, rot_only=True)
    t0 = time.time()
    xs, ycs, yvs = zip(*[ds[i] for i in range(len(ds))])
    X, YC, YV = torch.stack(xs), torch.stack(ycs), torch.stack(yvs)
    print(f"  rendered {len(ds)} images in {time.time() - t0:.1f}s")
    opt = torch.optim.Adam(model.parameters(), lr=5e-4)
    g = torch.Generator().manual_seed(99)
    t0 = time.time()
    for step in range(n_steps):
        idx = torch.randint(0, len(ds), (B,), generator=g)
        loss = ref_sde.diffusion_loss_eps(model, sde, X[idx], YC[idx], YV[idx], p_uncond=0.1)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
        if step % 100 == 0 or step == n_steps - 1:
            print(f"    step {step} loss {loss.item():.4f} ({time.time() - t0:.0f}s)")
    return model.state_dict(), X[:8], YC[:8], YV[:8]


def gen_loss(name: str) -> None:
    """diffusion_loss_eps with the global RNG seeded: draws u, eps, drop in the reference's
    order (sde_score_model.py:380-391).  Stores the drawn tensors so no RNG is needed to check."""
    torch.manual_seed(0)
    model = ref_sde.CondUNetTiny(n_types=4, y_cont_dim=4, base_ch=16)
    sde = ref_sde.VPSDE(0.1, 30.0)
    g = torch.Generator().manual_seed(21)
    B = 4
    x0 = torch.rand(B, 1, 64, 64, generator=g)
    y_cat, y_cont = cond_inputs(B, null_last=False)
    torch.manual_seed(77)
    u = torch.rand((B,))
    eps = torch.randn((B, 1, 64, 64))
    drop_u = torch.rand((B,))
    torch.manual_seed(77)
    loss = ref_sde.diffusion_loss_eps(model, sde, x0, y_cat, y_cont, p_uncond=0.5, t_power=1.0)
    loss.backward()
    grads = {"g/" + k: p.grad.numpy() for k, p in model.named_parameters()
             if k in ("out.weight", "out.bias", "down1.net.0.weight", "attn.qkv.bias", "cond_emb.cat_emb.weight")}
    save(name, x0=x0.numpy(), y_cat=y_cat.numpy(), y_cont=y_cont.numpy(), u=u.numpy(), eps=eps.numpy(),
         drop_u=drop_u.numpy(), p_uncond=np.float64(0.5), loss=np.float64(loss.item()), base_ch=np.int64(16), **grads)


def gen_vpsde(name: str) -> None:
    sde = ref_sde.VPSDE(beta_min=0.1, beta_max=30.0)
    steps, t_end = 300, 0.005
    u = torch.linspace(0.0, 1.0, steps + 1)
    ts = t_end + (1.0 - t_end) * (1.0 - u) ** 2
    save(name, ts=ts.numpy(), beta=sde.beta(ts).numpy(), alpha=sde.alpha(ts).numpy(),
         sigma=sde.sigma(ts).numpy(), int_beta=sde.int_beta(ts).numpy(), steps=np.int64(steps),
         t_end=np.float64(t_end))


# ---------------------------------------------------------------- VAE
def gen_vae(name: str, cond: bool) -> None:
    torch.manual_seed(0)
    model = ref_vae.CondVAE(z_dim=32, n_types=4, y_cont_dim=4, cond_drop=0.0) if cond else ref_vae.VAE(z_dim=32)
    ck = sd_checksums(model)
    model.eval()
    g = torch.Generator().manual_seed(4)
    B = 4
    x = torch.rand(B, 1, 64, 64, generator=g)
    y_cat = torch.tensor([0, 1, 2, 3])
    y_cont = torch.zeros(B, 4)
    y_cont[:, 1] = torch.rand(B, generator=g)
    # forward() draws eps = randn_like(std) inside reparameterise (vae.py:57-60)
    torch.manual_seed(8)
    rep_eps = torch.randn(B, 32)
    torch.manual_seed(8)
    with torch.no_grad():
        if cond:
            x_hat, mu, logvar = model(x, y_cat, y_cont)
        else:
            x_hat, mu, logvar = model(x)
    sys.path.insert(0, "/root/reference")
    from scripts.train_vae import kl_stats  # reference loss helper
    recon = torch.mean((x_hat - x) ** 2)
    kl_used, kl_raw = kl_stats(mu, logvar, free_bits=0.05)
    beta = 3e-4 * min(1.0, (0 + 1) / 5.0)
    loss = recon + beta * kl_used
    save(name, x=x.numpy(), y_cat=y_cat.numpy(), y_cont=y_cont.numpy(), rep_eps=rep_eps.numpy(),
         x_hat=x_hat.numpy(), mu=mu.numpy(), logvar=logvar.numpy(), recon=np.float64(recon.item()),
         kl_used=np.float64(kl_used.item()), kl_raw=np.float64(kl_raw.item()), loss=np.float64(loss.item()),
         beta=np.float64(beta), **ck)


# ---------------------------------------------------------------- latent prior
def gen_prior(name: str, width: int, n_blocks: int, store_weights: bool) -> None:
    torch.manual_seed(0)
    model = ref_prior.DiffusionPriorFiLM(z_dim=32, n_types=4, y_cont_dim=4, t_emb_dim=64, width=width,
                                         n_blocks=n_blocks, y_cat_emb_dim=64)
    ck = sd_checksums(model)
    if store_weights:
        perturb_norms(model, 12)
    model.eval()
    g = torch.Generator().manual_seed(6)
    B = 5
    z_t = torch.randn(B, 32, generator=g)
    t = torch.tensor([0, 1, 17, 500, 999])
    y_cat = torch.tensor([0, 1, 2, 3, 1])
    y_cont = torch.zeros(B, 4)
    y_cont[:, 1] = torch.rand(B, generator=g)
    with torch.no_grad():
        eps = model(z_t, t, y_cat, y_cont)
        te = ref_prior.timestep_embedding(t, 64)
    sched = ref_prior.DiffusionSchedule.linear(T=1000, beta_start=1e-4, beta_end=0.05, device=torch.device("cpu"))
    torch.manual_seed(31)
    z_init = torch.randn(B, 32)
    torch.manual_seed(31)
    with torch.no_grad():
        z0 = sched.ddim_sample(model, y_cat=y_cat, y_cont=y_cont, n_steps=4, eta=0.0)
    eps_q = torch.randn(B, 32, generator=g)
    zq = sched.q_sample(z_t, t, eps_q)
    extra = sd_arrays(model) if store_weights else {}
    save(name, z_t=z_t.numpy(), t=t.numpy(), y_cat=y_cat.numpy(), y_cont=y_cont.numpy(), eps=eps.numpy(),
         temb=te.numpy(), ddim_z_init=z_init.numpy(), ddim_z0=z0.numpy(), ddim_steps=np.int64(4),
         alpha_bars=sched.alpha_bars.numpy(), q_eps=eps_q.numpy(), q_out=zq.numpy(),
         width=np.int64(width), n_blocks=np.int64(n_blocks), **ck, **extra)


# ---------------------------------------------------------------- training (backward) goldens
def _grad_sample(name: str, g: torch.Tensor, k: int = 64) -> dict:
    """Checksums + k fixed-index samples of a gradient (full tensors for small ones)."""
    a = g.detach().double().reshape(-1).numpy()
    out = {"gck/" + name: np.array([a.sum(), np.abs(a).sum(), float(a.size)])}
    if a.size <= 4096:
        out["g/" + name] = g.detach().numpy()
    else:
        idx = np.random.RandomState(abs(hash(name)) % (2 ** 31)).choice(a.size, size=k, replace=False)
        idx.sort()
        out["gi/" + name] = idx.astype(np.int64)
        out["gs/" + name] = a[idx].astype(np.float32)
    return out


def gen_train_score32(name: str) -> None:
    """One diffusion_loss_eps backward at base_ch=32 (every conv eligible for the split path of the
    training convs), draws recorded; gradients as checksums + fixed-index samples."""
    torch.manual_seed(0)
    model = ref_sde.CondUNetTiny(n_types=4, y_cont_dim=4, base_ch=32)
    perturb_norms(model, 5)
    ck = sd_checksums(model)
    sde = ref_sde.VPSDE(0.1, 30.0)
    g = torch.Generator().manual_seed(29)
    B = 4
    x0 = torch.rand(B, 1, 64, 64, generator=g)
    y_cat, y_cont = cond_inputs(B, null_last=False)
    torch.manual_seed(200)
    u = torch.rand((B,))
    eps = torch.randn((B, 1, 64, 64))
    drop_u = torch.rand((B,))
    torch.manual_seed(200)
    loss = ref_sde.diffusion_loss_eps(model, sde, x0, y_cat, y_cont, p_uncond=0.5, t_power=1.0)
    loss.backward()
    gs = {}
    for k, p in model.named_parameters():
        gs.update(_grad_sample(k, p.grad))
    save(name, x0=x0.numpy(), y_cat=y_cat.numpy(), y_cont=y_cont.numpy(), u=u.numpy(), eps=eps.numpy(),
         drop=drop_u.numpy(), loss=np.float64(loss.item()), p_uncond=np.float64(0.5), base_ch=np.int64(32), **ck, **gs)


def _param_sample(prefix: str, name: str, t: torch.Tensor, idx: np.ndarray) -> dict:
    return {f"{prefix}/{name}": t.detach().double().reshape(-1).numpy()[idx].astype(np.float64)}


def gen_train_score96(name: str) -> None:
    """Config 3's width: one diffusion_loss_eps backward at base_ch=96 (the 96/192/384-
    channel dgrad / wgrad forms and the first conv of the training path), then one torch.optim.Adam step and
    the EMA update (train_sde_score_model.py:217-240), draws injected.  Stored: seeds, inputs, draws, the
    loss, per-parameter gradient checksums + 64 fixed-index samples, and 64 fixed-index samples of every
    parameter after the Adam step and of its EMA (no weights: they are rebuilt from the seed)."""
    torch.manual_seed(0)
    model = ref_sde.CondUNetTiny(n_types=4, y_cont_dim=4, base_ch=96)
    perturb_norms(model, 5)
    ck = sd_checksums(model)
    ema = ref_sde.CondUNetTiny(n_types=4, y_cont_dim=4, base_ch=96)
    ema.load_state_dict(model.state_dict())
    sde = ref_sde.VPSDE(0.1, 30.0)
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    g = torch.Generator().manual_seed(31)
    B = 3
    x0 = torch.rand(B, 1, 64, 64, generator=g)
    y_cat, y_cont = cond_inputs(B, null_last=False)
    torch.manual_seed(300)
    u = torch.rand((B,))
    eps = torch.randn((B, 1, 64, 64))
    drop_u = torch.rand((B,))
    torch.manual_seed(300)
    loss = ref_sde.diffusion_loss_eps(model, sde, x0, y_cat, y_cont, p_uncond=0.5, t_power=1.0)
    opt.zero_grad(set_to_none=True)
    loss.backward()
    gs = {}
    rs = np.random.RandomState(96)
    grads = {}
    for k, p in model.named_parameters():
        gs.update(_grad_sample(k, p.grad))
        grads[k] = p.grad.detach().clone()
    opt.step()
    with torch.no_grad():
        for pe, p in zip(ema.parameters(), model.parameters()):
            pe.data.mul_(0.9).add_(p.data, alpha=1.0 - 0.9)
    ps = {}
    for (k, p), pe in zip(model.named_parameters(), ema.parameters()):
        n = p.numel()
        idx = np.sort(rs.choice(n, size=min(n, 64), replace=False)).astype(np.int64)
        ps["pi/" + k] = idx
        ps.update(_param_sample("gp", k, grads[k], idx))  # the gradient at these indices (sign reliability)
        ps.update(_param_sample("p1", k, p, idx))
        ps.update(_param_sample("ema1", k, pe, idx))
    save(name, x0=x0.numpy(), y_cat=y_cat.numpy(), y_cont=y_cont.numpy(), u=u.numpy(), eps=eps.numpy(),
         drop=drop_u.numpy(), loss=np.float64(loss.item()), p_uncond=np.float64(0.5), base_ch=np.int64(96),
         lr=np.float64(1e-3), ema_decay=np.float64(0.9), **ck, **gs, **ps)


def gen_train_score(name: str) -> None:
    """diffusion_loss_eps backward (all parameter grads) + two torch.optim.Adam steps + EMA
    (train_sde_score_model.py:217-240) at base_ch=16, draws recorded."""
    torch.manual_seed(0)
    model = ref_sde.CondUNetTiny(n_types=4, y_cont_dim=4, base_ch=16)
    perturb_norms(model, 5)
    ck = sd_checksums(model)
    ema = ref_sde.CondUNetTiny(n_types=4, y_cont_dim=4, base_ch=16)
    ema.load_state_dict(model.state_dict())
    sde = ref_sde.VPSDE(0.1, 30.0)
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    g = torch.Generator().manual_seed(23)
    B = 3
    x0 = torch.rand(B, 1, 64, 64, generator=g)
    y_cat, y_cont = cond_inputs(B, null_last=False)
    out = {}
    for step in range(2):
        torch.manual_seed(100 + step)
        u = torch.rand((B,))
        eps = torch.randn((B, 1, 64, 64))
        drop_u = torch.rand((B,))
        torch.manual_seed(100 + step)
        loss = ref_sde.diffusion_loss_eps(model, sde, x0, y_cat, y_cont, p_uncond=0.5, t_power=1.0)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        if step == 0:
            for k, p in model.named_parameters():
                out["g/" + k] = p.grad.numpy().copy()
        opt.step()
        with torch.no_grad():
            for pe, p in zip(ema.parameters(), model.parameters()):
                pe.data.mul_(0.9).add_(p.data, alpha=1.0 - 0.9)
        out[f"u{step}"] = u.numpy()
        out[f"eps{step}"] = eps.numpy()
        out[f"drop{step}"] = drop_u.numpy()
        out[f"loss{step}"] = np.float64(loss.item())
    keep = ("down1.net.0.weight", "mid.net.1.weight", "attn.qkv.weight", "cond_emb.cat_emb.weight",
            "up1.net.3.bias", "out.weight", "time_mlp.0.weight")
    for k, p in model.named_parameters():
        if k in keep:
            out["p2/" + k] = p.detach().numpy().copy()
    for (k, _), pe in zip(model.named_parameters(), ema.parameters()):
        if k in keep:
            out["ema2/" + k] = pe.detach().numpy().copy()
    save(name, x0=x0.numpy(), y_cat=y_cat.numpy(), y_cont=y_cont.numpy(), p_uncond=np.float64(0.5), lr=np.float64(1e-3),
         ema_decay=np.float64(0.9), base_ch=np.int64(16), **ck, **out)


def gen_train_vae(name: str) -> None:
    """CondVAE training step (train_vae.py:299-312): forward in train mode with cond_drop=0.1,
    recon + beta * kl_used (free bits 0.05), backward.  Draws (reparam eps, keep mask u) recorded."""
    torch.manual_seed(0)
    model = ref_vae.CondVAE(z_dim=32, n_types=4, y_cont_dim=4, cond_drop=0.1)
    ck = sd_checksums(model)
    model.train()
    g = torch.Generator().manual_seed(41)
    B = 4
    x = torch.rand(B, 1, 64, 64, generator=g)
    y_cat = torch.tensor([0, 1, 2, 3])
    y_cont = torch.zeros(B, 4)
    y_cont[:, 1] = torch.rand(B, generator=g)
    torch.manual_seed(9)
    rep_eps = torch.randn(B, 32)
    keep_u = torch.rand((B, 1))
    torch.manual_seed(9)
    x_hat, mu, logvar = model(x, y_cat, y_cont)
    sys.path.insert(0, "/root/reference")
    from scripts.train_vae import kl_stats
    recon = torch.mean((x_hat - x) ** 2)
    kl_used, kl_raw = kl_stats(mu, logvar, free_bits=0.05)
    beta = 3e-4 * min(1.0, (0 + 1) / 5.0)
    loss = recon + beta * kl_used
    loss.backward()
    gs = {}
    for k, p in model.named_parameters():
        gs.update(_grad_sample(k, p.grad))
    save(name, x=x.numpy(), y_cat=y_cat.numpy(), y_cont=y_cont.numpy(), rep_eps=rep_eps.numpy(),
         keep_u=keep_u.numpy(), x_hat=x_hat.detach().numpy(), mu=mu.detach().numpy(),
         logvar=logvar.detach().numpy(), loss=np.float64(loss.item()), recon=np.float64(recon.item()),
         kl_used=np.float64(kl_used.item()), beta=np.float64(beta), free_bits=np.float64(0.05), **ck, **gs)


def gen_train_prior(name: str) -> None:
    """Prior training step (train_diffusion_prior.py:251-277): t = clamp(long(u^2 T)), q_sample,
    MSE, backward; width 64, 2 blocks, T = 200 (the CLI default), stored weights (perturbed norms)."""
    torch.manual_seed(0)
    model = ref_prior.DiffusionPriorFiLM(z_dim=32, n_types=4, y_cont_dim=4, t_emb_dim=64, width=64, n_blocks=2,
                                         y_cat_emb_dim=64)
    perturb_norms(model, 13)
    ck = sd_checksums(model)
    model.train()
    sched = ref_prior.DiffusionSchedule.linear(T=200, beta_start=1e-4, beta_end=1.0, device=torch.device("cpu"))
    g = torch.Generator().manual_seed(51)
    B = 6
    z0 = torch.randn(B, 32, generator=g)
    y_cat = torch.tensor([0, 1, 2, 3, 1, 0])
    y_cont = torch.zeros(B, 4)
    y_cont[:, 1] = torch.rand(B, generator=g)
    torch.manual_seed(61)
    u = torch.rand((B,))
    t = torch.clamp((u ** 2 * 200).long(), 0, 199)
    eps = torch.randn_like(z0)
    z_t = sched.q_sample(z0=z0, t=t, eps=eps)
    eps_pred = model(z_t, t, y_cat, y_cont)
    loss = torch.mean((eps_pred - eps) ** 2)
    loss.backward()
    grads = {"g/" + k: p.grad.numpy() for k, p in model.named_parameters()}
    save(name, z0=z0.numpy(), y_cat=y_cat.numpy(), y_cont=y_cont.numpy(), u=u.numpy(), t=t.numpy(), eps=eps.numpy(),
         z_t=z_t.detach().numpy(), eps_pred=eps_pred.detach().numpy(), loss=np.float64(loss.item()),
         T=np.int64(200), beta_end=np.float64(1.0), **ck, **grads)


def gen_train_prior_w1024(name: str) -> None:
    """Config 4's prior training step at its size (train_diffusion_prior.py:251-277 over
    diffusion_prior.py:39-127): DiffusionPriorFiLM width 1024, 8 blocks (103 M parameters),
    T = 1000 (beta 1e-4 .. 0.05), B = 32; t = clamp(long(u^2 T)), q_sample, MSE, backward.
    Seeded weights (not stored) with perturbed LayerNorm affines (stored: 18 x 1024 values);
    gradients as checksums + 256 fixed-index samples per tensor (full for tensors <= 4096)."""
    torch.manual_seed(0)
    model = ref_prior.DiffusionPriorFiLM(z_dim=32, n_types=4, y_cont_dim=4, t_emb_dim=64, width=1024, n_blocks=8,
                                         y_cat_emb_dim=64)
    ck = sd_checksums(model)  # of the seeded init, before the norm perturbation
    perturb_norms(model, 17)
    norms = {"w/" + k: v.detach().numpy().copy() for k, v in model.state_dict().items() if ".norm" in k or "norm" in k.split(".")[-2]}
    model.train()
    T = 1000
    sched = ref_prior.DiffusionSchedule.linear(T=T, beta_start=1e-4, beta_end=0.05, device=torch.device("cpu"))
    g = torch.Generator().manual_seed(71)
    B = 32
    z0 = torch.randn(B, 32, generator=g)
    y_cat = torch.tensor([i % 4 for i in range(B)])
    y_cont = torch.zeros(B, 4)
    y_cont[:, 1] = torch.rand(B, generator=g) * (math.pi / 3)
    torch.manual_seed(81)
    u = torch.rand((B,))
    t = torch.clamp((u ** 2 * T).long(), 0, T - 1)
    eps = torch.randn_like(z0)
    z_t = sched.q_sample(z0=z0, t=t, eps=eps)
    eps_pred = model(z_t, t, y_cat, y_cont)
    loss = torch.mean((eps_pred - eps) ** 2)
    loss.backward()
    gs = {}
    for k, p in model.named_parameters():
        a = p.grad.detach().double().reshape(-1).numpy()
        gs["gck/" + k] = np.array([a.sum(), np.abs(a).sum(), float(np.abs(a).max())])
        if a.size <= 4096:
            gs["g/" + k] = p.grad.detach().numpy().copy()
        else:
            idx = np.sort(np.random.RandomState(len(k) * 7919 + a.size % 100003).choice(a.size, size=256, replace=False))
            gs["gi/" + k] = idx.astype(np.int64)
            gs["gs/" + k] = a[idx].astype(np.float32)
    save(name, z0=z0.numpy(), y_cat=y_cat.numpy(), y_cont=y_cont.numpy(), u=u.numpy(), t=t.numpy(), eps=eps.numpy(),
         z_t=z_t.detach().numpy(), eps_pred=eps_pred.detach().numpy(), loss=np.float64(loss.item()),
         T=np.int64(T), beta_end=np.float64(0.05), norm_seed=np.int64(17), **ck, **norms, **gs)


def gen_bf16_emulated(name: str) -> None:
    """Error model for config 5's bf16 path ("bf16 MFMA conv-as-GEMM", BASELINE.json configs[4]):
    the REFERENCE's own 300-step reverse SDE (CFG 1.5, t_end 0.005) on the trained base-96 model with
    the recorded draws of sde96_trained_300, but with every conv operand rounded to bf16 (RNE) and
    fp32 accumulation — each nn.Conv2d's weight once and its input at every call (forward
    pre-hook), the bias kept fp32 — and the attention's q, k, v and softmax P rounded to bf16 (the
    operands of the two bf16 MFMA products).  Its distance from the fp32 run is the drift bf16
    operand rounding alone causes on this trajectory; the GPU test gates the bf16 path at 2x it."""
    import torch.nn.functional as Fn
    sd = {k: torch.from_numpy(v) for k, v in np.load(os.path.join(HERE, "trained96_ema.npz")).items()}
    torch.manual_seed(0)
    model = ref_sde.CondUNetTiny(n_types=4, y_cont_dim=4, base_ch=96)
    model.load_state_dict(sd)
    model.eval()
    bf = lambda t: t.to(torch.bfloat16).to(torch.float32)  # noqa: E731
    hooks = []
    with torch.no_grad():
        for m in model.modules():
            if isinstance(m, torch.nn.Conv2d):
                m.weight.copy_(bf(m.weight))
                hooks.append(m.register_forward_pre_hook(lambda mod, inp: (bf(inp[0]),) + tuple(inp[1:])))
    sdpa = Fn.scaled_dot_product_attention

    def sdpa_bf16(q, k, v, *a, **kw):
        assert not a and not kw
        s = bf(q) @ bf(k).transpose(-2, -1) / math.sqrt(q.shape[-1])
        return bf(torch.softmax(s, dim=-1)) @ bf(v)

    Fn.scaled_dot_product_attention = sdpa_bf16
    try:
        sde = ref_sde.VPSDE(beta_min=0.1, beta_max=30.0)
        B, steps, H = 8, 300, 64
        y_cat = torch.tensor([i % 4 for i in range(B)], dtype=torch.int64)
        y_cont = torch.zeros(B, 4)
        y_cont[:, 1] = torch.linspace(0.0, math.pi / 3, B)
        shape = (B, 1, H, H)
        seed = 1234
        t0 = time.time()
        torch.manual_seed(seed)
        with torch.no_grad():
            out = ref_sde.sample_reverse_sde_euler_maruyama(model=model, sde=sde, y_cat=y_cat, y_cont=y_cont,
                                                            img_shape=shape, n_steps=steps, guidance_scale=1.5,
                                                            t_end=0.005)
            torch.manual_seed(seed)
            x0 = _unclamped(model, sde, y_cat, y_cont, shape, steps, 1.5, 0.005, "sde")
        print(f"  {name}: bf16-emulated reference sampler {time.time() - t0:.1f}s")
    finally:
        Fn.scaled_dot_product_attention = sdpa
        for h in hooks:
            h.remove()
    ref = np.load(os.path.join(HERE, "sde96_trained_300.npz"))
    assert int(ref["noise_seed"]) == seed and int(ref["B"]) == B
    d = np.abs(out.numpy() - ref["out"])
    print(f"  emulated bf16 vs fp32 reference: image max {d.max():.3e} mean {d.mean():.3e} "
          f"p99 {np.quantile(d, 0.99):.3e} off>1e-2 {100 * (d > 1e-2).mean():.2f} %")
    save(name, out=out.numpy(), x0_unclamped=x0.numpy(), noise_seed=np.int64(seed), B=np.int64(B),
         steps=np.int64(steps))


def main() -> int:
    torch.set_num_threads(8)
    which = set(sys.argv[1:])

    def want(k):
        return not which or k in which

    if want("unet"):
        gen_unet(16, 3, "unet16_b3", store_weights=True)
        gen_unet(96, 2, "unet96_b2", store_weights=False)
        gen_unet(32, 2, "unet32_b2_h32", store_weights=False, H=32)
    if want("unet256"):
        # config 5's resolution: 64x64 = 4096 tokens at the attention level (key-tiled kernel)
        gen_unet(96, 2, "unet96_b2_h256", store_weights=False, H=256)
        # the metric's sampler at 256^2 (config 5): 2 reverse-SDE steps + projection, noise by seed
        gen_sampler("sde96_2step_h256", "sde", 96, 2, 2, 1.5, 0.005, store_noise=False, H=256)
    if want("cfg"):
        gen_cfg("cfg16_b3")
    if want("vpsde"):
        gen_vpsde("vpsde_grid300")
    if want("samplers"):
        gen_sampler("sde16_3step", "sde", 16, 3, 3, 1.5, 0.005)
        gen_sampler("ode16_2step", "ode", 16, 3, 2, 1.5, 0.005)
        gen_sampler("sde96_2step_b2", "sde", 96, 2, 2, 1.5, 0.005)
    if want("trained"):
        sd, X, YC, YV = train_fixture_model()
        np.savez_compressed(os.path.join(HERE, "trained32_state.npz"),
                            **{k: v.numpy() for k, v in sd.items()})
        print("  wrote trained32_state.npz")
        # (its 300-step reverse SDE saturated every pixel; replaced by sde96_trained_300 below)
        gen_sampler("ode32_trained_20", "ode", 32, 4, 20, 1.5, 0.005, state_dict=sd, store_noise=False)
    if want("trained96"):
        # the EMA weights of a 40-epoch run of the README recipe (README.md:104) through this repo's
        # mirror train_sde_score_model.py on the MI355X (tools/gpu/recipe40.sh; loss curve in
        # profiles/r02_a_recipe40_metrics.jsonl), loaded into the REFERENCE model here
        sd = {k: torch.from_numpy(v) for k, v in np.load(os.path.join(HERE, "trained96_ema.npz")).items()}
        gen_sampler("sde96_trained_300", "sde", 96, 8, 300, 1.5, 0.005, state_dict=sd, store_noise=False)
        gen_sampler("ode96_trained_50", "ode", 96, 4, 50, 1.5, 0.005, state_dict=sd, store_noise=False)
    if want("loss"):
        gen_loss("loss16_b4")
    if want("vae"):
        gen_vae("condvae_b4", cond=True)
        gen_vae("vae_b4", cond=False)
    if want("prior"):
        gen_prior("prior_w64_b2", 64, 2, store_weights=True)
        gen_prior("prior_w1024_b8", 1024, 8, store_weights=False)
    if want("train32"):
        gen_train_score32("train32_b4")
    if want("train96"):
        gen_train_score96("train96_b3")
    if want("train"):
        gen_train_score("train16_b3")
        gen_train_vae("train_condvae_b4")
        gen_train_prior("train_prior_w64")
    if want("bf16emu"):
        gen_bf16_emulated("sde96_trained_300_bf16emu")
    if want("train_prior_w1024"):
        gen_train_prior_w1024("train_prior_w1024_b32")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
