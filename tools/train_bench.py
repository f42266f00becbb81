#!/usr/bin/env python3
"""Training-step throughput of the three models on one MI355X:

  score  : diffusion_loss_eps + backward + fused Adam (+ EMA 0.999), CondUNetTiny(base_ch=96),
           B=128, synthetic 64x64 batch; algorithmic work 21.43 GFLOP / image / step
  vae    : CondVAE(z=32, cond_drop 0.1) recon + beta*KL(free bits) + backward + Adam, B=128
  prior  : DiffusionPriorFiLM(width=1024, 8 blocks) q_sample + MSE + backward + Adam, B=256

Prints one JSON line per model: steps/s, images (samples)/s, ms/step and, for the score model,
achieved TFLOP/s against the 157.3 TF fp32 peak.  usage: python tools/train_bench.py [score vae prior]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vae-diffusion-toy-crystals_amd"))

import torch  # noqa: E402

from toycrystals_amd import functional as TF  # noqa: E402
from toycrystals_amd.optim import Adam, ema_update  # noqa: E402

STEPS = int(os.environ.get("STEPS", "10"))
WARM = int(os.environ.get("WARM", "3"))


def timed(step_fn):
    for _ in range(WARM):
        step_fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(STEPS):
        step_fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / STEPS


def bench_score():
    from toycrystals_amd.models.sde_score_model import CondUNetTiny, VPSDE, diffusion_loss_eps
    torch.manual_seed(0)
    B = int(os.environ.get("B", "128"))
    model = CondUNetTiny(4, 4, 96).cuda().train()
    ema = CondUNetTiny(4, 4, 96).cuda()
    ema.load_state_dict(model.state_dict())
    sde = VPSDE(0.1, 30.0)
    opt = Adam(model.parameters(), lr=1e-4)
    x0 = torch.rand(B, 1, 64, 64, device="cuda")
    y_cat = (torch.arange(B, device="cuda") % 4).to(torch.int64)
    y_cont = torch.zeros(B, 4, device="cuda")
    y_cont[:, 1] = torch.linspace(0, 1.047, B, device="cuda")

    def step():
        loss = diffusion_loss_eps(model, sde, x0, y_cat, y_cont, p_uncond=0.1)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
        ema_update(ema, model, 0.999)

    dt = timed(step)
    tf = 21.4276e9 * B / dt / 1e12
    return {"model": "score CondUNetTiny(base_ch=96)", "batch": B, "ms_per_step": round(dt * 1e3, 3),
            "images_per_s": round(B / dt, 2), "tflops": round(tf, 2), "frac_fp32_peak": round(tf / 157.3, 4)}


def bench_vae():
    from toycrystals_amd.models.vae import CondVAE
    torch.manual_seed(0)
    B = int(os.environ.get("B_VAE", "128"))
    m = CondVAE(z_dim=32, n_types=4, y_cont_dim=4, cond_drop=0.1).cuda().train()
    opt = Adam(m.parameters(), lr=2e-3)
    x = torch.rand(B, 1, 64, 64, device="cuda")
    y_cat = (torch.arange(B, device="cuda") % 4).to(torch.int64)
    y_cont = torch.rand(B, 4, device="cuda")

    def step():
        x_hat, mu, lv = m(x, y_cat, y_cont)
        kl_used, _ = TF.kl_stats(mu, lv, 0.05)
        loss = TF.mse_loss(x_hat, x) + 3e-4 * kl_used
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()

    dt = timed(step)
    return {"model": "CondVAE(z=32)", "batch": B, "ms_per_step": round(dt * 1e3, 3), "images_per_s": round(B / dt, 1)}


def bench_prior():
    from toycrystals_amd._lib import check, lib, ptr, stream_ptr
    from toycrystals_amd.models.diffusion_prior import DiffusionPriorFiLM, DiffusionSchedule
    torch.manual_seed(0)
    B, T = int(os.environ.get("B_PRIOR", "256")), 1000
    m = DiffusionPriorFiLM(32, 4, 4, t_emb_dim=64, width=1024, n_blocks=8, y_cat_emb_dim=64).cuda().train()
    opt = Adam(m.parameters(), lr=1e-4)
    sched = DiffusionSchedule.linear(T, 1e-4, 0.05, torch.device("cuda"))
    z0 = torch.randn(B, 32, device="cuda")
    y_cat = (torch.arange(B, device="cuda") % 4).to(torch.int64)
    y_cont = torch.rand(B, 4, device="cuda")
    t = torch.empty(B, device="cuda", dtype=torch.int64)
    z_t = torch.empty_like(z0)

    def step():
        u = torch.rand(B, device="cuda")
        eps = torch.randn_like(z0)
        check(lib().tcx_prior_qsample(ptr(z0), ptr(eps), ptr(u), ptr(sched.sqrt_alpha_bars),
                                      ptr(sched.sqrt_one_minus_alpha_bars), T, B, 32, ptr(t), ptr(z_t),
                                      stream_ptr()), "qsample")
        loss = TF.mse_loss(m(z_t, t, y_cat, y_cont), eps)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()

    dt = timed(step)
    return {"model": "DiffusionPriorFiLM(w=1024, 8 blocks)", "batch": B, "ms_per_step": round(dt * 1e3, 3),
            "samples_per_s": round(B / dt, 1), "tflops": round(0.6180e9 * B / dt / 1e12, 2)}


def bench_ddim():
    """DDIM-50 sampling of the w1024 x 8 prior for the 36-sample grid (config 4's sampler, HBM-bound:
    the 412 MB of weights are read once per step)."""
    from toycrystals_amd.models.diffusion_prior import DiffusionPriorFiLM, DiffusionSchedule
    torch.manual_seed(0)
    n = 36
    m = DiffusionPriorFiLM(32, 4, 4, t_emb_dim=64, width=1024, n_blocks=8, y_cat_emb_dim=64).cuda().eval()
    sched = DiffusionSchedule.linear(1000, 1e-4, 0.05, torch.device("cuda"))
    y_cat = (torch.arange(n, device="cuda") % 4).to(torch.int64)
    y_cont = torch.rand(n, 4, device="cuda")
    # bytes streamed per DDIM step: the trunk's fc1 + fc2 weights (8 blocks x 2 x 1024 x 4096 x 4 B = 268 MB);
    # the FiLM projections and the t / y branches are hoisted out of the step loop, so the
    # remaining ~144 MB of the 412 MB of parameters is read once per call, not per step
    wbytes = sum(b.fc1.weight.numel() + b.fc2.weight.numel() for b in m.blocks) * 4

    def step():
        with torch.no_grad():
            sched.ddim_sample(m, y_cat, y_cont, n_steps=50)

    dt = timed(step)
    return {"model": "DiffusionPriorFiLM(w=1024, 8 blocks) DDIM-50", "batch": n, "ms_per_sample_call": round(dt * 1e3, 3),
            "ms_per_ddim_step": round(dt * 1e3 / 50, 4), "trunk_weight_stream_TBps": round(wbytes * 50 / dt / 1e12, 3),
            "trunk_bytes_per_step": wbytes}


if __name__ == "__main__":
    which = sys.argv[1:] or ["score", "vae", "prior"]
    fns = {"score": bench_score, "vae": bench_vae, "prior": bench_prior, "ddim": bench_ddim}
    for w in which:
        print(json.dumps(fns[w]()), flush=True)
