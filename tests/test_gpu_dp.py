"""GPU: batch-DP equivalence of the training steps on the real HIP path.

A data-parallel step computes the loss on each rank's equal shard of the global batch and averages
the gradients (BucketedGradAllReduce).  Because every loss of the path is a mean over the batch
(diffusion_loss_eps, the VAE's recon + beta * kl_used, the prior's MSE), the mean of the shard
gradients must equal the full-batch gradient.  These tests run, in one process, the libtcx training
step on the full batch and on its two halves with the SAME injected draws (the global draws of the
reference's order, sliced per shard: what the mirrors' --global-draws mode feeds each rank) and
compare every parameter gradient.  Tolerance: 1e-5 x the tensor's max |g| (fp32 reduction order:
full-batch and per-shard pixel sums are split differently; observed values are printed).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _grads(model):
    return {k: p.grad.detach().double().cpu().clone() for k, p in model.named_parameters() if p.grad is not None}


def _compare(full, shards, what):
    worst = 0.0
    for k, g in full.items():
        mean = sum(s[k] for s in shards) / len(shards)
        e = float((mean - g).abs().max()) / max(float(g.abs().max()), 1e-12)
        worst = max(worst, e)
        assert e < 1e-5, (what, k, e)
    print(f"{what}: max over parameters of |mean(shard grads) - full grad| / max|g| = {worst:.2e}")


@pytest.mark.parametrize("base", [32, 96])
def test_score_step_shards_equal_full_batch(base):
    from toycrystals_amd.models.sde_score_model import CondUNetTiny, VPSDE, diffusion_loss_eps
    torch.manual_seed(0)
    m = CondUNetTiny(4, 4, base).cuda().train()
    sde = VPSDE(0.1, 30.0)
    B = 8
    g = torch.Generator().manual_seed(3)
    x0 = torch.rand(B, 1, 64, 64, generator=g).cuda()
    y_cat = (torch.arange(B) % 4).cuda()
    y_cont = torch.rand(B, 4, generator=g).cuda()
    # the global draws in the reference's order (sde_score_model.py:380-391)
    u = torch.rand(B, generator=g).cuda()
    eps = torch.randn(B, 1, 64, 64, generator=g).cuda()
    drop = torch.rand(B, generator=g).cuda()

    def step(sl):
        m.zero_grad(set_to_none=True)
        loss = diffusion_loss_eps(m, sde, x0[sl], y_cat[sl], y_cont[sl], p_uncond=0.3,
                                  draws=(u[sl], eps[sl], drop[sl]))
        loss.backward()
        return float(loss.detach()), _grads(m)

    lf, full = step(slice(0, B))
    l0, s0 = step(slice(0, B // 2))
    l1, s1 = step(slice(B // 2, B))
    assert abs((l0 + l1) / 2 - lf) <= 1e-6 * lf
    _compare(full, [s0, s1], f"CondUNetTiny({base}) diffusion_loss_eps")


def test_condvae_step_shards_equal_full_batch():
    from toycrystals_amd import functional as TF
    from toycrystals_amd.models.vae import CondVAE
    torch.manual_seed(0)
    m = CondVAE(z_dim=32, n_types=4, y_cont_dim=4, cond_drop=0.1).cuda().train()
    B = 16
    g = torch.Generator().manual_seed(5)
    x = torch.rand(B, 1, 64, 64, generator=g).cuda()
    y_cat = (torch.arange(B) % 4).cuda()
    y_cont = torch.rand(B, 4, generator=g).cuda()
    rep_eps = torch.randn(B, 32, generator=g).cuda()
    keep_u = torch.rand(B, 1, generator=g).cuda()

    def step(sl):
        m.zero_grad(set_to_none=True)
        x_hat, mu, logvar = m(x[sl], y_cat[sl], y_cont[sl], draws=(rep_eps[sl], keep_u[sl]))
        kl_used, _ = TF.kl_stats(mu, logvar, free_bits=0.05)
        loss = TF.mse_loss(x_hat, x[sl]) + 6e-5 * kl_used
        loss.backward()
        return _grads(m)

    full = step(slice(0, B))
    _compare(full, [step(slice(0, B // 2)), step(slice(B // 2, B))], "CondVAE recon + beta*KL")


def test_prior_step_shards_equal_full_batch():
    from toycrystals_amd import functional as TF
    from toycrystals_amd.models.diffusion_prior import DiffusionPriorFiLM
    torch.manual_seed(0)
    m = DiffusionPriorFiLM(z_dim=32, n_types=4, y_cont_dim=4, t_emb_dim=64, width=256, n_blocks=2,
                           y_cat_emb_dim=64).cuda().train()
    B = 32
    g = torch.Generator().manual_seed(7)
    z_t = torch.randn(B, 32, generator=g).cuda()
    t = torch.randint(0, 1000, (B,), generator=g).cuda()
    y_cat = (torch.arange(B) % 4).cuda()
    y_cont = torch.rand(B, 4, generator=g).cuda()
    eps = torch.randn(B, 32, generator=g).cuda()

    def step(sl):
        m.zero_grad(set_to_none=True)
        loss = TF.mse_loss(m(z_t[sl], t[sl], y_cat[sl], y_cont[sl]), eps[sl])
        loss.backward()
        return _grads(m)

    full = step(slice(0, B))
    _compare(full, [step(slice(0, B // 2)), step(slice(B // 2, B))], "DiffusionPriorFiLM MSE")


@pytest.mark.parametrize("sampler_name", ["sde", "ode"])
@pytest.mark.parametrize("world", [2, 3])
def test_sample_sharded_equals_one_gpu_run(monkeypatch, sampler_name, world):
    """dist.sample_sharded: every rank samples its shard with the batch's ONE seed and its Philox
    element offset, so the concatenated shards equal the whole batch sampled in one call, bit for
    bit (ragged shards at B = 7; the reference draws one stream per batch, sde_score_model.py:537,557).
    Ranks are emulated in one process through RANK / WORLD_SIZE (no process group: gather=False)."""
    from toycrystals_amd.dist import sample_sharded
    from toycrystals_amd.models.sde_score_model import (CondUNetTiny, VPSDE, sample_probability_flow_ode,
                                                        sample_reverse_sde_euler_maruyama)
    fn = sample_reverse_sde_euler_maruyama if sampler_name == "sde" else sample_probability_flow_ode
    torch.manual_seed(0)
    model = CondUNetTiny(4, 4, 32).cuda().eval()
    sde = VPSDE(0.1, 30.0)
    B = 7
    y_cat = (torch.arange(B) % 4).cuda()
    y_cont = torch.zeros(B, 4, device="cuda")
    y_cont[:, 1] = torch.linspace(0, 1.0, B, device="cuda")
    kw = dict(n_steps=3, guidance_scale=1.5, t_end=0.005)
    full = fn(model, sde, y_cat, y_cont, (B, 1, 64, 64), seed=11, **kw)
    parts = []
    for r in range(world):
        monkeypatch.setenv("RANK", str(r))
        monkeypatch.setenv("WORLD_SIZE", str(world))
        parts.append(sample_sharded(fn, model, sde, y_cat, y_cont, (B, 1, 64, 64), base_seed=11, gather=False, **kw))
    assert sum(p.shape[0] for p in parts) == B
    assert torch.equal(torch.cat(parts), full)
