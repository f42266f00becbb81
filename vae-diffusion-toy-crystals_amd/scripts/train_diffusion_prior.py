#!/usr/bin/env python3
"""MI355X drop-in for scripts/train_diffusion_prior.py (reference): same CLI (:110-136), latent
cache file {z0, y_cat, y_cont, z_mean, z_std} (:162-190), standardisation, prior training step
(:251-277: t = clamp(long(u^2 T)), q_sample, MSE, 4 t-buckets), checkpoints/diffusion_prior_last.pt
(state_dict, always this path: reference quirk :283) and results/diffusion_{samples,loss}.png.

Device path: the frozen CondVAE encoder, q_sample (tcx_prior_qsample), the FiLM prior forward /
backward and Adam all run in libtcx; latents stay in HBM and batches are index gathers.
"""
from __future__ import annotations

import argparse
import math
import os

import _common  # noqa: F401
import torch
from tqdm import tqdm

from toycrystals_amd import functional as TF
from toycrystals_amd._lib import check, lib, ptr, stream_ptr
from toycrystals_amd.dist import BucketedGradAllReduce, ZeroAdam, dp_active
from toycrystals_amd.disk_data import DeviceBatches, ToyCrystalsDiskDataset
from toycrystals_amd.models.diffusion_prior import DiffusionPriorFiLM, DiffusionSchedule
from toycrystals_amd.models.vae import CondVAE
from toycrystals_amd.optim import Adam


@torch.no_grad()
def build_latent_dataset(vae, dl, device, z_target: str = "mu", max_items=None):
    """Encode the dataset with the frozen VAE (reference :17-58); returns (z0, y_cat, y_cont) on the CPU."""
    vae.eval()
    zs, ycats, yconts, seen = [], [], [], 0
    for x, y_cat, y_cont in tqdm(dl, desc="encoding latents"):
        mu, logvar = vae.encode(x, y_cat, y_cont)
        if z_target == "mu":
            z0 = mu
        elif z_target == "sample":
            z0 = vae.reparameterise(mu, logvar)
        else:
            raise ValueError(f"unknown z_target={z_target}")
        zs.append(z0.detach().cpu())
        ycats.append(y_cat.detach().cpu())
        yconts.append(y_cont.detach().cpu())
        seen += x.shape[0]
        if max_items is not None and seen >= max_items:
            break
    return torch.cat(zs), torch.cat(ycats), torch.cat(yconts)


@torch.no_grad()
def save_diffusion_samples(vae, prior, sched, out_path, device, z_mean, z_std, n: int = 36,
                           theta_max: float = math.pi / 3.0, ddim_steps: int = 50) -> None:
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    vae.eval()
    prior.eval()
    y_cat = torch.tensor([i % vae.n_types for i in range(n)], device=device, dtype=torch.int64)
    y_cont = torch.zeros((n, vae.y_cont_dim), device=device)
    y_cont[:, 1] = torch.linspace(0.0, theta_max, steps=n, device=device)
    z_norm = sched.ddim_sample(prior, y_cat=y_cat, y_cont=y_cont, n_steps=ddim_steps, eta=0.0)
    z = z_norm * z_std.to(device) + z_mean.to(device)
    x = vae.decode(z, y_cat, y_cont)
    fig, axes = plt.subplots(6, 6, figsize=(6, 6))
    for i, ax in enumerate(axes.flat):
        ax.imshow(x[i, 0].cpu(), cmap="gray", vmin=0.0, vmax=1.0)
        ax.set_title(f"t={int(y_cat[i].item())}", fontsize=7)
        ax.axis("off")
    fig.tight_layout()
    fig.savefig(out_path, dpi=200)
    plt.close(fig)


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser()
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--device", type=str, default="cuda")
    p.add_argument("--data-path", type=str, default="data/toycrystals_train_rotonly.pt")
    p.add_argument("--vae-ckpt", type=str, default="checkpoints/vae_last.pt")
    p.add_argument("--z-dim", type=int, default=32)
    p.add_argument("--n-types", type=int, default=4)
    p.add_argument("--y-cont-dim", type=int, default=4)
    p.add_argument("--z-target", type=str, choices=["mu", "sample"], default="mu")
    p.add_argument("--latent-cache", type=str, default="data/latents_rotonly_mu.pt")
    p.add_argument("--rebuild-latents", action="store_true")
    p.add_argument("--max-items", type=int, default=50_000)
    p.add_argument("--T", type=int, default=200)
    p.add_argument("--beta-start", type=float, default=1e-4)
    p.add_argument("--beta-end", type=float, default=1)
    p.add_argument("--t-emb-dim", type=int, default=64)
    p.add_argument("--width", type=int, default=512)
    p.add_argument("--batch-size", type=int, default=256)
    p.add_argument("--epochs", type=int, default=600)
    p.add_argument("--lr", type=float, default=1e-4)
    p.add_argument("--ddim-steps", type=int, default=50)
    p.add_argument("--prior-ckpt", type=str, default="checkpoints/diffusion_prior_last.pt")
    p.add_argument("--resume", action="store_true")
    p.add_argument("--sample-only", action="store_true")
    # additive (not in the reference): batch-DP draw semantics
    p.add_argument("--global-draws", type=int, default=1, choices=[0, 1],
                   help="1: every rank draws u/eps for the WHOLE global batch from one shared device generator and "
                        "keeps its slice (N GPUs = 1 GPU); 0: per-rank draws of the local shard")
    p.add_argument("--zero", type=int, default=1, choices=[0, 1],
                   help="batch-DP only: 1 = ZeRO-1 (gradient reduce-scatter, fused Adam on this rank's 1/N shard, "
                        "parameter all-gather); 0 = bucketed all-reduce + whole-model Adam on every rank")
    return p


def main() -> int:
    args = build_parser().parse_args()
    rank, world, dp_dev = _common.init_dp()
    torch.manual_seed(args.seed)
    device = dp_dev if dp_dev is not None else _common.pick_device(args.device)
    torch.cuda.manual_seed(args.seed if args.global_draws else args.seed + 7919 * rank)
    lead = rank == 0
    for d in ("results", "checkpoints", "data"):
        os.makedirs(d, exist_ok=True)
    ds = ToyCrystalsDiskDataset(args.data_path)
    vae = CondVAE(z_dim=args.z_dim, n_types=args.n_types, y_cont_dim=args.y_cont_dim, cond_drop=0.0).to(device)
    vae.load_state_dict(torch.load(args.vae_ckpt, map_location=device, weights_only=True))
    vae.eval()
    for p_ in vae.parameters():
        p_.requires_grad_(False)
    # Rank 0 alone loads or builds the latent set (and writes the cache); under torchrun the other
    # ranks receive rank 0's tensors by broadcast, so every rank trains on the same latents even
    # with --z-target sample (whose reparameterisation draws noise) and the encode runs once.
    latents = None
    if lead:
        if (not args.rebuild_latents) and os.path.exists(args.latent_cache):
            obj = torch.load(args.latent_cache, map_location="cpu", weights_only=True)
            z0, y_cat, y_cont = obj["z0"], obj["y_cat"], obj["y_cont"]
            if "z_mean" in obj and "z_std" in obj:
                z_mean, z_std = obj["z_mean"], obj["z_std"]
            else:
                z_mean = z0.mean(dim=0, keepdim=True)
                z_std = torch.clamp(z0.std(dim=0, keepdim=True), min=1e-6)
            print(f"loaded latents: {args.latent_cache}  z0={tuple(z0.shape)}")
        else:
            dl = DeviceBatches(ds, 512, device, shuffle=False, drop_last=False)
            z0, y_cat, y_cont = build_latent_dataset(vae, dl, device=device, z_target=args.z_target,
                                                     max_items=args.max_items)
            z_mean = z0.mean(dim=0, keepdim=True)
            z_std = torch.clamp(z0.std(dim=0, keepdim=True), min=1e-6)
            torch.save({"z0": z0, "y_cat": y_cat, "y_cont": y_cont, "z_mean": z_mean, "z_std": z_std},
                       args.latent_cache)
            print(f"saved latents: {args.latent_cache}  z0={tuple(z0.shape)}")
        latents = [z0, y_cat, y_cont, z_mean, z_std]
    z0, y_cat, y_cont, z_mean, z_std = _common.broadcast_from_lead(latents, world, device)
    # rank 0's build drew reparameterisation noise (--z-target sample) as the one-GPU run does:
    # continue every rank from its generator state so the --global-draws streams stay equal
    _common.sync_rng_from_lead(world, device)
    z0n = ((z0 - z_mean) / z_std).to(device).contiguous()
    y_cat_d, y_cont_d = y_cat.to(device).contiguous(), y_cont.to(device).contiguous()
    prior = DiffusionPriorFiLM(z_dim=args.z_dim, n_types=args.n_types, y_cont_dim=args.y_cont_dim,
                               t_emb_dim=args.t_emb_dim, width=args.width, n_blocks=8, y_cat_emb_dim=64).to(device)
    sched = DiffusionSchedule.linear(T=args.T, beta_start=args.beta_start, beta_end=args.beta_end, device=device)
    if (args.sample_only or args.resume) and os.path.exists(args.prior_ckpt):
        prior.load_state_dict(torch.load(args.prior_ckpt, map_location=device, weights_only=True))
        if lead:
            print(f"loaded diffusion prior: {args.prior_ckpt}")
    if args.sample_only:
        if lead:
            save_diffusion_samples(vae=vae, prior=prior, sched=sched, out_path="results/diffusion_samples.png",
                                   device=device, z_mean=z_mean, z_std=z_std, ddim_steps=args.ddim_steps)
            print("sample-only: saved results/diffusion_samples.png")
        _common.shutdown_dp(world)
        return 0
    params = [p for p in prior.parameters() if p.requires_grad]
    zero = bool(args.zero) and dp_active()
    if zero:
        # ZeRO-1: the gradients reduce-scattered per bucket while backward runs, Adam
        # on this rank's shard (1/N of the moments and of the update's HBM traffic), the updated
        # shards all-gathered; the same Adam arithmetic as torch.optim.Adam element for element
        opt = ZeroAdam(params, lr=args.lr)
        grad_ar = None
    else:
        opt = Adam(prior.parameters(), lr=args.lr)
        # gradient averaging overlapped with backward (bucketed RCCL all-reduces; no-op on one GPU)
        grad_ar = BucketedGradAllReduce(params)
    loss_hist = []
    if lead:
        print("starting diffusion training loop.")
        print("gpu:", torch.cuda.get_device_name(device), f"x{world}")
    N, B = z0n.shape[0], args.batch_size
    if B % world:
        raise SystemExit(f"--batch-size {B} must be divisible by the world size {world}")
    per = B // world
    L = lib()
    st = stream_ptr(device)
    t = torch.empty((per,), device=device, dtype=torch.int64)
    z_t = torch.empty((per, args.z_dim), device=device)
    for epoch in range(args.epochs):
        bucket_sum = torch.zeros(4, device=device)
        bucket_n = torch.zeros(4, device=device)
        prior.train()
        total = torch.zeros((), device=device, dtype=torch.float64)
        order = torch.randperm(N).to(device)
        nb = N // B
        for i in range(nb):
            idx = order[i * B + rank * per:i * B + (rank + 1) * per]
            z0b, ycb, yvb = z0n.index_select(0, idx), y_cat_d.index_select(0, idx), y_cont_d.index_select(0, idx)
            if args.global_draws:  # reference order (:251-256) over the global batch, this rank's slice
                sl = slice(rank * per, (rank + 1) * per)
                u = torch.rand((B,), device=device)[sl].contiguous()
                eps = torch.randn((B, args.z_dim), device=device)[sl].contiguous()
            else:
                u = torch.rand((per,), device=device)
                eps = torch.randn_like(z0b)
            check(L.tcx_prior_qsample(ptr(z0b), ptr(eps), ptr(u), ptr(sched.sqrt_alpha_bars),
                                      ptr(sched.sqrt_one_minus_alpha_bars), args.T, per, args.z_dim, ptr(t), ptr(z_t),
                                      st), "tcx_prior_qsample")
            eps_pred = prior(z_t, t, ycb, yvb)
            loss = TF.mse_loss(eps_pred, eps)
            with torch.no_grad():
                per_s = ((eps_pred - eps) ** 2).mean(dim=1)
                q = torch.clamp((t.float() / args.T * 4).long(), 0, 3)
                bucket_sum.index_add_(0, q, per_s)
                bucket_n.index_add_(0, q, torch.ones_like(per_s))
            if zero:
                opt.zero_grad()  # grads = zeroed views into the reduce-scatter buckets
                loss.backward()
                opt.step()  # reduce-scatter wait, shard Adam, all-gather
            else:
                grad_ar.zero_grad()  # grads = zeroed views into the all-reduce buckets
                loss.backward()
                grad_ar.finish()
                opt.step()
            total += loss.detach()
        avg = _common.allreduce_scalar_mean(float(total.item()) / max(nb, 1), world, device)
        loss_hist.append(avg)
        if lead:
            print(f"epoch {epoch + 1:02d}/{args.epochs} diffusion_loss={avg:.6f}")
            # (cloned: under ZeRO-1 the parameters are views into the flat buckets, whose whole storage a
            # view would drag into the file)
            torch.save({k: v.clone() for k, v in prior.state_dict().items()}, "checkpoints/diffusion_prior_last.pt")
            with _common.lead_only_rng(device):  # the other ranks do not draw: keep the streams in step
                save_diffusion_samples(vae=vae, prior=prior, sched=sched, out_path="results/diffusion_samples.png",
                                       device=device, z_mean=z_mean, z_std=z_std, ddim_steps=args.ddim_steps)
            bucket_avg = (bucket_sum / torch.clamp(bucket_n, min=1)).detach().cpu().tolist()
            print("  bucket loss (low t -> high t):", [f"{v:.3f}" for v in bucket_avg])
    if lead:
        import matplotlib
        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
        fig = plt.figure(figsize=(5, 3))
        plt.plot(loss_hist, label="diffusion_loss")
        plt.xlabel("epoch")
        plt.ylabel("loss")
        plt.legend()
        plt.tight_layout()
        plt.savefig("results/diffusion_loss.png", dpi=200)
        plt.close(fig)
        print("saved: results/diffusion_samples.png, results/diffusion_loss.png, checkpoints/diffusion_prior_last.pt")
    _common.shutdown_dp(world)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
