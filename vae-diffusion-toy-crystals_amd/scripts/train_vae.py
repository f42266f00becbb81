#!/usr/bin/env python3
"""MI355X drop-in for scripts/train_vae.py (reference): same CLI flags/defaults (:225-242),
kl_stats (:17-36), loss (:309-312), outputs checkpoints/vae_last.pt (state_dict) and
results/{vae_recon, vae_samples_prior, vae_samples_mop, vae_loss}.png.

`--data-path ""` renders the reference's in-memory dataset (toycrystals.data.ToyCrystalsDataset,
non-rot-only, seed --seed) on the GPU once (toycrystals_amd.data, csrc/render.hip) and keeps it in HBM.
"""
from __future__ import annotations

import argparse
import math
import os

import _common  # noqa: F401
import torch

from toycrystals_amd import functional as TF
from toycrystals_amd.dist import BucketedGradAllReduce
from toycrystals_amd.data import ToyCrystalsDataset
from toycrystals_amd.disk_data import DeviceBatches, ToyCrystalsDiskDataset
from toycrystals_amd.models.vae import CondVAE, VAE
from toycrystals_amd.optim import Adam


def kl_stats(mu: torch.Tensor, logvar: torch.Tensor, free_bits: float = 0.0):
    """(kl_used, kl_raw) averaged over the batch; free bits in nats per latent dim (:17-36)."""
    return TF.kl_stats(mu, logvar, free_bits)


def _plt():
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    return plt


@torch.no_grad()
def save_recon_grid(model, x, y_cat, y_cont, out_path, n_pairs: int = 16, uncond: bool = False) -> None:
    plt = _plt()
    model.eval()
    x_hat, _, _ = model(x) if uncond else model(x, y_cat, y_cont)
    n = min(n_pairs, x.shape[0])
    fig, axes = plt.subplots(4, 8, figsize=(8, 4))
    axes = list(axes.flat)
    for i in range(n):
        t = int(y_cat[i].item())
        axes[2 * i].imshow(x[i, 0].cpu(), cmap="gray", vmin=0.0, vmax=1.0)
        axes[2 * i].set_title(f"X (type={t})")
        axes[2 * i].axis("off")
        axes[2 * i + 1].imshow(x_hat[i, 0].cpu(), cmap="gray", vmin=0.0, vmax=1.0)
        axes[2 * i + 1].set_title(f"X̂ (type={t})")
        axes[2 * i + 1].axis("off")
    fig.tight_layout()
    fig.savefig(out_path, dpi=200)
    plt.close(fig)


def _grid_cond(model, n, device, theta_max):
    y_cat = torch.tensor([i % model.n_types for i in range(n)], device=device, dtype=torch.int64)
    y_cont = torch.zeros((n, model.y_cont_dim), device=device)
    y_cont[:, 1] = torch.linspace(0.0, theta_max, steps=n, device=device)
    return y_cat, y_cont


def _save_grid(x, out_path, titles=None):
    plt = _plt()
    fig, axes = plt.subplots(6, 6, figsize=(6, 6))
    for i, ax in enumerate(axes.flat):
        ax.imshow(x[i, 0].cpu(), cmap="gray", vmin=0.0, vmax=1.0)
        if titles is not None:
            ax.set_title(f"t={int(titles[i].item())}", fontsize=7)
        ax.axis("off")
    fig.tight_layout()
    fig.savefig(out_path, dpi=200)
    plt.close(fig)


@torch.no_grad()
def save_prior_samples(model, out_path, device, uncond: bool, theta_max: float = math.pi / 3.0) -> None:
    model.eval()
    n = 36
    z = torch.randn((n, model.z_dim), device=device)
    if uncond:
        _save_grid(model.decode(z), out_path)
    else:
        y_cat, y_cont = _grid_cond(model, n, device, theta_max)
        _save_grid(model.decode(z, y_cat, y_cont), out_path, y_cat)


@torch.no_grad()
def save_mop_samples(model, dl, out_path, device, uncond: bool, pool_size: int = 4096,
                     theta_max: float = math.pi / 3.0, decode_with_target: bool = True) -> None:
    """Mixture-of-posteriors baseline (reference :113-220): nearest same-type example per grid cell,
    z ~ q(z | x), decoded with the target condition."""
    model.eval()
    n = 36
    xs, ycs, yvs, seen = [], [], [], 0
    for x, y_cat, y_cont in dl:
        xs.append(x)
        ycs.append(y_cat)
        yvs.append(y_cont)
        seen += x.shape[0]
        if seen >= pool_size:
            break
    x_pool, yc_pool, yv_pool = (torch.cat(v)[:pool_size] for v in (xs, ycs, yvs))
    if uncond:
        idx = torch.randint(0, x_pool.shape[0], (n,), device=device)
        mu, lv = model.encode(x_pool[idx])
        _save_grid(model.decode(model.reparameterise(mu, lv)), out_path)
        return
    t_cat, t_cont = _grid_cond(model, n, device, theta_max)
    idxs = []
    for i in range(n):
        mask = yc_pool == t_cat[i]
        if not torch.any(mask):
            idxs.append(int(torch.randint(0, x_pool.shape[0], (1,)).item()))
            continue
        pi = torch.nonzero(mask, as_tuple=False).squeeze(1)
        idxs.append(int(pi[int(torch.argmin((yv_pool[pi, 1] - t_cont[i, 1]).abs()).item())].item()))
    idx = torch.tensor(idxs, device=device, dtype=torch.long)
    mu, lv = model.encode(x_pool[idx], yc_pool[idx], yv_pool[idx])
    z = model.reparameterise(mu, lv)
    if decode_with_target:
        _save_grid(model.decode(z, t_cat, t_cont), out_path, t_cat)
    else:
        _save_grid(model.decode(z, yc_pool[idx], yv_pool[idx]), out_path, yc_pool[idx])


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser()
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--img-size", type=int, default=64)
    p.add_argument("--n-samples", type=int, default=50_000)
    p.add_argument("--batch-size", type=int, default=128)
    p.add_argument("--epochs", type=int, default=15)
    p.add_argument("--lr", type=float, default=2e-3)
    p.add_argument("--z-dim", type=int, default=32)
    p.add_argument("--n-types", type=int, default=4)
    p.add_argument("--y-cont-dim", type=int, default=4)
    p.add_argument("--beta", type=float, default=0.0003)
    p.add_argument("--device", type=str, default="cuda")
    p.add_argument("--num-workers", type=int, default=0)
    p.add_argument("--data-path", type=str, default="data/toycrystals_train_rotonly.pt")
    p.add_argument("--cond-drop", type=float, default=0.0)
    p.add_argument("--uncond", dest="uncond", action="store_true", help="Train unconditional VAE.")
    p.add_argument("--cond", dest="uncond", action="store_false", help="Train conditional VAE.")
    p.add_argument("--free-bits", type=float, default=0.05, help="Free bits threshold in nats per latent dim (0 disables).")
    p.set_defaults(uncond=False)
    # additive (not in the reference): replay a recorded reference run
    p.add_argument("--replay-draws", type=str, default="",
                   help="npz with a reference run's DataLoader item order ('order') and reparameterisation draws "
                        "('eps' [steps, B, z]) (tests/golden/make_config1_golden.py): train on exactly those "
                        "batches and draws and log every step to results/vae_steps.jsonl (parity runs)")
    # additive (not in the reference): batch-DP draw semantics
    p.add_argument("--global-draws", type=int, default=1, choices=[0, 1],
                   help="1: every rank draws the reparameterisation eps and the condition-dropout mask for the "
                        "WHOLE global batch from one shared device generator and keeps its slice (N GPUs = 1 GPU); "
                        "0: per-rank draws of the local shard")
    return p


def main() -> int:
    args = build_parser().parse_args()
    rank, world, dp_dev = _common.init_dp()
    torch.manual_seed(args.seed)
    device = dp_dev if dp_dev is not None else _common.pick_device(args.device)
    torch.cuda.manual_seed(args.seed if args.global_draws else args.seed + 7919 * rank)
    lead = rank == 0
    os.makedirs("results", exist_ok=True)
    os.makedirs("checkpoints", exist_ok=True)
    if args.data_path:
        ds = ToyCrystalsDiskDataset(args.data_path)
    else:  # the reference's in-memory renderer (:259-260): non-rot-only, generator seed --seed
        ds = ToyCrystalsDataset(n_samples=args.n_samples, img_size=args.img_size, seed=args.seed,
                                device=device).materialize()
    replay = None
    if args.replay_draws:
        import numpy as np
        z = np.load(args.replay_draws, allow_pickle=False)
        replay = {"order": torch.from_numpy(z["order"].astype(np.int64)), "eps": torch.from_numpy(z["eps"])}
        if args.uncond or args.cond_drop > 0.0:
            raise SystemExit("--replay-draws covers the conditional VAE with --cond-drop 0 (reparameterise draws only)")
    dl = DeviceBatches(ds, args.batch_size, device, shuffle=True, drop_last=True, rank=rank, world=world,
                       fixed_order=None if replay is None else replay["order"])
    if replay is not None:  # the recording must cover every step of this run at this batch size
        need = args.epochs * len(dl)
        if replay["eps"].ndim != 3 or replay["eps"].shape[0] < need or replay["eps"].shape[1] != args.batch_size \
                or replay["eps"].shape[2] != args.z_dim:
            raise SystemExit(f"--replay-draws: eps {tuple(replay['eps'].shape)} does not cover {args.epochs} epoch(s) x "
                             f"{len(dl)} steps of batch {args.batch_size}, z_dim {args.z_dim}")
        if args.epochs > 1:
            raise SystemExit("--replay-draws records ONE epoch's item order: run it with --epochs 1")
    step_log = open(os.path.join("results", "vae_steps.jsonl"), "w", encoding="utf-8") if (replay and lead) else None
    try:
        return _train(args, rank, world, device, lead, ds, dl, replay, step_log)
    finally:
        if step_log is not None:
            step_log.close()


def _train(args, rank, world, device, lead, ds, dl, replay, step_log) -> int:
    if args.uncond:
        model = VAE(z_dim=args.z_dim).to(device)
    else:
        if lead:
            print("Training conditional VAE")
        model = CondVAE(z_dim=args.z_dim, n_types=args.n_types, y_cont_dim=args.y_cont_dim,
                        cond_drop=args.cond_drop).to(device)
    opt = Adam(model.parameters(), lr=args.lr)
    params = [p for p in model.parameters() if p.requires_grad]
    # gradient averaging overlapped with backward (bucketed RCCL all-reduces; no-op on one GPU)
    grad_ar = BucketedGradAllReduce(params)
    loss_hist, recon_hist, kl_hist, klr_hist = [], [], [], []
    if lead:
        print("starting training loop...")
        print("gpu:", torch.cuda.get_device_name(device), f"x{world}")
    for epoch in range(args.epochs):
        model.train()
        tot = torch.zeros(4, device=device, dtype=torch.float64)
        for step, (x, y_cat, y_cont) in enumerate(dl):
            draws = None
            if replay is not None:
                per = x.shape[0]
                k = epoch * len(dl) + step
                draws = (replay["eps"][k, rank * per:(rank + 1) * per].to(device), None)
            elif args.global_draws:
                # reference order (vae.py:57-60 then :65-67): reparam eps, then the keep mask
                Bg, per = args.batch_size, x.shape[0]
                sl = slice(rank * per, (rank + 1) * per)
                rep = torch.randn((Bg, args.z_dim), device=device)[sl]
                keep = (torch.rand((Bg, 1), device=device)[sl]
                        if (not args.uncond and args.cond_drop > 0.0) else None)
                draws = (rep,) if args.uncond else (rep, keep)
            x_hat, mu, logvar = model(x, draws=draws) if args.uncond else model(x, y_cat, y_cont, draws=draws)
            recon = TF.mse_loss(x_hat, x)
            kl_used, kl_raw = kl_stats(mu, logvar, free_bits=args.free_bits)
            beta = args.beta * min(1.0, (epoch + 1) / 5.0)
            loss = recon + beta * kl_used
            grad_ar.zero_grad()  # grads = zeroed views into the all-reduce buckets
            loss.backward()
            grad_ar.finish()
            opt.step()
            tot += torch.stack([loss.detach(), recon.detach(), kl_used.detach(), kl_raw.detach()]).double()
            if step_log is not None:
                import json
                step_log.write(json.dumps({"epoch": epoch + 1, "step": step + 1, "loss": float(loss.item()),
                                           "recon": float(recon.item()), "kl_used": float(kl_used.item()),
                                           "kl_raw": float(kl_raw.item())}) + "\n")
        nb = max(len(dl), 1)
        avg = [_common.allreduce_scalar_mean(v / nb, world, device) for v in tot.tolist()]
        loss_hist.append(avg[0])
        recon_hist.append(avg[1])
        kl_hist.append(avg[2])
        klr_hist.append(avg[3])
        if lead:
            print(f"epoch {epoch + 1:02d}/{args.epochs} loss={avg[0]:.4f} recon={avg[1]:.4f} kl={avg[2]:.6f}")
            if step_log is not None:
                step_log.flush()
            torch.save(model.state_dict(), "checkpoints/vae_last.pt")
    if lead:
        x0, y0_cat, y0_cont = next(iter(dl))
        x0, y0_cat, y0_cont = x0[:16], y0_cat[:16], y0_cont[:16]
        save_recon_grid(model, x0, y0_cat, y0_cont, "results/vae_recon.png", uncond=args.uncond)
        save_prior_samples(model, "results/vae_samples_prior.png", device=device, uncond=args.uncond)
        save_mop_samples(model, dl, "results/vae_samples_mop.png", device=device, uncond=args.uncond, pool_size=4096,
                         decode_with_target=True)
        plt = _plt()
        fig = plt.figure(figsize=(5, 3))
        plt.plot(loss_hist, label="total")
        plt.plot(recon_hist, label="recon")
        plt.plot(kl_hist, label="kl")
        plt.xlabel("epoch")
        plt.ylabel("loss")
        plt.legend()
        plt.tight_layout()
        plt.savefig("results/vae_loss.png", dpi=200)
        plt.close(fig)
        print("saved: results/vae_recon.png, results/vae_samples_prior.png, results/vae_loss.png")
    _common.shutdown_dp(world)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
