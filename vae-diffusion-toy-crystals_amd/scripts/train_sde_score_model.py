#!/usr/bin/env python3
"""MI355X drop-in for scripts/train_sde_score_model.py (reference :1-300): same CLI flags and
defaults (:84-122), run-dir naming (:26-32), checkpoint dict {epoch_next, model, opt, loss_hist,
config[, ema]} at <out>/checkpoints/sde_score_model_last.pt (:35-79), metrics.jsonl, sample grids.

Differences by design: batches come from a device-resident dataset (toycrystals_amd.disk_data.
DeviceBatches: one HIP gather per batch) instead of a host DataLoader; the optimiser is the fused
multi-tensor Adam (state_dict-compatible with torch.optim.Adam); under torchrun each rank trains
on an equal slice of every global batch and gradients are averaged with one RCCL all-reduce
(the mean of equal-shard means is the global mean, so the loss semantics are unchanged), and
with --global-draws 1 (default) every rank draws the whole global batch's u/eps/drop from one
shared device stream and keeps its slice, so an N-GPU run computes the 1-GPU run's step.
"""
from __future__ import annotations

import argparse
import json
import os
from datetime import datetime
from typing import Any

import _common  # noqa: F401  (package path)
import torch
from tqdm import tqdm

from toycrystals_amd.dist import BucketedGradAllReduce
from toycrystals_amd.disk_data import DeviceBatches, ToyCrystalsDiskDataset
from toycrystals_amd.models.sde_score_model import CondUNetTiny, VPSDE, diffusion_loss_eps, save_sde_samples
from toycrystals_amd.optim import Adam, ema_update


def _make_run_name(args: argparse.Namespace) -> str:
    ts = datetime.now().strftime("%Y%m%d_%H%M%S")
    return f"{ts}_lr{args.lr:.2e}_ch{args.base_ch}_b{args.beta_max:g}_tp{args.t_power:g}_pu{args.p_uncond:g}"


def _save_checkpoint(ckpt_path: str, *, epoch_next: int, model, opt, loss_hist, config, ema_model=None) -> None:
    d: dict[str, Any] = {"epoch_next": int(epoch_next), "model": model.state_dict(), "opt": opt.state_dict(),
                         "loss_hist": list(loss_hist), "config": dict(config)}
    if ema_model is not None:
        d["ema"] = ema_model.state_dict()
    torch.save(d, ckpt_path)


def _try_load_checkpoint(ckpt_path: str, device, model, opt, ema_model=None):
    if not os.path.exists(ckpt_path):
        return 0, []
    obj = torch.load(ckpt_path, map_location=device, weights_only=True)
    model.load_state_dict(obj["model"])
    opt.load_state_dict(obj["opt"])
    if ema_model is not None:
        ema_model.load_state_dict(obj["ema"] if "ema" in obj else model.state_dict())
    return int(obj.get("epoch_next", 0)), list(obj.get("loss_hist", []))


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser()
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--device", type=str, default="cuda")
    p.add_argument("--data-path", type=str, default="data/toycrystals_train_rotonly.pt")
    p.add_argument("--out-dir", type=str, default=None, help="Run output directory. If omitted, a timestamped run dir is created under runs/sde_score/")
    p.add_argument("--resume", action="store_true")
    p.add_argument("--n-types", type=int, default=4)
    p.add_argument("--y-cont-dim", type=int, default=4)
    p.add_argument("--base-ch", type=int, default=96)
    p.add_argument("--emb-dim", type=int, default=128)
    p.add_argument("--cond-ch", type=int, default=8)
    p.add_argument("--time-ch", type=int, default=8)
    p.add_argument("--beta-min", type=float, default=0.1)
    p.add_argument("--beta-max", type=float, default=30.0)
    p.add_argument("--batch-size", type=int, default=128)
    p.add_argument("--epochs", type=int, default=40)
    p.add_argument("--lr", type=float, default=1e-4)
    p.add_argument("--p-uncond", type=float, default=0.1)
    p.add_argument("--t-power", type=float, default=1.0, help="Sample t as t=u**t_power. >1 biases towards small t.")
    p.add_argument("--ema-decay", type=float, default=0.0, help="0 disables EMA. Typical: 0.999 or 0.9999")
    p.add_argument("--sample-every", type=int, default=10000)
    p.add_argument("--sample-steps", type=int, default=200)
    p.add_argument("--cfg", type=float, default=0)
    p.add_argument("--t-end", type=float, default=1e-3)
    p.add_argument("--sample-from-ema", type=int, default=1, choices=[0, 1], help="If EMA enabled, save sample grids using EMA weights.")
    # additive (not in the reference): batch-DP draw semantics
    p.add_argument("--global-draws", type=int, default=1, choices=[0, 1],
                   help="1: every rank draws u/eps/drop for the WHOLE global batch from the same device generator "
                        "(reference order, sde_score_model.py:380-391) and keeps its slice, so an N-GPU run equals "
                        "the 1-GPU run; 0: per-rank draws of the local shard only")
    return p


def main() -> int:
    args = build_parser().parse_args()
    rank, world, dp_dev = _common.init_dp()
    torch.manual_seed(args.seed)  # identical init on every rank
    device = dp_dev if dp_dev is not None else _common.pick_device(args.device)
    # global draws: one device stream shared by all ranks; else per-rank streams
    torch.cuda.manual_seed(args.seed if args.global_draws else args.seed + 7919 * rank)
    if args.out_dir is None:
        args.out_dir = os.path.join("runs", "sde_score", _make_run_name(args))
    lead = rank == 0
    if lead:
        print(f"run dir: {args.out_dir}")
    results_dir = os.path.join(args.out_dir, "results")
    ckpt_dir = os.path.join(args.out_dir, "checkpoints")
    os.makedirs(results_dir, exist_ok=True)
    os.makedirs(ckpt_dir, exist_ok=True)
    metrics_path = os.path.join(args.out_dir, "metrics.jsonl")
    ckpt_path = os.path.join(ckpt_dir, "sde_score_model_last.pt")

    ds = ToyCrystalsDiskDataset(args.data_path)
    dl = DeviceBatches(ds, args.batch_size, device, shuffle=True, drop_last=True, rank=rank, world=world)

    mk = lambda: CondUNetTiny(n_types=args.n_types, y_cont_dim=args.y_cont_dim, base_ch=args.base_ch,  # noqa: E731
                              emb_dim=args.emb_dim, cond_ch=args.cond_ch, time_ch=args.time_ch).to(device)
    model = mk()
    ema_model = None
    if args.ema_decay > 0.0:
        if not (0.0 < args.ema_decay < 1.0):
            raise ValueError("--ema-decay must be in (0,1) or 0 to disable.")
        ema_model = mk()
        ema_model.load_state_dict(model.state_dict())
        ema_model.eval()
        for p_ in ema_model.parameters():
            p_.requires_grad_(False)
    sde = VPSDE(beta_min=args.beta_min, beta_max=args.beta_max)
    config = {"img_ch": 1, "n_types": args.n_types, "y_cont_dim": args.y_cont_dim, "base_ch": args.base_ch,
              "emb_dim": args.emb_dim, "cond_ch": args.cond_ch, "time_ch": args.time_ch, "beta_min": args.beta_min,
              "beta_max": args.beta_max, "t_power": args.t_power, "p_uncond": args.p_uncond}
    opt = Adam(model.parameters(), lr=args.lr)
    start_epoch, loss_hist = 0, []
    if args.resume:
        start_epoch, loss_hist = _try_load_checkpoint(ckpt_path, device, model, opt, ema_model)
        if start_epoch > 0 and lead:
            print(f"resumed from: {ckpt_path} (next epoch {start_epoch + 1})")
    if lead:
        print("starting SDE score-model training loop.")
        print("gpu:", torch.cuda.get_device_name(device), f"x{world}")
        if not os.path.exists(metrics_path):
            open(metrics_path, "w", encoding="utf-8").close()
    params = [p for p in model.parameters() if p.requires_grad]
    # gradient averaging overlapped with backward (bucketed RCCL all-reduces; no-op on one GPU)
    grad_ar = BucketedGradAllReduce(params)
    for epoch in range(start_epoch, args.epochs):
        model.train()
        total = torch.zeros((), device=device, dtype=torch.float64)
        it = tqdm(dl, desc=f"epoch {epoch + 1:03d}/{args.epochs}", disable=not lead)
        for x0, y_cat, y_cont in it:
            draws = None
            if args.global_draws:
                # the global batch's draws in the reference's order, this rank's slice (DeviceBatches
                # yields rows [rank*per, (rank+1)*per) of every global batch)
                Bg, per = args.batch_size, x0.shape[0]
                u = torch.rand((Bg,), device=device)
                eps = torch.randn((Bg,) + tuple(x0.shape[1:]), device=device)
                drop = torch.rand((Bg,), device=device) if args.p_uncond > 0.0 else None
                sl = slice(rank * per, (rank + 1) * per)
                draws = (u[sl], eps[sl], drop[sl] if drop is not None else None)
            loss = diffusion_loss_eps(model=model, sde=sde, x0=x0, y_cat=y_cat, y_cont=y_cont,
                                      p_uncond=args.p_uncond, t_power=args.t_power, draws=draws)
            grad_ar.zero_grad()  # grads = zeroed views into the all-reduce buckets
            loss.backward()
            grad_ar.finish()
            opt.step()
            if ema_model is not None:
                ema_update(ema_model, model, float(args.ema_decay))
            total += loss.detach()
        avg = _common.allreduce_scalar_mean(float(total.item()) / max(len(dl), 1), world, device)
        loss_hist.append(avg)
        if lead:
            print(f"epoch {epoch + 1:03d}/{args.epochs}: loss={avg:.6f}")
            _save_checkpoint(ckpt_path, epoch_next=epoch + 1, model=model, opt=opt, loss_hist=loss_hist,
                             config=config, ema_model=ema_model)
            with open(metrics_path, "a", encoding="utf-8") as f:
                f.write(json.dumps({"epoch": epoch + 1, "loss": avg}) + "\n")
            if ((epoch + 1) % args.sample_every == 0) or (epoch == args.epochs - 1):
                out_path = os.path.join(results_dir, f"sde_samples_epoch_{epoch + 1:03d}.png")
                sample_model = ema_model if (ema_model is not None and args.sample_from_ema == 1) else model
                with _common.lead_only_rng(device):  # the other ranks do not draw: keep the streams in step
                    save_sde_samples(model=sample_model, sde=sde, out_path=out_path, device=device,
                                     steps=args.sample_steps, cfg=args.cfg, t_end=args.t_end)
                print(f"  saved: {out_path}")
    if lead:
        import matplotlib
        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
        fig = plt.figure(figsize=(5, 3))
        plt.plot(loss_hist, label="eps_mse")
        plt.xlabel("epoch")
        plt.ylabel("loss")
        plt.legend()
        plt.tight_layout()
        loss_png = os.path.join(results_dir, "sde_loss.png")
        plt.savefig(loss_png, dpi=200)
        plt.close(fig)
        print(f"saved: {loss_png}")
        print(f"checkpoint: {ckpt_path}")
    _common.shutdown_dp(world)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
