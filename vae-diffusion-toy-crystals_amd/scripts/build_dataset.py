#!/usr/bin/env python3
"""MI355X drop-in for scripts/build_dataset.py (reference :1-47): the same flags and defaults
(:13-21, including `--rot-only` being a store_true that defaults to True, so every dataset is
rotation-only), the same file (torch.save of {"x_u8" [N,1,H,W] uint8, "y_cat" [N] int64,
"y_cont" [N,4] float32}, :26-40) and the same per-item content.  Items are generated in batches:
the draws and atom positions on the host (toycrystals_amd.data, bit-identical to the reference),
the Gaussian splatting + normalisation + uint8 quantisation in one tcx_render_crystals launch
per batch on the GPU (the reference renders each item on the CPU).
"""
from __future__ import annotations

import argparse
import os
import time
from pathlib import Path

import _common  # noqa: F401
import torch

from toycrystals_amd.data import ToyCrystalsDataset


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser()
    p.add_argument("--out", type=str, default="data/toycrystals_train_rotonly.pt")
    p.add_argument("--n-samples", type=int, default=50_000)
    p.add_argument("--img-size", type=int, default=64)
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--n-types", type=int, default=4)
    p.add_argument("--simple", default=False, action="store_true")
    p.add_argument("--rot-only", default=True, action="store_true")
    p.add_argument("--device", type=str, default="cuda")
    p.add_argument("--render-batch", type=int, default=4096, help="images per GPU render launch")
    return p


def build(args) -> dict:
    ds = ToyCrystalsDataset(n_samples=args.n_samples, img_size=args.img_size, seed=args.seed, n_types=args.n_types,
                            simple=args.simple, rot_only=args.rot_only, device=args.device)
    n, s = args.n_samples, args.img_size
    x_u8 = torch.empty((n, 1, s, s), dtype=torch.uint8)
    y_cat = torch.empty((n,), dtype=torch.int64)
    y_cont = torch.empty((n, 4), dtype=torch.float32)
    for i0 in range(0, n, args.render_batch):
        idx = list(range(i0, min(n, i0 + args.render_batch)))
        x, yc, yv = ds.render(idx, u8=True)
        x_u8[i0:i0 + len(idx)] = x.cpu()
        y_cat[i0:i0 + len(idx)] = yc.cpu()
        y_cont[i0:i0 + len(idx)] = yv.cpu()
        print(f"{i0}/{n}", flush=True)
    return {"x_u8": x_u8, "y_cat": y_cat, "y_cont": y_cont}


def main() -> int:
    args = build_parser().parse_args()
    out_path = Path(args.out)
    os.makedirs(out_path.parent, exist_ok=True)
    t0 = time.perf_counter()
    obj = build(args)
    torch.save(obj, out_path)
    print(f"saved {out_path} ({args.n_samples} images in {time.perf_counter() - t0:.1f}s)")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
