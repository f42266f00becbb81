#!/usr/bin/env python3
"""Golden fixtures for the toy-crystal renderer, made by importing the REFERENCE (build container only):

    PYTHONDONTWRITEBYTECODE=1 PYTHONPATH=/root/reference/src:/root/reference \
        python tests/golden/make_render_goldens.py

Reference call sites (file:line in /root/reference):
  ToyCrystalsDataset.__getitem__   src/toycrystals/data.py:171-221  (draws, render, normalise)
  _make_points                     src/toycrystals/data.py:73-129   (lattice, rotation, vacancy, jitter, crop)
  _render_gaussians                src/toycrystals/data.py:132-153
  build_dataset.py x_u8            scripts/build_dataset.py:31-36   ((x.clamp(0,1) * 255).to(uint8))

Stored per case: the (seed, idx, flags), the reference's atom centres (float32, exactly as
_make_points returns them), sigma, the float image, the uint8 image and (y_cat, y_cont).  Data only.
"""
from __future__ import annotations

import math
import os

import numpy as np
import torch

from toycrystals import data as ref_data

HERE = os.path.dirname(os.path.abspath(__file__))


def case(ds, idx):
    # re-run the reference's draw sequence to capture its point set as well
    g = torch.Generator()
    g.manual_seed(ds.seed + int(idx))
    H = W = ds.img_size
    lt = int(torch.randint(0, ds.n_types, (1,), generator=g).item())
    a = ref_data._uniform(g, 6.0, 14.0)
    theta = ref_data._uniform(g, 0.0, math.pi / 3.0)
    vac = ref_data._uniform(g, 0.0, 0.25)
    jit = ref_data._uniform(g, 0.0, 0.6)
    if ds.simple:
        a, theta, vac, jit = 10.0, 0.0, 0.0, 0.0
    if ds.rot_only:
        a, vac, jit = 10.0, 0.0, 0.0
    pts = ref_data._make_points(lattice_type=lt, a=a, H=H, W=W, theta=theta, vacancy=vac, jitter=jit, g=g)
    sigma = max(0.6, 0.12 * a)
    x, yc, yv = ds[idx]
    u8 = (x.clamp(0.0, 1.0) * 255.0).to(torch.uint8)
    return pts.numpy(), sigma, x.numpy(), u8.numpy(), int(yc), yv.numpy()


def main():
    out = {}
    cases = [(0, False, False, 64, list(range(0, 12))), (7, False, True, 64, list(range(0, 8))),
             (3, True, False, 64, [0, 1, 2, 3]), (11, False, False, 32, [0, 1, 2, 3, 4, 5])]
    k = 0
    for seed, simple, rot_only, size, idxs in cases:
        ds = ref_data.ToyCrystalsDataset(n_samples=1000, img_size=size, seed=seed, n_types=4, simple=simple,
                                         rot_only=rot_only)
        for idx in idxs:
            pts, sigma, x, u8, yc, yv = case(ds, idx)
            p = f"c{k}/"
            out[p + "meta"] = np.array([seed, idx, int(simple), int(rot_only), size], np.int64)
            out[p + "pts"] = pts.astype(np.float32)
            out[p + "sigma"] = np.array(sigma, np.float64)
            out[p + "x"] = x.astype(np.float32)
            out[p + "u8"] = u8
            out[p + "y_cat"] = np.array(yc, np.int64)
            out[p + "y_cont"] = yv.astype(np.float32)
            k += 1
    out["n_cases"] = np.array(k)
    np.savez_compressed(os.path.join(HERE, "render_ref.npz"), **out)
    print(f"wrote {k} cases")


if __name__ == "__main__":
    main()
