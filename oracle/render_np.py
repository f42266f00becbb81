"""TEST INFRASTRUCTURE ONLY (never imported by the product path): numpy restatement of the
toy-crystal Gaussian splatting, used as the checker of tcx_render_crystals.

Follows /root/reference/src/toycrystals/data.py:132-153 (_render_gaussians: dx = x - px,
dy = y - py in fp32, d2 = dx*dx + dy*dy with separate roundings, arg = -d2 / fp32(2 sigma^2),
exp, sum over atoms), :204-206 (img / (max + 1e-8), clamp to [0, 1]) and
scripts/build_dataset.py:34 ((x * 255).to(uint8): fp32 product, truncation).  The sum over atoms
is accumulated in float64 and rounded once (the reference's torch sum order is a blocked cascade;
any fp32 order differs from it by a few ulp).  Pinned against the reference's own images in
tests/golden/render_ref.npz (tests/test_render_cpu.py).
"""
from __future__ import annotations

import numpy as np


def render_gaussians(points_xy: np.ndarray, H: int, W: int, sigma: float) -> np.ndarray:
    f32 = np.float32
    if points_xy.size == 0:
        return np.zeros((H, W), f32)
    yy, xx = np.meshgrid(np.arange(H, dtype=f32), np.arange(W, dtype=f32), indexing="ij")
    P = points_xy.astype(f32)
    dx = (xx[None, :, :] - P[:, 0][:, None, None]).astype(f32)
    dy = (yy[None, :, :] - P[:, 1][:, None, None]).astype(f32)
    d2 = (dx * dx + dy * dy).astype(f32)
    arg = (-d2 / f32(2.0 * sigma * sigma)).astype(f32)
    return np.exp(arg.astype(np.float64)).sum(axis=0).astype(f32)


def normalise(img: np.ndarray) -> np.ndarray:
    f32 = np.float32
    return np.clip((img / (img.max() + f32(1e-8))).astype(f32), f32(0.0), f32(1.0))


def to_u8(x: np.ndarray) -> np.ndarray:
    return (np.clip(x, 0.0, 1.0).astype(np.float32) * np.float32(255.0)).astype(np.uint8)


def render_item(points_xy: np.ndarray, H: int, W: int, sigma: float):
    x = normalise(render_gaussians(points_xy, H, W, sigma))
    return x, to_u8(x)
