"""Procedural toy-crystal dataset (drop-in for /root/reference/src/toycrystals/data.py) with the
Gaussian splatting on the MI355X.

The reference renders each item on the CPU: per-item draws from a torch.Generator seeded with
seed + idx (:171-190), a lattice point set (_make_points :73-129: lattice vectors and basis
:21-70, rotation about the centre, vacancies, jitter, crop), then one isotropic Gaussian per
atom summed over an [N,H,W] tensor (_render_gaussians :132-153, ~14 ms per 64x64 image) and a
max-normalisation (:204-206).

Here the draws and the point sets stay on the host and reproduce the reference bit for bit: the
same generator calls in the same order and the same fp32 tensor operations, with the reference's
Python double loop over lattice indices (:96-103) replaced by one broadcast expression that
forms every point with the same two roundings (i*v1 + j*v2, then + basis[k]) in the same
(i, j, k) order.  The splatting, the per-image max, the normalisation and the uint8 quantisation
of scripts/build_dataset.py (:31-36) run in one HIP kernel over a whole batch of images
(tcx_render_crystals, csrc/render.hip).
"""
from __future__ import annotations

import math
from typing import List, Sequence, Tuple

import torch
from torch.utils.data import Dataset

from ._lib import check, lib, ptr, stream_ptr


def _uniform(g: torch.Generator, low: float, high: float) -> float:
    """data.py:10-12: one fp32 uniform draw, returned as a Python float."""
    return float((low + (high - low) * torch.rand((), generator=g)).item())


def _rotation_matrix(theta: float) -> torch.Tensor:
    c, s = math.cos(theta), math.sin(theta)
    return torch.tensor([[c, -s], [s, c]], dtype=torch.float32)


def _lattice_definition(lattice_type: int, a: float, g: torch.Generator):
    """data.py:21-70: lattice vectors v1, v2 and the basis (pixel units).  Type 1 draws its
    aspect ratio from g."""
    a = float(a)
    if lattice_type == 0:
        v1, v2, basis = [a, 0.0], [0.0, a], [[0.0, 0.0]]
    elif lattice_type == 1:
        b = a * _uniform(g, 0.75, 1.35)
        v1, v2, basis = [a, 0.0], [0.0, b], [[0.0, 0.0]]
    elif lattice_type == 2:
        v1, v2, basis = [a, 0.0], [0.5 * a, (math.sqrt(3) / 2.0) * a], [[0.0, 0.0]]
    elif lattice_type == 3:
        v1, v2 = [a, 0.0], [0.5 * a, (math.sqrt(3) / 2.0) * a]
        basis = [[0.0, 0.0], [0.5 * a, (math.sqrt(3) / 6.0) * a]]
    else:
        raise ValueError(f"Unknown lattice_type={lattice_type}")
    f = torch.float32
    return torch.tensor(v1, dtype=f), torch.tensor(v2, dtype=f), torch.tensor(basis, dtype=f)


def _make_points(lattice_type: int, a: float, H: int, W: int, theta: float, vacancy: float, jitter: float,
                 g: torch.Generator) -> torch.Tensor:
    """data.py:73-129 (same draws, same fp32 results; the index loops are one broadcast)."""
    v1, v2, basis = _lattice_definition(lattice_type, a, g)
    centre = torch.tensor([W / 2.0, H / 2.0], dtype=torch.float32)
    margin = 2.0 * a
    extent = max(H, W) + margin
    n1 = int(math.ceil(extent / float(v1.norm().item()))) + 2
    n2 = int(math.ceil(extent / float(v2.norm().item()))) + 2
    i = torch.arange(-n1, n1 + 1, dtype=torch.float32).view(-1, 1, 1, 1)
    j = torch.arange(-n2, n2 + 1, dtype=torch.float32).view(1, -1, 1, 1)
    P = ((i * v1 + j * v2) + basis.view(1, 1, -1, 2)).reshape(-1, 2)
    P = P + centre
    # (P - centre) @ R.T + centre (:108-110).  The reference's result depends on the host's sgemm
    # kernel; written out as that kernel computes it on the reference host where the goldens were
    # made (out_j = fma(y, R[j,1], x * R[j,0]): an fp32 product, then one fused multiply-add,
    # emulated exactly in float64), so the points are the same on every machine.
    R = _rotation_matrix(theta)
    Q = P - centre
    x, y = Q[:, 0], Q[:, 1]
    Rd = R.double()
    o0 = (y.double() * Rd[0, 1] + (x * R[0, 0]).double()).float()
    o1 = (y.double() * Rd[1, 1] + (x * R[1, 0]).double()).float()
    P = torch.stack([o0, o1], dim=1) + centre
    if vacancy > 0.0:
        keep = torch.rand((P.shape[0],), generator=g) > vacancy
        P = P[keep]
    if jitter > 0.0:
        P = P + torch.randn(P.shape, generator=g) * jitter
    x, y = P[:, 0], P[:, 1]
    keep = (x > -margin) & (x < W + margin) & (y > -margin) & (y < H + margin)
    return P[keep]


class ToyCrystalsDataset(Dataset):
    """data.py:156-221: item idx is generated from seed + idx; returns (x [1,H,W] f32 in [0,1],
    y_cat int64, y_cont [4] f32).  Item access renders one image on the GPU (`device`); use
    `render(indices)` for batches."""

    def __init__(self, n_samples: int = 50_000, img_size: int = 64, seed: int = 0, n_types: int = 4,
                 simple: bool = False, rot_only: bool = False, device="cuda") -> None:
        self.n_samples = int(n_samples)
        self.img_size = int(img_size)
        self.seed = int(seed)
        self.n_types = n_types
        self.simple = simple
        self.rot_only = rot_only
        self.device = torch.device(device)

    def __len__(self) -> int:
        return self.n_samples

    def params(self, idx: int) -> Tuple[torch.Tensor, float, int, torch.Tensor]:
        """(points [N,2], sigma, y_cat, y_cont) of item idx — the host half of :171-221."""
        g = torch.Generator()
        g.manual_seed(self.seed + int(idx))
        H = W = self.img_size
        lattice_type = int(torch.randint(0, self.n_types, (1,), generator=g).item())
        a = _uniform(g, 6.0, 14.0)
        theta = _uniform(g, 0.0, math.pi / 3.0)
        vacancy = _uniform(g, 0.0, 0.25)
        jitter = _uniform(g, 0.0, 0.6)
        if self.simple:
            a, theta, vacancy, jitter = 10.0, 0.0, 0.0, 0.0
        if self.rot_only:
            a, vacancy, jitter = 10.0, 0.0, 0.0
        pts = _make_points(lattice_type, a, H, W, theta, vacancy, jitter, g)
        sigma = max(0.6, 0.12 * a)
        if self.simple:
            y_cont = torch.zeros(4, dtype=torch.float32)
        elif self.rot_only:
            y_cont = torch.tensor([0.0, theta, 0.0, 0.0], dtype=torch.float32)
        else:
            y_cont = torch.tensor([a, theta, vacancy, jitter], dtype=torch.float32)
        return pts, sigma, lattice_type, y_cont

    def render(self, indices: Sequence[int], u8: bool = False):
        """Render a batch on the GPU: (x [B,1,H,W] f32 (or uint8 quantised as build_dataset.py),
        y_cat [B] int64, y_cont [B,4] f32), all on self.device."""
        items = [self.params(i) for i in indices]
        x = render_points([it[0] for it in items], [it[1] for it in items], self.img_size, self.img_size,
                          self.device, u8=u8)
        y_cat = torch.tensor([it[2] for it in items], dtype=torch.int64)
        y_cont = torch.stack([it[3] for it in items]) if items else torch.empty((0, 4))
        return x, y_cat.to(self.device), y_cont.to(self.device)

    def materialize(self, batch: int = 4096) -> "RenderedSet":
        """Render every item once, kept on self.device (the in-memory dataset of train_vae.py
        with --data-path '' (:259-260), batched by DeviceBatches instead of a DataLoader)."""
        xs, ycs, yvs = [], [], []
        for i0 in range(0, self.n_samples, batch):
            x, yc, yv = self.render(range(i0, min(self.n_samples, i0 + batch)))
            xs.append(x)
            ycs.append(yc)
            yvs.append(yv)
        return RenderedSet(torch.cat(xs), torch.cat(ycs), torch.cat(yvs))

    def __getitem__(self, idx: int):
        x, y_cat, y_cont = self.render([idx])
        return x[0].cpu(), y_cat[0].cpu(), y_cont[0].cpu()


class RenderedSet:
    """Device-resident float images + labels (x_f32 [N,1,H,W], y_cat [N], y_cont [N,4])."""

    def __init__(self, x_f32: torch.Tensor, y_cat: torch.Tensor, y_cont: torch.Tensor) -> None:
        self.x_f32, self.y_cat, self.y_cont = x_f32, y_cat, y_cont

    def __len__(self) -> int:
        return int(self.x_f32.shape[0])

    def __getitem__(self, idx: int):
        return self.x_f32[idx], self.y_cat[idx], self.y_cont[idx]


def render_points(points: List[torch.Tensor], sigmas: List[float], H: int, W: int, device, u8: bool = False):
    """Splat each image's atoms (exp(-|p - c|^2 / (2 sigma^2)) summed over atoms, :132-153),
    normalise by (max + 1e-8) and clamp (:204-206); optionally quantise to uint8 as
    build_dataset.py :34.  One tcx_render_crystals launch for the batch."""
    device = torch.device(device)
    n = len(points)
    counts = [int(p.shape[0]) for p in points]
    offs = torch.zeros(n + 1, dtype=torch.int32)
    if n:
        offs[1:] = torch.tensor(counts, dtype=torch.int64).cumsum(0).to(torch.int32)
    flat = torch.cat([p.reshape(-1, 2).to(torch.float32) for p in points]) if sum(counts) else torch.zeros((1, 2))
    # the reference divides the fp32 tensor by the Python double 2*sigma^2: an fp32 operand
    s2 = torch.tensor([2.0 * s * s for s in sigmas], dtype=torch.float32)
    flat_d, offs_d, s2_d = flat.to(device), offs.to(device), s2.to(device)
    out = torch.empty((n, 1, H, W), device=device, dtype=torch.uint8 if u8 else torch.float32)
    if n:
        check(lib().tcx_render_crystals(ptr(flat_d), ptr(offs_d), ptr(s2_d), n, H, W,
                                        None if u8 else ptr(out), ptr(out) if u8 else None, stream_ptr(device)),
              "tcx_render_crystals")
    return out
