#!/usr/bin/env python3
"""Dataset-renderer throughput: host draws + point sets (toycrystals_amd.data) and the HIP splat
(tcx_render_crystals) for a batch of items, timed separately.  usage: render_bench.py [N] [rot_only]"""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "vae-diffusion-toy-crystals_amd"))
import torch
from toycrystals_amd.data import ToyCrystalsDataset, render_points

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
rot = len(sys.argv) > 2 and sys.argv[2] == "1"
ds = ToyCrystalsDataset(50_000, 64, 0, 4, False, rot)
ds.render(range(64), u8=True)
torch.cuda.synchronize()
t0 = time.perf_counter()
items = [ds.params(i) for i in range(n)]
t1 = time.perf_counter()
pts, sig = [it[0] for it in items], [it[1] for it in items]
render_points(pts, sig, 64, 64, "cuda", u8=True)
torch.cuda.synchronize()
t2 = time.perf_counter()
for _ in range(3):
    render_points(pts, sig, 64, 64, "cuda", u8=True)
torch.cuda.synchronize()
t3 = time.perf_counter()
natoms = sum(int(p.shape[0]) for p in pts)
print(f"{n} images (rot_only={rot}), {natoms / n:.0f} atoms/image: host draws+points {1e3 * (t1 - t0) / n:.3f} ms/img, "
      f"GPU render (incl. H2D) {1e6 * (t3 - t2) / 3 / n:.2f} us/img -> {n * 3 / (t3 - t2):.0f} img/s render-only")
