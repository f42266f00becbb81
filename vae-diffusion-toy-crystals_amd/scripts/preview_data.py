#!/usr/bin/env python3
"""MI355X drop-in for scripts/preview_data.py (reference :1-35): a 6 x 6 grid of the first 36
procedural toy-crystal items (ToyCrystalsDataset(n_samples=10_000, img_size=64, seed=0,
n_types=4, simple=False)), titled by lattice type, saved to results/preview_toycrystals.png at
dpi 200.  The 36 images are rendered in ONE tcx_render_crystals launch (dataset.render) instead
of 36 per-item CPU renders; the items are bit-identical to the reference's (tests/test_render_cpu.py,
tests/test_gpu_render.py)."""
from __future__ import annotations

import os

import _common  # noqa: F401
import matplotlib

matplotlib.use("Agg")
import matplotlib.pyplot as plt  # noqa: E402

from toycrystals_amd.data import ToyCrystalsDataset  # noqa: E402


def main() -> int:
    os.makedirs("results", exist_ok=True)
    ds = ToyCrystalsDataset(n_samples=10_000, img_size=64, seed=0, n_types=4, simple=False)
    rows, cols = 6, 6
    x, y_cat, _ = ds.render(range(rows * cols))
    x, y_cat = x.cpu(), y_cat.cpu()
    fig, axes = plt.subplots(rows, cols, figsize=(6, 6))
    for i, ax in enumerate(axes.flat):
        ax.imshow(x[i, 0], cmap="gray", vmin=0.0, vmax=1.0)
        ax.set_title(f"type={int(y_cat[i].item())}", fontsize=8)
        ax.axis("off")
    fig.tight_layout()
    out_path = "results/preview_toycrystals.png"
    fig.savefig(out_path, dpi=200)
    plt.close(fig)
    print(f"Saved {out_path}")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
