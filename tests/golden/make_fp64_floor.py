#!/usr/bin/env python3
"""The fp64 trajectory of the metric's 300-step golden (tests/golden/sde96_trained_300.npz): the same
weights (trained96_ema.npz), conditions and draws, run through the torch-CPU restatement
(oracle/score_model_torch.py, bit-identical to the reference in fp32) in float64.  It measures the
reference's OWN fp32 rounding noise along the trajectory (fp32 reference vs fp64), the floor under
which no parity gate can discriminate.  ~11 min on 8 cores.

    python tests/golden/make_fp64_floor.py      # writes tests/golden/sde96_trained_300_fp64.npz
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vae-diffusion-toy-crystals_amd")]

from oracle.score_model_torch import TorchScoreUNet, sample_reverse_sde  # noqa: E402
from toycrystals_amd.models.sde_score_model import host_noise  # noqa: E402


def main():
    torch.set_num_threads(8)
    g = dict(np.load(os.path.join(HERE, "sde96_trained_300.npz")))
    sd = {k: torch.from_numpy(v) for k, v in np.load(os.path.join(HERE, "trained96_ema.npz")).items()}
    B, steps = int(g["B"]), int(g["steps"])
    noise = host_noise((B, 1, 64, 64), steps + 1, torch.Generator().manual_seed(int(g["noise_seed"])))
    o = TorchScoreUNet(sd, dtype=torch.float64)
    x0 = sample_reverse_sde(o, float(g["beta_min"]), float(g["beta_max"]), torch.from_numpy(g["y_cat"]),
                            torch.from_numpy(g["y_cont"]), (B, 1, 64, 64), steps, float(g["cfg"]),
                            float(g["t_end"]), return_x0_hat=True, noise=noise.double()).numpy()
    ref = g["x0_unclamped"]
    print("fp32 reference vs fp64: x0_hat rel", np.abs(x0 - ref).max() / max(1.0, np.abs(ref).max()))
    np.savez_compressed(os.path.join(HERE, "sde96_trained_300_fp64.npz"), x0_fp64=x0)


if __name__ == "__main__":
    main()
