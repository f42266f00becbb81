#!/usr/bin/env python3
"""DDIM-50 of the w1024 x 8 prior (tools/train_bench.py bench_ddim's model and grid, seed 0) saved to argv[1]: the
A/B of a library variant compares the two samples bit for bit."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vae-diffusion-toy-crystals_amd"))
import numpy as np
import torch
from toycrystals_amd.models.diffusion_prior import DiffusionPriorFiLM, DiffusionSchedule

torch.manual_seed(0)
n = 36
m = DiffusionPriorFiLM(32, 4, 4, t_emb_dim=64, width=1024, n_blocks=8, y_cat_emb_dim=64).cuda().eval()
sched = DiffusionSchedule.linear(1000, 1e-4, 0.05, torch.device("cuda"))
y_cat = (torch.arange(n, device="cuda") % 4).to(torch.int64)
y_cont = torch.rand(n, 4, device="cuda")
torch.manual_seed(1)
with torch.no_grad():
    z = sched.ddim_sample(m, y_cat, y_cont, n_steps=50)
np.save(sys.argv[1], z.float().cpu().numpy())
print("saved", sys.argv[1], float(z.abs().max()))
