#!/usr/bin/env python3
"""Three prior training steps (tools/train_bench.py bench_prior's model, optimiser and batch, seed 0) and the
resulting parameters saved to argv[1] (.npz): the A/B of a library variant compares them bit for bit."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vae-diffusion-toy-crystals_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import numpy as np
import torch
os.environ.setdefault("STEPS", "3")
os.environ.setdefault("WARM", "0")
import train_bench

captured = {}
_orig_adam = train_bench.Adam


class CapAdam(_orig_adam):
    def __init__(self, params, *a, **k):
        params = list(params)
        captured["params"] = params
        super().__init__(params, *a, **k)


train_bench.Adam = CapAdam
print(train_bench.bench_prior())
np.savez(sys.argv[1], *[p.detach().float().cpu().numpy() for p in captured["params"]])
print("saved", sys.argv[1], len(captured["params"]))
