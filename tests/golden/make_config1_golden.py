#!/usr/bin/env python3
"""Config 1 fixture (BASELINE.json configs[0]): the REFERENCE's CPU `scripts/train_vae.py` run
`--data-path "" --n-samples 5000 --batch-size 128 --epochs 1` (z_dim 32, CondVAE, cond_drop 0,
lr 2e-3, beta 3e-4, free bits 0.05, seed 0), with its random draws recorded.

Run ONLY in the build container (the reference is not on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 PYTHONPATH=/root/reference/src:/root/reference \
        python tests/golden/make_config1_golden.py

The training loop below is the reference script's loop (/root/reference/scripts/train_vae.py:245-321)
driving the reference's own modules and `kl_stats` (imported from the script file): in-memory
ToyCrystalsDataset(5000, 64, seed 0), DataLoader(shuffle=True, drop_last=True) on torch's global
generator, CondVAE + torch.optim.Adam.  Two hooks RECORD (not alter) the draws: the dataset logs
the item order the DataLoader asks for, and CondVAE.reparameterise stores its `torch.randn_like`
eps (vae.py:57-60; cond_drop 0 draws no keep mask).  Stored (data only, .npz):
  order [39*128] int32       the DataLoader's item order of the epoch
  eps [39,128,32] f32        the reparameterisation draws of each step
  steps [39,4] f64           per-step loss, recon, kl_used, kl_raw (float(x.item()) as the script logs)
  epoch [4] f64              the epoch averages the script prints
  ck/<param> [3] f64         sum, |sum|, numel of every final parameter
  pick/<param> [64] f32 + idx/<param> [64] int64: 64 sampled final entries per parameter
"""
from __future__ import annotations

import importlib.util
import os
import time

import numpy as np
import torch
from torch.utils.data import DataLoader

from toycrystals.data import ToyCrystalsDataset  # reference
from toycrystals.models import vae as ref_vae  # reference

HERE = os.path.dirname(os.path.abspath(__file__))
REF_SCRIPT = "/root/reference/scripts/train_vae.py"


def main() -> None:
    spec = importlib.util.spec_from_file_location("ref_train_vae", REF_SCRIPT)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)  # defines kl_stats; main() is behind __name__ == "__main__"
    kl_stats = mod.kl_stats

    seed, n_samples, img_size, B, z_dim, lr, beta, free_bits = 0, 5000, 64, 128, 32, 2e-3, 3e-4, 0.05
    torch.manual_seed(seed)
    ds = ToyCrystalsDataset(n_samples=n_samples, img_size=img_size, seed=seed)
    order = []
    get = ds.__getitem__

    class Logged(torch.utils.data.Dataset):
        def __len__(self):
            return len(ds)

        def __getitem__(self, i):
            order.append(int(i))
            return get(i)

    dl = DataLoader(Logged(), batch_size=B, shuffle=True, num_workers=0, drop_last=True, pin_memory=False)
    model = ref_vae.CondVAE(z_dim=z_dim, n_types=4, y_cont_dim=4, cond_drop=0.0)
    eps_log = []
    orig = ref_vae.CondVAE.reparameterise

    def reparameterise(self, mu, logvar):
        std = torch.exp(0.5 * logvar)
        eps = torch.randn_like(std)
        eps_log.append(eps.detach().clone())
        return mu + eps * std

    ref_vae.CondVAE.reparameterise = reparameterise
    opt = torch.optim.Adam(model.parameters(), lr=lr)
    steps = []
    epoch = 0
    model.train()
    t0 = time.time()
    for x, y_cat, y_cont in dl:
        x_hat, mu, logvar = model(x, y_cat, y_cont)
        recon = torch.mean((x_hat - x) ** 2)
        kl_used, kl_raw = kl_stats(mu, logvar, free_bits=free_bits)
        b = beta * min(1.0, (epoch + 1) / 5.0)
        loss = recon + b * kl_used
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
        steps.append([float(loss.item()), float(recon.item()), float(kl_used.item()), float(kl_raw.item())])
        print(f"step {len(steps):2d}: loss {steps[-1][0]:.6f} recon {steps[-1][1]:.6f} kl {steps[-1][2]:.4f} "
              f"({time.time() - t0:.0f}s)", flush=True)
    ref_vae.CondVAE.reparameterise = orig
    steps = np.array(steps, dtype=np.float64)
    out = {"order": np.array(order, dtype=np.int32), "eps": torch.stack(eps_log).numpy().astype(np.float32),
           "steps": steps, "epoch": steps.mean(axis=0),
           "cfg": np.array([seed, n_samples, img_size, B, z_dim, lr, beta, free_bits], dtype=np.float64)}
    g = np.random.default_rng(0)
    for k, v in model.state_dict().items():
        a = v.detach().double().numpy().ravel()
        out["ck/" + k] = np.array([a.sum(), np.abs(a).sum(), float(a.size)])
        idx = np.sort(g.choice(a.size, size=min(64, a.size), replace=False)).astype(np.int64)
        out["idx/" + k] = idx
        out["pick/" + k] = a[idx].astype(np.float32)
    assert len(order) == len(steps) * B and len(eps_log) == len(steps)
    path = os.path.join(HERE, "config1_vae_5k_b128.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path}: {len(steps)} steps, epoch avg loss {out['epoch'][0]:.6f}")


if __name__ == "__main__":
    main()
