#!/usr/bin/env python3
"""Config 1 TEACHER-FORCED gradient fixture: where (if anywhere) the mirror's CondVAE backward departs
from the reference's, independent of how Adam carries rounding differences along the trajectory.

Run ONLY in the build container (the reference is not on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 PYTHONPATH=/root/reference/src:/root/reference \
        python tests/golden/make_config1_grads.py

It re-runs the reference loop of make_config1_golden.py (/root/reference/scripts/train_vae.py:292-321:
in-memory ToyCrystalsDataset(5000, 64, seed 0), DataLoader(shuffle, drop_last) on the global
generator, CondVAE(z 32, cond_drop 0) + Adam(lr 2e-3), beta 3e-4, free bits 0.05) — the same seed,
so the same item order and reparameterisation draws as config1_vae_5k_b128.npz (asserted) — and
at steps s in STEPS evaluates the reference's loss and gradients on a COPY of the model whose
parameters are a compact reconstruction of the reference's parameters before step s:

    P_s' = P_init + clip(round((P_s - P_init) / U), -127, 127) * U,   U = lr / 3

(P_init = torch.manual_seed(0); CondVAE(...), asserted equal to the loop's initial model; the int8
codes q_s are stored, so the test rebuilds P_s' bit for bit).  Both implementations then evaluate
the SAME parameters on the SAME batch and eps: their gradients may differ only by fp32 rounding.

Stored (data only, .npz):
  steps [S] int                       the teacher-forced steps (1-based, as the script logs them)
  init_ck/<p> [2] f64                 sum and |sum| of P_init (guards the mirror's seeded init)
  q<s>/<p> int8                       the reconstruction codes (s > 1)
  sc<s> [4] f64                       loss, recon, kl_used, kl_raw at P_s'
  mu<s>, lv<s> [128,32] f32           encoder outputs (full)
  xh<s>_idx [1024] int64, xh<s> f32   sampled x_hat entries
  gst<s>/<p> [3] f64                  gradient sum, sum of squares, max |g|
  gi<s>/<p> int64, gv<s>/<p> f32      gradient entries: all of a tensor <= 4096 entries, else 1024
                                      random + the 64 largest |g|
  act/<j>_idx, act/<j> f32, act/<j>_st [2] f64: step-1 encoder activations after ReLU j (NCHW
                                      flat index), 1024 sampled + sum, sum of squares
"""
from __future__ import annotations

import copy
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
STEPS = (1, 2, 10, 38)


def _entries(a: np.ndarray, g: np.random.Generator):
    if a.size <= 4096:
        return np.arange(a.size, dtype=np.int64)
    rnd = g.choice(a.size, size=1024, replace=False)
    top = np.argsort(-np.abs(a))[:64]
    return np.unique(np.concatenate([rnd, top])).astype(np.int64)


def main() -> None:
    spec = importlib.util.spec_from_file_location("ref_train_vae", REF_SCRIPT)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    kl_stats = mod.kl_stats

    seed, n_samples, img_size, B, z_dim, lr, beta, free_bits = 0, 5000, 64, 128, 32, 2e-3, 3e-4, 0.05
    U = lr / 3.0
    torch.manual_seed(seed)
    init = ref_vae.CondVAE(z_dim=z_dim, n_types=4, y_cont_dim=4, cond_drop=0.0).state_dict()
    init = {k: v.detach().clone() for k, v in init.items()}
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
    for k, v in model.state_dict().items():
        assert torch.equal(v, init[k]), f"loop model init != manual_seed({seed}); CondVAE(): {k}"
    eps_log = []
    forced = {"eps": None}
    orig = ref_vae.CondVAE.reparameterise

    def reparameterise(self, mu, logvar):
        std = torch.exp(0.5 * logvar)
        if forced["eps"] is not None:  # the teacher-forced copy replays the step's draw
            return mu + forced["eps"] * std
        eps = torch.randn_like(std)
        eps_log.append(eps.detach().clone())
        return mu + eps * std

    ref_vae.CondVAE.reparameterise = reparameterise
    opt = torch.optim.Adam(model.parameters(), lr=lr)
    out = {"steps": np.array(STEPS, dtype=np.int64), "unit": np.array([U])}
    for k, v in init.items():
        a = v.double().numpy()
        out["init_ck/" + k] = np.array([a.sum(), np.abs(a).sum()])
    g = np.random.default_rng(1)
    model.train()
    t0 = time.time()
    s = 0
    epoch = 0
    for x, y_cat, y_cont in dl:
        s += 1
        before = {k: v.detach().clone() for k, v in model.state_dict().items()} if s in STEPS else None
        x_hat, mu, logvar = model(x, y_cat, y_cont)
        recon = torch.mean((x_hat - x) ** 2)
        kl_used, kl_raw = kl_stats(mu, logvar, free_bits=free_bits)
        b = beta * min(1.0, (epoch + 1) / 5.0)
        loss = recon + b * kl_used
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
        if before is None:
            continue
        # ---- teacher-forced evaluation at P_s' on a copy (no global RNG is consumed)
        fm = copy.deepcopy(model)
        sd = {}
        for k, v in before.items():
            if s == 1:
                sd[k] = init[k].clone()
            else:
                q = torch.clamp(torch.round((v.double() - init[k].double()) / U), -127, 127).to(torch.int8)
                out[f"q{s}/{k}"] = q.numpy()
                sd[k] = (init[k].double() + q.double() * U).float()
        fm.load_state_dict(sd)
        fm.zero_grad(set_to_none=True)
        acts = []
        hooks = []
        if s == 1:
            for j in (1, 3, 5, 7):
                hooks.append(fm.enc[j].register_forward_hook(lambda m, i, o: acts.append(o.detach().clone())))
        forced["eps"] = eps_log[-1]
        fx_hat, fmu, flv = fm(x, y_cat, y_cont)
        forced["eps"] = None
        for h in hooks:
            h.remove()
        frec = torch.mean((fx_hat - x) ** 2)
        fku, fkr = kl_stats(fmu, flv, free_bits=free_bits)
        floss = frec + b * fku
        floss.backward()
        out[f"sc{s}"] = np.array([floss.item(), frec.item(), fku.item(), fkr.item()], dtype=np.float64)
        out[f"mu{s}"] = fmu.detach().numpy().astype(np.float32)
        out[f"lv{s}"] = flv.detach().numpy().astype(np.float32)
        xa = fx_hat.detach().numpy().ravel()
        xi = np.sort(g.choice(xa.size, size=1024, replace=False)).astype(np.int64)
        out[f"xh{s}_idx"], out[f"xh{s}"] = xi, xa[xi].astype(np.float32)
        for k, p in fm.named_parameters():
            a = p.grad.detach().double().numpy().ravel()
            out[f"gst{s}/{k}"] = np.array([a.sum(), (a * a).sum(), np.abs(a).max()])
            idx = _entries(a, g)
            out[f"gi{s}/{k}"], out[f"gv{s}/{k}"] = idx, a[idx].astype(np.float32)
        for j, a_t in enumerate(acts):
            a = a_t.double().numpy().ravel()
            ai = np.sort(g.choice(a.size, size=1024, replace=False)).astype(np.int64)
            out[f"act/{j}_idx"], out[f"act/{j}"] = ai, a[ai].astype(np.float32)
            out[f"act/{j}_st"] = np.array([a.sum(), (a * a).sum()])
        print(f"step {s:2d}: teacher-forced loss {floss.item():.6f} (trajectory {loss.item():.6f}) "
              f"kl_raw {fkr.item():.5f} ({time.time() - t0:.0f}s)", flush=True)
    ref_vae.CondVAE.reparameterise = orig
    # the same run as config1_vae_5k_b128.npz: same order and draws
    prev = np.load(os.path.join(HERE, "config1_vae_5k_b128.npz"), allow_pickle=False)
    assert np.array_equal(prev["order"], np.array(order, dtype=np.int32))
    assert np.array_equal(prev["eps"], torch.stack(eps_log).numpy().astype(np.float32))
    path = os.path.join(HERE, "config1_grads.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path} ({os.path.getsize(path) / 1e6:.2f} MB)")


if __name__ == "__main__":
    main()
