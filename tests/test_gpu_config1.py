"""GPU: BASELINE.json configs[0] end to end at its stated size — `train_vae.py --data-path ""
--n-samples 5000 --batch-size 128 --epochs 1` (CondVAE z 32, lr 2e-3, free bits 0.05) — against the
REFERENCE's own CPU run (tests/golden/config1_vae_5k_b128.npz, made by make_config1_golden.py: the
reference script's loop and modules, its DataLoader order and reparameterisation draws recorded).

The mirror renders the 5,000 images on the GPU (uint8-exact vs the reference, float within 1 ulp),
replays the recorded item order and draws (`--replay-draws`), and logs every step; the 39 per-step
losses (recon + beta kl_used), recons, kl_used and kl_raw, the epoch averages and sampled final
parameters are compared.  /root/reference/scripts/train_vae.py:256-260,292-321.

Tolerance (stated): the two runs differ by fp32 rounding (GPU vs CPU reduction orders, the
renderer's 1-ulp pixels), and Adam (lr 2e-3) carries such differences forward over the 39 steps; the
per-step loss and recon are gated at 1e-4 relative (a 1e-4 loss change is ~1/100 of one step's
decrease; observed 1.6e-5 / 3.6e-6, r03_b), sampled final parameters within one Adam step (lr) of the
reference's: Adam moves an entry by up to lr per step whatever its gradient's size, so the ReLU
encoder's near-dead channels (gradients at rounding level) drift by a fraction of lr (observed
enc.4.bias 0.36 lr on the r03_i box, 1.8e-2 of that tensor's scale).  The KL terms are gated in absolute nats: with free bits 0.05 the
gradient of kl_used is zero for every latent dim below the threshold, so which dims sit above it is
decided by rounding-level differences late in the epoch (observed |d kl_used| 4e-3 of 1.6, |d kl_raw|
1.3e-2 of 0.7 at step 38 on the r03_b box; 1.66e-2 / 1.66e-2 on the r03_i box, where the loss still
agreed to 1.6e-5; beta * kl is 1 % of the loss): gates 5e-2 nats for both (3 % of kl_used)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCRIPTS = os.path.join(ROOT, "vae-diffusion-toy-crystals_amd", "scripts")


def test_config1_train_vae_5k_b128_vs_reference_cpu_run(tmp_path, golden):
    import torch
    g = golden("config1_vae_5k_b128")
    seed, n, img, B, z, lr, beta, fb = g["cfg"]
    cmd = [sys.executable, os.path.join(SCRIPTS, "train_vae.py"), "--data-path", "", "--n-samples", str(int(n)),
           "--img-size", str(int(img)), "--batch-size", str(int(B)), "--epochs", "1", "--z-dim", str(int(z)),
           "--lr", str(lr), "--beta", str(beta), "--free-bits", str(fb), "--seed", str(int(seed)),
           "--replay-draws", os.path.join(ROOT, "tests", "golden", "config1_vae_5k_b128.npz")]
    r = subprocess.run(cmd, cwd=tmp_path, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    rows = [json.loads(s) for s in open(tmp_path / "results" / "vae_steps.jsonl")]
    got = np.array([[q["loss"], q["recon"], q["kl_used"], q["kl_raw"]] for q in rows])
    ref = g["steps"]
    assert got.shape == ref.shape == (39, 4)
    rel = np.abs(got - ref) / np.abs(ref)
    for j, name in enumerate(("loss", "recon", "kl_used", "kl_raw")):
        print(f"{name}: max rel {rel[:, j].max():.3e} (step {int(rel[:, j].argmax()) + 1}), "
              f"first step {rel[0, j]:.3e}, last {rel[-1, j]:.3e}")
    print("step 1/20/39 loss mirror", got[[0, 19, 38], 0], "reference", ref[[0, 19, 38], 0])
    assert rel[:, 0].max() < 1e-4 and rel[:, 1].max() < 1e-4
    dkl = np.abs(got[:, 2:] - ref[:, 2:]).max(axis=0)
    print(f"kl_used max abs diff {dkl[0]:.3e} nats, kl_raw {dkl[1]:.3e} nats")
    assert dkl[0] < 5e-2 and dkl[1] < 5e-2
    sd = torch.load(tmp_path / "checkpoints" / "vae_last.pt", map_location="cpu", weights_only=True)
    worst = (0.0, "")
    for k, v in sd.items():
        a = v.double().numpy().ravel()
        pick = a[g["idx/" + k]]
        e = float(np.abs(pick - g["pick/" + k]).max()) / lr
        worst = max(worst, (e, k))
    print(f"final parameters (64 sampled entries per tensor): worst {worst[1]} differs by {worst[0]:.3e} lr")
    assert worst[0] < 1.0
