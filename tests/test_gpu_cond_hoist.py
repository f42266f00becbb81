"""GPU: the sampler's hoisted conditioning changes no bit of its output.

TCX_COND_HOIST (default on): the sampler computes the time maps of its n_steps + 1 t values and the
condition maps of its rows once per call (k_cond_maps), folds them into a per-(step, image) first-conv
bias table (k_bias_table) and every evaluation's first conv reads its rows — instead of the
per-evaluation k_cond (timestep_embedding + time_mlp + ConditionEmbedding for every U-Net call, as the
reference does, sde_score_model.py:243-252).  Same arithmetic, so the images are bit-identical.

(A GroupNorm finalize folded into the producing conv's last workgroup per image was built and measured
in round 3 and removed: profiles/r03_h_*)

Each setting runs in its own child process (the knob is read once per process); the reverse SDE
(CFG and not, in-kernel Philox, 4 lanes and 1) and the PF-ODE outputs must be equal bit for bit."""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys, numpy as np, torch
sys.path.insert(0, sys.argv[1] + "/vae-diffusion-toy-crystals_amd")
from toycrystals_amd._lib import lib
from toycrystals_amd.models.sde_score_model import (CondUNetTiny, VPSDE, sample_reverse_sde_euler_maruyama,
                                                    sample_probability_flow_ode)
torch.manual_seed(0)
m = CondUNetTiny(4, 4, 96).cuda().eval()
sde = VPSDE(0.1, 30.0)
B = 6
yc = (torch.arange(B) % 4).cuda()
yv = torch.zeros(B, 4, device="cuda"); yv[:, 1] = torch.linspace(0, 1, B, device="cuda")
out = {}
for lanes in (1, 4):
    lib().tcx_set_sample_lanes(lanes)
    out[f"sde{lanes}"] = sample_reverse_sde_euler_maruyama(m, sde, yc, yv, (B, 1, 64, 64), n_steps=4, guidance_scale=1.5,
                                                           t_end=0.005, seed=5, return_x0_hat=True).cpu().numpy()
lib().tcx_set_sample_lanes(1)
out["ode"] = sample_probability_flow_ode(m, sde, yc, yv, (B, 1, 64, 64), n_steps=3, guidance_scale=1.5, t_end=0.005,
                                         seed=6, return_x0_hat=True).cpu().numpy()
out["sde_nocfg"] = sample_reverse_sde_euler_maruyama(m, sde, yc, yv, (B, 1, 64, 64), n_steps=3, guidance_scale=0.0,
                                                     t_end=0.005, seed=7, return_x0_hat=True).cpu().numpy()
np.savez(sys.argv[2], **out)
"""


def run(tmp_path, name, env_over):
    env = dict(os.environ)
    env.update(env_over)
    path = str(tmp_path / f"{name}.npz")
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT, path], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    return dict(np.load(path))


@pytest.mark.parametrize("prec", ["f16x3", "fp32"])
def test_cond_hoist_is_bit_identical(tmp_path, prec):
    old = run(tmp_path, "old", {"TCX_COND_HOIST": "0", "TCX_CONV_PRECISION": prec})
    new = run(tmp_path, "new", {"TCX_COND_HOIST": "1", "TCX_CONV_PRECISION": prec})
    for k in old:
        assert np.isfinite(old[k]).all()
        assert np.array_equal(old[k], new[k]), (k, float(np.abs(old[k] - new[k]).max()))
    assert np.array_equal(new["sde1"], new["sde4"])
