"""GPU: the non-default split-path conv variants stay parity-green.

The kernel variant is chosen once per process from the environment (csrc/conv3l.hip TCX_CONV3L,
csrc/conv3g.hip TCX_CONV3G; the measured-slower variants were removed in round 3), so each variant runs in ONE child process
(sequential, one GPU process at a time besides this one) that checks the 3x3 and 4x4/s2 U-Net
conv shapes against the fp64 numpy oracle at the fp32 gate (2e-5 of the output scale, as
test_gpu_h2.py).  The default variants are covered by test_gpu_h2.py in this process."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys
import numpy as np
sys.path[:0] = [ROOT, ROOT + "/tests", ROOT + "/vae-diffusion-toy-crystals_amd"]
from oracle import nn_np
from test_gpu_h2 import run_conv_h2
rng = np.random.default_rng(11)
worst = 0.0
for (B, Ci, Co, H, ks, s) in [(2, 96, 96, 64, 3, 1), (2, 192, 192, 32, 3, 1), (2, 192, 192, 16, 3, 1),
                              (2, 96, 96, 64, 4, 2), (2, 192, 192, 32, 4, 2)]:
    x = rng.standard_normal((B, Ci, H, H))
    w = rng.standard_normal((Co, Ci, ks, ks)) / np.sqrt(Ci * ks * ks)
    b = rng.standard_normal(Co)
    ref = nn_np.conv2d(x, w, b, stride=s, padding=1, mode="circular")
    got = run_conv_h2(x, w, b, s, 1, True)
    err = float(np.abs(got - ref).max()) / max(1.0, float(np.abs(ref).max()))
    worst = max(worst, err)
# GroupNorm+SiLU prologue (tcx_conv2d_h2_pro) at the 64^2, 32^2 and 16^2 shapes of the evaluator (only on
# the kernels that have one: not with TCX_CONV3G=0, where the evaluator falls back to apply passes)
import os
from test_gpu_h2 import run_conv_h2_pro, gn_silu_ref, rand_tabs
for (B, Ci, H) in ([(2, 96, 64), (2, 192, 32), (2, 192, 16)] if os.environ.get("TCX_CONV3G") != "0" else []):
    x = rng.standard_normal((B, Ci, H, H)) * 2.0
    w = rng.standard_normal((Ci, Ci, 3, 3)) / np.sqrt(Ci * 9)
    b = rng.standard_normal(Ci)
    tabs = rand_tabs(B, Ci, 3)
    ref = nn_np.conv2d(gn_silu_ref(x.astype(np.float32).astype(np.float64), tabs), w, b, padding=1, mode="circular")
    got = run_conv_h2_pro(x, w, b, True, tabs)
    err = float(np.abs(got - ref).max()) / max(1.0, float(np.abs(ref).max()))
    worst = max(worst, err)
print("worst", worst)
assert worst <= 2e-5, worst
""".replace("ROOT", repr(ROOT))


@pytest.mark.parametrize("env", [
    {"TCX_CONV3L": "0"},                          # k_conv3g (B fragments from global) at 32/64-px rows
    {"TCX_CONV3G": "0"},                          # k_conv3p (plain packed weights) on every 3x3 row width
])
def test_conv_variant_vs_oracle(env):
    e = dict(os.environ)
    e.update(env)
    r = subprocess.run([sys.executable, "-c", CHILD], env=e, cwd=ROOT, capture_output=True, text=True, timeout=150)
    print(r.stdout[-2000:], r.stderr[-2000:])
    assert r.returncode == 0, r.stderr[-2000:]
