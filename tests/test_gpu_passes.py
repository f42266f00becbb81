"""GPU: the round-5 forms of the U-Net evaluation's bandwidth passes against the forms they replace, one
process per setting (the library reads its knobs once): k_attn_prep (the attention block's input side in
one pass per image) against the four passes it replaces (TCX_ATTN_PREP=0), and the chunk-major skip
tensors (TCX_SKIP_CM) against the pixel-major in-place apply, on whole forwards."""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

CHILD = r"""
import sys, numpy as np, torch
sys.path[:0] = [sys.argv[1], sys.argv[1] + "/tests", sys.argv[1] + "/vae-diffusion-toy-crystals_amd"]
from toycrystals_amd import _lib
from test_gpu_models import cu, unet
prec, B, H = sys.argv[3], int(sys.argv[4]), int(sys.argv[5])
g = np.random.default_rng(11)
x = g.standard_normal((B, 1, H, H)).astype(np.float32)
t = g.uniform(0.05, 0.95, B).astype(np.float32)
y = (np.arange(B) % 4).astype(np.int64)
yc = g.uniform(-1, 1, (B, 4)).astype(np.float32)
m = unet(96)
_lib.set_conv_precision(prec)
with torch.no_grad():
    e = m(cu(x), cu(t), cu(y), cu(yc)).cpu().numpy()
np.save(sys.argv[2], e)
"""


def _forward(tmp_path, tag, env, prec, B, H):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    path = str(tmp_path / f"e_{tag}.npy")
    r = subprocess.run([sys.executable, "-c", CHILD, root, path, prec, str(B), str(H)], capture_output=True,
                       text=True, timeout=300, env=dict(os.environ, **env))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    return np.load(path)


@pytest.mark.parametrize("prec", ["f16x3", "bf16"])
def test_attention_input_pass_vs_four_passes(tmp_path, prec):
    """k_attn_prep (GN+SiLU in place, attn.norm statistics, tables and records in one pass per image) against
    the four-pass form: the residual values are the same fmaf + SiLU; the attn.norm statistics are the same
    fp64 sums in another order, so the tables can differ in the last fp32 bit — the forward agrees to
    2e-6 of its scale (f16x3; bf16 records: 2e-3, one bf16 rounding of a value one ulp apart can flip)."""
    a = _forward(tmp_path, "fused", {"TCX_ATTN_PREP": "1"}, prec, 64, 64)
    b = _forward(tmp_path, "four", {"TCX_ATTN_PREP": "0"}, prec, 64, 64)
    scale = max(1.0, float(np.abs(b).max()))
    d = float(np.abs(a - b).max()) / scale
    print(f"attention input pass vs four passes ({prec}): max {d:.2e} of scale")
    assert d <= (2e-6 if prec == "f16x3" else 2e-3)


@pytest.mark.parametrize("H", [64, 32])
def test_chunk_major_skips_bit_identical(tmp_path, H):
    """Skip tensors h1 / h2 written chunk-major by gn_apply_cm (the same fmaf + SiLU + record split as the
    in-place apply) and read by the downsample and the concat conv from their planes: the whole forward is
    bit-identical to TCX_SKIP_CM=0 (at 32^2 only h1 qualifies: h2's downsample output is 8 px wide)."""
    a = _forward(tmp_path, "cm", {"TCX_SKIP_CM": "3"}, "f16x3", 64, H)
    b = _forward(tmp_path, "pm", {"TCX_SKIP_CM": "0"}, "f16x3", 64, H)
    assert np.array_equal(a, b)


def test_conv3m_h2_output_form_bit_identical(tmp_path):
    """k_conv3m's PRO 3 form (h2 output, no activation: the us1 / us2 convs) against the generic epilogue
    (TCX_CONV3M_OH2=0): the same values, the same stores; the whole 64^2 forward is bit-identical."""
    a = _forward(tmp_path, "oh2", {"TCX_CONV3M_OH2": "1"}, "f16x3", 64, 64)
    b = _forward(tmp_path, "gen", {"TCX_CONV3M_OH2": "0"}, "f16x3", 64, 64)
    assert np.array_equal(a, b)


@pytest.mark.parametrize("prec", ["f16x3", "bf16"])
def test_quad_epilogue_static_output_form_bit_identical(tmp_path, prec):
    """The quad epilogue with its output form compiled in (fp32 / h2 records / 2-byte bf16: the
    downsamples, the 1x1 convs, k_conv3lb) against the run-time choice (TCX_EPI_STATIC=0): the whole
    forward is bit-identical."""
    a = _forward(tmp_path, "st", {"TCX_EPI_STATIC": "1"}, prec, 64, 64)
    b = _forward(tmp_path, "rt", {"TCX_EPI_STATIC": "0"}, prec, 64, 64)
    assert np.array_equal(a, b)
