"""GPU: the one-channel convolutions (csrc/thin.hip, round 6) that tcx_conv2d / tcx_conv_wgrad route the
score net's first conv (1 -> 96, sde_score_model.py:246), its out conv (96 -> 1, :264) and their
gradients to, against the numpy oracle (oracle/nn_np.py, fp64) and a float64 im2col weight gradient.

These are fp32 VALU reductions (no split products): the gate is 2e-5 of the output scale for the
forwards (test_gpu_ops' conv gate) and 2^-16 of sum |x||dY| per weight (+1e-6 of the largest) for the
weight gradients, whose fp32 sums run sequentially over a few hundred pixels per thread (n u ~ 2^-16 for
n = 256 terms at u = 2^-24), then over the streams and the split planes in a fixed order."""
import numpy as np
import pytest
import torch

from oracle import nn_np
from test_gpu_ops import L, chk, close, dev, run_conv, st
from test_gpu_wgrad import im2col

pytestmark = pytest.mark.gpu

rng = np.random.default_rng(23)


@pytest.mark.parametrize("B,Co,H,W,circ,act,bb", [
    (2, 96, 64, 64, True, 0, True),    # the first conv (per-batch bias of the folded maps)
    (2, 96, 64, 64, True, 0, False),   # the out conv's data gradient (no bias)
    (3, 32, 17, 9, False, 3, True),    # zero padding, ragged, SiLU
    (1, 4, 5, 6, True, 1, False),
])
def test_thin_cin1_forward(B, Co, H, W, circ, act, bb):
    x = rng.standard_normal((B, 1, H, W))
    w = rng.standard_normal((Co, 1, 3, 3))
    b = rng.standard_normal(Co)
    bias_b = rng.standard_normal((B, Co)) if bb else None
    ref = nn_np.conv2d(x, w, b, padding=1, mode="circular" if circ else "zeros")
    if bb:
        ref = ref + bias_b[:, :, None, None]
    ref = [ref, np.maximum(ref, 0), 1 / (1 + np.exp(-ref)), ref / (1 + np.exp(-ref))][act]
    close(run_conv(x, w, b, 1, 1, circ, act=act, bias_b=bias_b), ref)


@pytest.mark.parametrize("B,Ci,H,W,circ,act,res", [
    (2, 96, 64, 64, True, 0, False),   # the out conv
    (2, 32, 64, 64, False, 0, True),   # the VAE decoder's last conv shape (zero padding), residual
    (3, 16, 7, 11, True, 2, False),    # ragged, sigmoid
    (1, 48, 9, 5, False, 3, True),
])
def test_thin_cout1_forward(B, Ci, H, W, circ, act, res):
    x = rng.standard_normal((B, Ci, H, W))
    w = rng.standard_normal((1, Ci, 3, 3)) / np.sqrt(9 * Ci)
    b = rng.standard_normal(1)
    r = rng.standard_normal((B, 1, H, W)) if res else None
    ref = nn_np.conv2d(x, w, b, padding=1, mode="circular" if circ else "zeros")
    if res:
        ref = ref + r
    ref = [ref, np.maximum(ref, 0), 1 / (1 + np.exp(-ref)), ref / (1 + np.exp(-ref))][act]
    close(run_conv(x, w, b, 1, 1, circ, act=act, resid=r), ref)


@pytest.mark.parametrize("B,H,W,Cin,Cout,circ,beta", [
    (8, 64, 64, 96, 1, 1, 0.0),   # the out conv's weight gradient (B = 8 of the 128-image step)
    (8, 64, 64, 1, 96, 1, 0.0),   # the first conv's (x_t channel) weight gradient
    (3, 13, 10, 32, 1, 0, 1.0),   # zero padding, ragged rows, accumulate (beta = 1)
    (2, 9, 16, 1, 8, 0, 0.5),
])
def test_thin_wgrad_vs_float64(B, H, W, Cin, Cout, circ, beta):
    x = rng.standard_normal((B, H, W, Cin)).astype(np.float32)
    dy = (rng.standard_normal((B, H, W, Cout)) * 0.1).astype(np.float32)
    dw0 = rng.standard_normal((Cout, Cin, 3, 3)).astype(np.float32)
    nb = int(L().tcx_conv_wgrad_workspace(B, H, W, Cin, Cout, 3))
    ws = torch.empty(nb, dtype=torch.uint8, device="cuda")
    dw = dev(dw0)
    xd, dyd = dev(x), dev(dy)
    chk(L().tcx_conv_wgrad(xd.data_ptr(), None, B, H, W, Cin, 0, dyd.data_ptr(), Cout, 3, 1, 1, circ, beta,
                           dw.data_ptr(), ws.data_ptr(), nb, st()))
    got = dw.cpu().numpy()
    cols, _, _ = im2col(x.astype(np.float64), 3, 1, 1, circ)
    g = dy.astype(np.float64).reshape(-1, Cout)
    ref = (cols.T @ g).reshape(3, 3, Cin, Cout).transpose(3, 2, 0, 1) + beta * dw0
    mag = (np.abs(cols).T @ np.abs(g)).reshape(3, 3, Cin, Cout).transpose(3, 2, 0, 1) + abs(beta) * np.abs(dw0)
    err = np.abs(got - ref)
    bound = mag * 2.0 ** -16 + 1e-6 * float(mag.max())
    print(f"thin wgrad B={B} {H}x{W} Cin={Cin} Cout={Cout} circ={circ}: max err {float(err.max()):.3e}, "
          f"max err/bound {float((err / bound).max()):.3f}")
    assert np.all(err <= bound), float((err / bound).max())


def test_thin_wgrad_deterministic():
    """Fixed-order sums: two runs of the out conv's weight gradient are bit-identical."""
    B, H, W, C = 4, 64, 64, 96
    x = dev(rng.standard_normal((B, H, W, C)))
    dy = dev(rng.standard_normal((B, H, W, 1)))
    nb = int(L().tcx_conv_wgrad_workspace(B, H, W, C, 1, 3))
    ws = torch.empty(nb, dtype=torch.uint8, device="cuda")
    outs = []
    for _ in range(2):
        dw = torch.empty((1, C, 3, 3), device="cuda")
        chk(L().tcx_conv_wgrad(x.data_ptr(), None, B, H, W, C, 0, dy.data_ptr(), 1, 3, 1, 1, 1, 0.0, dw.data_ptr(),
                               ws.data_ptr(), nb, st()))
        outs.append(dw.cpu())
    assert torch.equal(outs[0], outs[1])
