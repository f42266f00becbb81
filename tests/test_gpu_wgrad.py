"""GPU: the f16x3 conv weight gradient tcx_conv_wgrad_h2 (csrc/gemm.hip k_wgrad_h2: 16-B record
pieces staged into swizzled pixel-major LDS images, MFMA operands by ds_read_b64_tr_b16) against a
float64 im2col reference on the decoded h2 operands.

The weight gradient of the reference's convs (torch autograd of nn.Conv2d, sde_score_model.py:102,105,
208,210,218,222; vae.py's zero-padded convs): dW[co][ci][ky][kx] = sum over (b, oy, ox) of
dY[b, oy, ox, co] * x[b, oy*s - p + ky, ox*s - p + kx, ci] (circular wrap or zero padding).  The three
f16 products per fp32 product (hi*hi + hi*lo + lo*hi) drop lo*lo (< 2^-22 of each product), so the
stated gate is 2^-19 of sum |dY||x| per weight (the K-long fp32 accumulation's own rounding bound),
plus 1e-6 of the largest such sum."""
import numpy as np
import pytest
import torch

from test_gpu_h2 import from_h2, to_h2
from test_gpu_ops import L, chk, dev, st

pytestmark = pytest.mark.gpu

rng = np.random.default_rng(11)


def im2col(x, ks, stride, pad, circular):
    B, H, W, C = x.shape
    Ho, Wo = (H + 2 * pad - ks) // stride + 1, (W + 2 * pad - ks) // stride + 1
    cols = np.zeros((B, Ho, Wo, ks, ks, C))
    for ky in range(ks):
        for kx in range(ks):
            ys = np.arange(Ho) * stride - pad + ky
            xs = np.arange(Wo) * stride - pad + kx
            if circular:
                cols[:, :, :, ky, kx, :] = x[:, ys % H][:, :, xs % W]
            else:
                vy, vx = (ys >= 0) & (ys < H), (xs >= 0) & (xs < W)
                sub = x[:, np.clip(ys, 0, H - 1)][:, :, np.clip(xs, 0, W - 1)]
                cols[:, :, :, ky, kx, :] = sub * vy[None, :, None, None] * vx[None, None, :, None]
    return cols.reshape(B * Ho * Wo, ks * ks * C), Ho, Wo


@pytest.fixture(params=[1, 0], ids=["halo", "im2col"])
def wgrad_mode(request):
    """1: the halo-staged 3x3 kernel (wgrad3h.hip, round 6) where it applies (3x3 stride 1, W in {16, 32, 64},
    C1 % 32 == 0, Cout % 96 == 0), 0: k_wgrad_h2 everywhere (tcx_debug_wgrad3h)."""
    prev = L().tcx_debug_wgrad3h(request.param)
    yield request.param
    L().tcx_debug_wgrad3h(prev)


@pytest.mark.parametrize("B,H,W,C1,C2,Cout,ks,stride,circ", [
    (2, 16, 16, 32, 0, 96, 3, 1, 1),     # NT = 3, one k block
    (2, 16, 16, 96, 96, 96, 3, 1, 1),    # two sources (the skip concats), 14 k blocks
    (1, 10, 10, 16, 0, 64, 3, 1, 1),     # NT = 2, M = 100 (a ragged last 32-pixel chunk)
    (2, 16, 16, 32, 0, 32, 4, 2, 1),     # NT = 1, the 4x4 / stride-2 downsample
    (2, 8, 8, 64, 0, 192, 3, 1, 0),      # zero padding (VAE), two co blocks
    (1, 9, 7, 40, 0, 48, 3, 1, 1),       # K = 360 (ragged k block), Cout 48 in a 64-wide block
    (4, 64, 64, 96, 0, 96, 3, 1, 1),     # the score model's 64^2 layer shape
    (2, 32, 32, 64, 0, 192, 3, 1, 0),    # halo kernel: zero padding at 32^2, two co blocks
    (2, 32, 32, 192, 192, 96, 3, 1, 1),  # halo kernel: up2.net.0's concat at 32^2 (12 channel groups)
    (3, 64, 64, 96, 96, 96, 3, 1, 0),    # halo kernel: up1.net.0's concat at 64^2, zero padding
    (2, 16, 16, 192, 0, 192, 3, 1, 1),   # halo kernel: the mid convs at 16^2 (4-row chunks)
])
def test_wgrad_h2_vs_float64(B, H, W, C1, C2, Cout, ks, stride, circ, wgrad_mode):
    pad = 1
    x1 = rng.standard_normal((B, H, W, C1)).astype(np.float32)
    x2 = rng.standard_normal((B, H, W, C2)).astype(np.float32) if C2 else None
    Ho, Wo = (H + 2 * pad - ks) // stride + 1, (W + 2 * pad - ks) // stride + 1
    dy = (rng.standard_normal((B, Ho, Wo, Cout)) * 0.1).astype(np.float32)
    x1h, dyh = to_h2(dev(x1)), to_h2(dev(dy))
    x2h = to_h2(dev(x2)) if C2 else None
    comb = torch.ones(1, device="cuda")
    dw = torch.empty((Cout, C1 + C2, ks, ks), device="cuda")
    nb = int(L().tcx_conv_wgrad_workspace(B, Ho, Wo, C1 + C2, Cout, ks))
    ws = torch.empty(nb, dtype=torch.uint8, device="cuda")
    chk(L().tcx_conv_wgrad_h2(x1h.data_ptr(), x2h.data_ptr() if C2 else None, B, H, W, C1, C2, dyh.data_ptr(), Cout, ks,
                              stride, pad, circ, 0.0, comb.data_ptr(), dw.data_ptr(), ws.data_ptr(), nb, st()))
    got = dw.cpu().numpy()
    # reference on the decoded operands (what the records hold), float64
    xd = from_h2(x1h).cpu().numpy().astype(np.float64)
    if C2:
        xd = np.concatenate([xd, from_h2(x2h).cpu().numpy().astype(np.float64)], axis=3)
    dyd = from_h2(dyh).cpu().numpy().astype(np.float64).reshape(-1, Cout)
    cols, _, _ = im2col(xd, ks, stride, pad, circ)
    ref = (cols.T @ dyd).reshape(ks, ks, C1 + C2, Cout).transpose(3, 2, 0, 1)
    mag = (np.abs(cols).T @ np.abs(dyd)).reshape(ks, ks, C1 + C2, Cout).transpose(3, 2, 0, 1)
    err = np.abs(got - ref)
    bound = mag * 2.0 ** -19 + 1e-6 * float(mag.max())
    print(f"wgrad_h2[{wgrad_mode}] B={B} {H}x{W} C={C1}+{C2} Cout={Cout} k={ks} s={stride} circ={circ}: "
          f"max err {float(err.max()):.3e}, max err/bound {float((err / bound).max()):.3f}")
    assert np.all(err <= bound), float((err / bound).max())


def test_wgrad3h_deterministic_and_close_to_im2col():
    """The halo kernel is deterministic (fixed chunk order per split, fixed plane order in the reduce) and agrees
    with k_wgrad_h2 to the fp32 accumulation-order difference (both sum the same f16x3 products)."""
    B, H, W, C, Cout = 4, 64, 64, 96, 96
    x1h = to_h2(dev(rng.standard_normal((B, H, W, C)).astype(np.float32)))
    dyh = to_h2(dev((rng.standard_normal((B, H, W, Cout)) * 0.1).astype(np.float32)))
    comb = torch.ones(1, device="cuda")
    nb = int(L().tcx_conv_wgrad_workspace(B, H, W, C, Cout, 3))
    ws = torch.empty(nb, dtype=torch.uint8, device="cuda")
    outs = []
    for mode in (1, 1, 0):
        prev = L().tcx_debug_wgrad3h(mode)
        dw = torch.empty((Cout, C, 3, 3), device="cuda")
        chk(L().tcx_conv_wgrad_h2(x1h.data_ptr(), None, B, H, W, C, 0, dyh.data_ptr(), Cout, 3, 1, 1, 1, 0.0,
                                  comb.data_ptr(), dw.data_ptr(), ws.data_ptr(), nb, st()))
        L().tcx_debug_wgrad3h(prev)
        outs.append(dw.cpu())
    assert torch.equal(outs[0], outs[1])
    scale = float(outs[2].abs().max())
    assert float((outs[0] - outs[2]).abs().max()) <= 1e-5 * scale
