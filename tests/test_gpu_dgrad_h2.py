"""GPU: the f16x3 transposed conv tcx_conv_transpose2x_h2 (csrc/conv.hip, round 6): the training step's
data gradient of the 4x4 / stride-2 circular downsamples ds1 / ds2 (the adjoint of sde_score_model.py's
nn.Conv2d(C, C, 4, 2, 1, padding_mode="circular")), on h2 records of dY and of the four phase weights,
against a float64 adjoint on the decoded records:

    dx[b, (2 oy - 1 + ky) mod H, (2 ox - 1 + kx) mod W, ci] += w[co][ci][ky][kx] dY[b, oy, ox, co]

Gate: 2^-19 of sum |w||dY| per element on f16-exact operands (the records hold them exactly, so what remains is
the K = 4 Cout fp32 accumulation's rounding), plus 1e-6 of the largest such sum; and agreement with the fp32
tcx_conv_transpose2x at the fp32 gate of test_gpu_ops (2e-5 of the output scale)."""
import numpy as np
import pytest
import torch

from test_gpu_h2 import from_h2, to_h2
from test_gpu_ops import L, chk, dev, rup, st

pytestmark = pytest.mark.gpu

rng = np.random.default_rng(31)


def adjoint64(dy, w, H, W):
    B, Ho, Wo, Co = dy.shape
    ci = w.shape[1]
    dx = np.zeros((B, H, W, ci))
    mag = np.zeros((B, H, W, ci))
    oy, ox = np.arange(Ho), np.arange(Wo)
    for ky in range(4):
        for kx in range(4):
            iy, ix = (2 * oy - 1 + ky) % H, (2 * ox - 1 + kx) % W
            c = dy @ w[:, :, ky, kx]
            m = np.abs(dy) @ np.abs(w[:, :, ky, kx])
            for a, yy in enumerate(iy):
                dx[:, yy, ix, :] += c[:, a]
                mag[:, yy, ix, :] += m[:, a]
    return dx, mag


@pytest.mark.parametrize("B,Hy,Co,Ci", [(2, 16, 192, 192), (2, 32, 96, 96), (1, 8, 64, 32)])
def test_convT2x_h2_vs_float64(B, Hy, Co, Ci):
    H = W = 2 * Hy
    # f16-exact operands: the records hold them exactly (lo = 0), so the gate measures the kernel alone
    dy = (rng.standard_normal((B, Hy, Hy, Co)) * 0.1).astype(np.float16).astype(np.float32)
    w = (rng.standard_normal((Co, Ci, 4, 4)) / np.sqrt(16 * Co)).astype(np.float16).astype(np.float32)
    kpad, cpad = 4 * Co, rup(Ci)
    wd = dev(w)
    wpk = torch.empty((4, cpad, kpad), device="cuda")
    chk(L().tcx_pack_convT_weight(wd.data_ptr(), wpk.data_ptr(), Co, Ci, cpad, kpad, st()))
    dyh, wh = to_h2(dev(dy)), to_h2(wpk)
    one = torch.ones(1, device="cuda")
    dx = torch.empty((B, H, W, Ci), device="cuda")
    chk(L().tcx_conv_transpose2x_h2(dyh.data_ptr(), B, Hy, Hy, Co, wh.data_ptr(), one.data_ptr(), None, dx.data_ptr(),
                                    Ci, cpad, kpad, 0, 1, st()))
    dx32 = torch.empty_like(dx)
    chk(L().tcx_conv_transpose2x(dev(dy).data_ptr(), B, Hy, Hy, Co, wpk.data_ptr(), None, dx32.data_ptr(), Ci, cpad,
                                 kpad, 0, 1, st()))
    torch.cuda.synchronize()
    got = dx.cpu().numpy().astype(np.float64)
    assert np.array_equal(from_h2(dyh).cpu().numpy(), dy)  # exact records
    ref, mag = adjoint64(dy.astype(np.float64), w.astype(np.float64), H, W)
    bound = mag * 2.0 ** -19 + 1e-6 * float(mag.max())
    err = np.abs(got - ref)
    print(f"convT2x_h2 B={B} {Hy}->{H} Co={Co} Ci={Ci}: max err {float(err.max()):.3e}, "
          f"max err/bound {float((err / bound).max()):.3f}")
    assert np.all(err <= bound), float((err / bound).max())
    scale = max(1.0, float(np.abs(dx32.cpu().numpy()).max()))
    assert float(np.abs(got - dx32.cpu().numpy()).max()) <= 2e-5 * scale
