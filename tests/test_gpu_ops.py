"""GPU: every libtcx primitive vs the numpy oracle ops (oracle/nn_np.py, fp64), called through
the C ABI.  Tolerances are stated per test: fp32 MFMA accumulation over K <= 3456 terms stays
within ~1e-6 of the fp64 result relative to sum|a*b|; gates are 2e-5 relative to the output
scale unless stated."""
import ctypes

import numpy as np
import pytest
import torch

from oracle import nn_np

pytestmark = pytest.mark.gpu


def L():
    from toycrystals_amd._lib import lib
    return lib()


def chk(rc):
    from toycrystals_amd._lib import check
    check(rc)


def st():
    return torch.cuda.current_stream().cuda_stream


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).cuda()


def nhwc(x):  # NCHW numpy -> NHWC
    return np.ascontiguousarray(x.transpose(0, 2, 3, 1))


def nchw(x):
    return np.ascontiguousarray(x.transpose(0, 3, 1, 2))


def rup(v, a=32):
    return (v + a - 1) // a * a


def pack(w):
    co, ci, ks, _ = w.shape
    kpad, cpad = rup(ks * ks * ci), rup(co)
    wd = dev(w)
    wpk = torch.empty((cpad, kpad), device="cuda")
    chk(L().tcx_pack_conv_weight(wd.data_ptr(), wpk.data_ptr(), co, ci, ks, cpad, kpad, st()))
    return wpk, cpad, kpad


def run_conv(x, w, b, stride, pad, circular, x2=None, ups=False, act=0, bias_b=None, resid=None, bmod=0, gn=False,
             Bt=None, pro1=None, pro2=None):
    """x, x2 NCHW numpy; returns NCHW numpy (and GN partials)."""
    B, C1, H, W = x.shape
    C2 = 0 if x2 is None else x2.shape[1]
    Bt = Bt or B
    co, ci, ks, _ = w.shape
    assert ci == C1 + C2
    wpk, cpad, kpad = pack(w)
    Hi, Wi = (2 * H, 2 * W) if ups else (H, W)
    Ho, Wo = (Hi + 2 * pad - ks) // stride + 1, (Wi + 2 * pad - ks) // stride + 1
    y = torch.empty((Bt, Ho, Wo, co), device="cuda")
    xd = dev(nhwc(x))
    x2d = dev(nhwc(x2)) if x2 is not None else None
    bd = dev(b) if b is not None else None
    bbd = dev(bias_b) if bias_b is not None else None
    rd = dev(nhwc(resid)) if resid is not None else None
    nsplit = -(-Ho * Wo // 128)
    gnd = torch.zeros((Bt, nsplit, co, 2), dtype=torch.float64, device="cuda") if gn else None
    p1 = [dev(a) for a in pro1] if pro1 is not None else [None, None]
    p2 = [dev(a) for a in pro2] if pro2 is not None else [None, None]
    pp = [t.data_ptr() if t is not None else None for t in p1 + p2]
    chk(L().tcx_conv2d(xd.data_ptr(), x2d.data_ptr() if x2d is not None else None, Bt, bmod, H, W, C1, C2,
                       wpk.data_ptr(), bd.data_ptr() if bd is not None else None,
                       bbd.data_ptr() if bbd is not None else None, rd.data_ptr() if rd is not None else None,
                       y.data_ptr(), co, cpad, kpad, ks, stride, pad, int(circular), int(ups), act,
                       gnd.data_ptr() if gnd is not None else None, *pp, st()))
    torch.cuda.synchronize()
    out = nchw(y.cpu().numpy())
    return (out, gnd.cpu().numpy()) if gn else out


def close(a, ref, rel=2e-5):
    scale = max(1.0, float(np.abs(ref).max()))
    err = float(np.abs(a - ref).max())
    assert err <= rel * scale, f"max err {err:.3e} > {rel * scale:.3e}"
    return err


rng = np.random.default_rng(0)


@pytest.mark.parametrize("B,Ci,Co,H,ks,stride", [
    (2, 96, 96, 64, 3, 1), (3, 96, 192, 32, 3, 1), (2, 192, 192, 16, 3, 1), (2, 96, 96, 64, 4, 2),
    (2, 192, 192, 32, 4, 2), (2, 16, 32, 16, 3, 1), (1, 8, 64, 8, 3, 1), (2, 192, 576, 16, 1, 1),
    (2, 36, 40, 12, 3, 1),  # K and Cout not multiples of 32, odd spatial size
])
def test_conv_circular(B, Ci, Co, H, ks, stride):
    x = rng.standard_normal((B, Ci, H, H))
    w = rng.standard_normal((Co, Ci, ks, ks)) / np.sqrt(Ci * ks * ks)
    b = rng.standard_normal(Co)
    pad = 0 if ks == 1 else 1
    ref = nn_np.conv2d(x, w, b, stride=stride, padding=pad, mode="circular")
    close(run_conv(x, w, b, stride, pad, True), ref)


def test_conv_concat_two_sources():
    x1 = rng.standard_normal((2, 96, 32, 32))
    x2 = rng.standard_normal((2, 64, 32, 32))
    w = rng.standard_normal((96, 160, 3, 3)) / 40
    b = rng.standard_normal(96)
    ref = nn_np.conv2d(np.concatenate([x1, x2], 1), w, b, padding=1, mode="circular")
    close(run_conv(x1, w, b, 1, 1, True, x2=x2), ref)


def test_conv_upsample_fused():
    x = rng.standard_normal((2, 32, 16, 16))
    w = rng.standard_normal((64, 32, 3, 3)) / 17
    b = rng.standard_normal(64)
    ref = nn_np.conv2d(nn_np.upsample_bilinear2x(x), w, b, padding=1, mode="circular")
    close(run_conv(x, w, b, 1, 1, True, ups=True), ref)


def test_conv_scalar_path_bias_b_bmod():
    """Cin=1 first conv: scalar im2col, per-batch bias, CFG batch aliasing (b reads b % bmod)."""
    x = rng.standard_normal((3, 1, 64, 64))
    w = rng.standard_normal((96, 1, 3, 3))
    bias_b = rng.standard_normal((6, 96))
    ref1 = nn_np.conv2d(x, w, None, padding=1, mode="circular")
    ref = np.concatenate([ref1, ref1], 0) + bias_b[:, :, None, None]
    close(run_conv(x, w, None, 1, 1, True, bias_b=bias_b, bmod=3, Bt=6), ref)


@pytest.mark.parametrize("act", [0, 1, 2, 3])
def test_conv_zero_pad_act_resid(act):
    x = rng.standard_normal((2, 32, 32, 32))
    w = rng.standard_normal((64, 32, 4, 4)) / 23
    b = rng.standard_normal(64)
    r = rng.standard_normal((2, 64, 16, 16))
    ref = nn_np.conv2d(x, w, b, stride=2, padding=1, mode="zeros") + r
    ref = [ref, np.maximum(ref, 0), 1 / (1 + np.exp(-ref)), ref / (1 + np.exp(-ref))][act]
    close(run_conv(x, w, b, 2, 1, False, act=act, resid=r), ref)


def test_conv_gn_partials_epilogue():
    x = rng.standard_normal((2, 96, 64, 64))
    w = rng.standard_normal((96, 96, 3, 3)) / 29
    b = rng.standard_normal(96)
    y, part = run_conv(x, w, b, 1, 1, True, gn=True)
    ref = nn_np.conv2d(x, w, b, padding=1, mode="circular")
    close(y, ref)
    s = part[..., 0].sum(1)
    q = part[..., 1].sum(1)
    np.testing.assert_allclose(s, ref.sum((2, 3)), rtol=1e-5, atol=1e-2)
    np.testing.assert_allclose(q, (ref ** 2).sum((2, 3)), rtol=1e-5)


def test_convT_phases():
    for cin, cout, act in [(256, 128, 1), (32, 1, 2), (64, 32, 0)]:
        x = rng.standard_normal((2, cin, 8, 8))
        w = rng.standard_normal((cin, cout, 4, 4)) / np.sqrt(cin * 4)
        b = rng.standard_normal(cout)
        ref = nn_np.conv_transpose2d(x, w, b)
        ref = [ref, np.maximum(ref, 0), 1 / (1 + np.exp(-ref))][act]
        kpad, cpad = rup(4 * cin), rup(cout)
        wd = dev(w)
        wpk = torch.empty((4, cpad, kpad), device="cuda")
        chk(L().tcx_pack_convT_weight(wd.data_ptr(), wpk.data_ptr(), cin, cout, cpad, kpad, st()))
        xd = dev(nhwc(x))
        y = torch.empty((2, 16, 16, cout), device="cuda")
        bd = dev(b)
        chk(L().tcx_convT2x(xd.data_ptr(), 2, 8, 8, cin, wpk.data_ptr(), bd.data_ptr(), y.data_ptr(), cout, cpad, kpad,
                            act, st()))
        close(nchw(y.cpu().numpy()), ref)


@pytest.mark.parametrize("C,H,groups,silu", [(96, 64, 8, 1), (192, 16, 8, 0), (16, 32, 8, 1), (12, 8, 4, 1)])
def test_groupnorm(C, H, groups, silu):
    x = rng.standard_normal((3, C, H, H)) * 2 + 0.7
    gm = rng.standard_normal(C)
    bt = rng.standard_normal(C)
    ref = nn_np.group_norm(x, groups, gm, bt)
    if silu:
        ref = nn_np.silu(ref)
    xd = dev(nhwc(x))
    HW = H * H
    ns = max(1, HW // 512)
    part = torch.empty((3, ns, C, 2), dtype=torch.float64, device="cuda")
    chk(L().tcx_gn_partials(xd.data_ptr(), 3, HW, C, ns, part.data_ptr(), st()))
    y = torch.empty_like(xd)
    gmd, btd = dev(gm), dev(bt)  # keep alive until the async kernel has run
    chk(L().tcx_gn_apply(xd.data_ptr(), y.data_ptr(), 3, HW, C, groups, part.data_ptr(), ns, gmd.data_ptr(),
                         btd.data_ptr(), 1e-5, silu, st()))
    torch.cuda.synchronize()
    close(nchw(y.cpu().numpy()), ref)


def test_upsample():
    x = rng.standard_normal((2, 24, 16, 16))
    xd = dev(nhwc(x))
    y = torch.empty((2, 32, 32, 24), device="cuda")
    chk(L().tcx_upsample2x(xd.data_ptr(), y.data_ptr(), 2, 16, 16, 24, None, None, st()))
    close(nchw(y.cpu().numpy()), nn_np.upsample_bilinear2x(x))


def test_upsample_with_gn_silu_prologue():
    x = rng.standard_normal((2, 24, 16, 16)) * 2 + 0.3
    sc = rng.standard_normal((2, 24))
    sh = rng.standard_normal((2, 24))
    ref = nn_np.upsample_bilinear2x(nn_np.silu(x * sc[:, :, None, None] + sh[:, :, None, None]))
    xd, scd, shd = dev(nhwc(x)), dev(sc), dev(sh)
    y = torch.empty((2, 32, 32, 24), device="cuda")
    chk(L().tcx_upsample2x(xd.data_ptr(), y.data_ptr(), 2, 16, 16, 24, scd.data_ptr(), shd.data_ptr(), st()))
    close(nchw(y.cpu().numpy()), ref)


@pytest.mark.parametrize("C1,C2,Co,H,ks,stride,which", [(96, 0, 96, 64, 3, 1, 1), (192, 192, 96, 32, 3, 1, 2),
                                                        (96, 96, 96, 64, 3, 1, 3), (96, 0, 96, 64, 4, 2, 1)])
def test_conv_fused_gn_silu_prologue(C1, C2, Co, H, ks, stride, which):
    """silu(x*scale[b,c] + shift[b,c]) applied to source 1 and/or 2 while staging (which: bit mask)."""
    B = 2
    x1 = rng.standard_normal((B, C1, H, H)) * 1.5 + 0.2
    x2 = rng.standard_normal((B, C2, H, H)) if C2 else None
    w = rng.standard_normal((Co, C1 + C2, ks, ks)) / np.sqrt((C1 + C2) * ks * ks)
    b = rng.standard_normal(Co)
    t1 = (rng.standard_normal((B, C1)), rng.standard_normal((B, C1))) if which & 1 else None
    t2 = (rng.standard_normal((B, C2)), rng.standard_normal((B, C2))) if (which & 2 and C2) else None
    s1 = nn_np.silu(x1 * t1[0][:, :, None, None] + t1[1][:, :, None, None]) if t1 else x1
    s2 = None if x2 is None else (nn_np.silu(x2 * t2[0][:, :, None, None] + t2[1][:, :, None, None]) if t2 else x2)
    xin = s1 if s2 is None else np.concatenate([s1, s2], 1)
    ref = nn_np.conv2d(xin, w, b, stride=stride, padding=1, mode="circular")
    close(run_conv(x1, w, b, stride, 1, True, x2=x2, pro1=t1, pro2=t2), ref, rel=5e-5)


def test_gn_finalize_tables():
    C, HW, groups = 96, 4096, 8
    x = rng.standard_normal((3, C, 64, 64)) * 2 + 0.7
    gm, bt = rng.standard_normal(C), rng.standard_normal(C)
    xd = dev(nhwc(x))
    part = torch.empty((3, 8, C, 2), dtype=torch.float64, device="cuda")
    chk(L().tcx_gn_partials(xd.data_ptr(), 3, HW, C, 8, part.data_ptr(), st()))
    sc = torch.empty((3, C), device="cuda")
    sh = torch.empty((3, C), device="cuda")
    gmd, btd = dev(gm), dev(bt)
    chk(L().tcx_gn_finalize(part.data_ptr(), 3, HW, C, groups, 8, gmd.data_ptr(), btd.data_ptr(), 1e-5,
                            sc.data_ptr(), sh.data_ptr(), st()))
    torch.cuda.synchronize()
    got = x * sc.cpu().numpy()[:, :, None, None] + sh.cpu().numpy()[:, :, None, None]
    close(got, nn_np.group_norm(x, groups, gm, bt))


@pytest.mark.parametrize("B,C,N,heads", [(2, 192, 256, 4), (3, 32, 256, 4), (2, 64, 64, 4),
                                          # N > 256: key-tiled online-softmax kernel (256x256 images)
                                          (1, 192, 4096, 4), (2, 64, 512, 4), (1, 128, 1024, 2), (1, 96, 768, 2)])
def test_attention(B, C, N, heads):
    qkv = rng.standard_normal((B, N, 3 * C))
    d = C // heads
    q = qkv[:, :, :C].reshape(B, N, heads, d).transpose(0, 2, 1, 3)
    k = qkv[:, :, C:2 * C].reshape(B, N, heads, d).transpose(0, 2, 1, 3)
    v = qkv[:, :, 2 * C:].reshape(B, N, heads, d).transpose(0, 2, 1, 3)
    ref = nn_np.sdpa(q, k, v).transpose(0, 2, 1, 3).reshape(B, N, C)
    qd = dev(qkv)
    o = torch.empty((B, N, C), device="cuda")
    chk(L().tcx_attention(qd.data_ptr(), o.data_ptr(), B, N, C, heads, st()))
    torch.cuda.synchronize()
    close(o.cpu().numpy(), ref)


@pytest.mark.parametrize("split", [False, True], ids=["plain", "ws"])
@pytest.mark.parametrize("M,K1,K2,N,act", [(256, 1024, 0, 4096, 3), (5, 64, 64, 1024, 0), (7, 4, 0, 64, 3),
                                            (300, 2048, 2048, 200, 1), (36, 1024, 0, 2048, 3),
                                            (36, 1024, 1024, 1024, 0), (36, 4096, 0, 1024, 2)])
def test_linear(M, K1, K2, N, act, split):
    """tcx_linear, and tcx_linear_ws (split-K over caller scratch for skinny batches: the DDIM
    sampler's 36-row linears; it falls back to tcx_linear where the tiles fill the chip)."""
    x1 = rng.standard_normal((M, K1))
    x2 = rng.standard_normal((M, K2)) if K2 else None
    w = rng.standard_normal((N, K1 + K2)) / np.sqrt(K1 + K2)
    b = rng.standard_normal(N)
    r = rng.standard_normal((M, N))
    xx = x1 if x2 is None else np.concatenate([x1, x2], 1)
    ref = nn_np.linear(xx, w, b) + r
    ref = [ref, np.maximum(ref, 0), 1 / (1 + np.exp(-ref)), nn_np.silu(ref)][act]
    wpk, npad, kpad = pack(w[:, :, None, None])
    y = torch.empty((M, N), device="cuda")
    x1d, rd, bd = dev(x1), dev(r), dev(b)
    x2d = dev(x2) if x2 is not None else None
    if split:
        nb = int(L().tcx_linear_workspace(M, N, K1, K2))
        if M == 36:
            assert nb > 0
        ws = torch.empty(max(nb, 1), dtype=torch.uint8, device="cuda")
        chk(L().tcx_linear_ws(x1d.data_ptr(), K1, x2d.data_ptr() if x2d is not None else None, K2, wpk.data_ptr(),
                              bd.data_ptr(), rd.data_ptr(), y.data_ptr(), M, N, npad, kpad, act, ws.data_ptr(), nb,
                              st()))
    else:
        chk(L().tcx_linear(x1d.data_ptr(), K1, x2d.data_ptr() if x2d is not None else None, K2, wpk.data_ptr(),
                           bd.data_ptr(), rd.data_ptr(), y.data_ptr(), M, N, npad, kpad, act, st()))
    torch.cuda.synchronize()
    close(y.cpu().numpy(), ref)


def test_layernorm_film():
    M, W = 6, 1024
    x = rng.standard_normal((M, W)) * 3 + 1
    lw, lb = rng.standard_normal(W), rng.standard_normal(W)
    gb = rng.standard_normal((M, 3 * W))
    ref = nn_np.layer_norm(x, lw, lb) * (1 + gb[:, :W]) + gb[:, W:2 * W]
    xd, y, gd = dev(x), torch.empty((M, W), device="cuda"), dev(gb)
    lwd, lbd = dev(lw), dev(lb)  # keep alive until the async kernel has run
    chk(L().tcx_layernorm_film(xd.data_ptr(), y.data_ptr(), M, W, lwd.data_ptr(), lbd.data_ptr(),
                               gd.data_ptr(), 3 * W, 1e-5, st()))
    torch.cuda.synchronize()
    close(y.cpu().numpy(), ref)


def test_philox_randn_moments():
    n = 1 << 22
    o = torch.empty(n, device="cuda")
    chk(L().tcx_randn(o.data_ptr(), n, 1234, 7, st()))
    a = o.double().cpu().numpy()
    assert abs(a.mean()) < 5e-3 and abs(a.var() - 1) < 5e-3
    assert abs((a ** 3).mean()) < 1e-2 and abs((a ** 4).mean() - 3) < 3e-2
    o2 = torch.empty(n, device="cuda")
    chk(L().tcx_randn(o2.data_ptr(), n, 1234, 7, st()))
    assert torch.equal(o, o2)  # counter-based: reproducible
    chk(L().tcx_randn(o2.data_ptr(), n, 1234, 8, st()))
    assert not torch.equal(o, o2)


def test_errors_are_reported():
    from toycrystals_amd._lib import TcxError, check
    rc = L().tcx_attention(None, None, 1, 1024, 192, 4, st())
    assert rc != 0
    with pytest.raises(TcxError, match="tcx_attention"):
        check(rc)
