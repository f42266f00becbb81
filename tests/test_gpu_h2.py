"""GPU: the f16x3 split path (h2 storage, csrc/h2.hpp) through the C ABI.

Every h2 conv is checked against the fp64 numpy oracle conv (oracle/nn_np.py) at the SAME gate
as the fp32-MFMA conv in test_gpu_ops.py (2e-5 of the output scale), and its error is also
required to stay within 2x the fp32-MFMA conv's error on the same inputs + 2e-7 of the scale
(fp32-grade, not merely "within tolerance").  h2 writers are checked by decoding (hi + lo) against
the fp32 value: |v - dec(v)| <= 2^-21 |v| + 2^-25 (f16 subnormal spacing / 2)."""
import numpy as np
import pytest
import torch

from oracle import nn_np

from test_gpu_ops import L, chk, close, dev, nchw, nhwc, pack, run_conv, rup, st

pytestmark = pytest.mark.gpu

rng = np.random.default_rng(7)


def to_h2(t, ovf=None):
    y = torch.empty_like(t)
    chk(L().tcx_f32_to_h2(t.data_ptr(), y.data_ptr(), t.numel(), ovf.data_ptr() if ovf is not None else None, st()))
    return y


def from_h2(t):
    y = torch.empty_like(t)
    chk(L().tcx_h2_to_f32(t.data_ptr(), y.data_ptr(), t.numel(), st()))
    return y


def dec_ok(dec, v, fp32_ulps=0):
    """fp32_ulps: allowance for a reference computed by a different fp32 kernel (FMA contraction)."""
    bound = np.abs(v) * (2.0 ** -21 + fp32_ulps * 2.0 ** -23) + 2.0 ** -25
    assert np.all(np.abs(dec - v) <= bound), float(np.max(np.abs(dec - v) - bound))


def test_h2_roundtrip_and_range_flag():
    v = np.concatenate([rng.standard_normal(4096) * 10.0 ** rng.uniform(-8, 4, 4096), [0.0, -0.0, 65503.0, -1e-30]])
    v = np.resize(v, 4104).astype(np.float32)
    t = dev(v)
    ovf = torch.zeros(1, dtype=torch.int32, device="cuda")
    d = from_h2(to_h2(t, ovf)).cpu().numpy()
    dec_ok(d, v)
    assert int(ovf.item()) == 0
    big = t.clone()
    big[5] = 70000.0
    to_h2(big, ovf)
    assert int(ovf.item()) == 1


def pack_h2(w):
    wpk, cpad, kpad = pack(w)
    wh = torch.empty_like(wpk)
    ws = torch.empty(4, device="cuda")
    chk(L().tcx_pack_conv_weight_h2(wpk.data_ptr(), wh.data_ptr(), ws.data_ptr(), cpad, kpad, st()))
    return wh, ws, cpad, kpad


def pack_frag(wh, cpad, kpad, cin):
    """Fragment-ordered copy for k_conv3g / k_conv3l* (3x3) or k_conv4s2g (4x4/s2); None where it does
    not apply (the call then runs k_conv3p / k_conv4s2h / the im2col kernel)."""
    if kpad == 9 * cin:
        nb, fn = int(L().tcx_conv_weight_h2_frag_bytes(cpad, cin)), L().tcx_pack_conv_weight_h2_frag
    elif kpad == 16 * cin:
        nb, fn = int(L().tcx_conv_weight_h2_frag4_bytes(cpad, cin)), L().tcx_pack_conv_weight_h2_frag4
    else:
        return None
    if not nb:
        return None
    wf = torch.empty(nb // 4, device="cuda")
    chk(fn(wh.data_ptr(), wf.data_ptr(), cpad, kpad, cin, st()))
    return wf


def run_conv_h2(x, w, b, stride, pad, circular, x2=None, act=0, resid=None, bmod=0, gn=False, Bt=None, out_h2=False,
                frag=True):
    """frag=True passes the fragment-ordered weights (3x3 convs k_conv3g covers run on it; the rest,
    and frag=False, on k_conv3p / k_conv4s2h / the im2col kernel)."""
    B, C1, H, W = x.shape
    C2 = 0 if x2 is None else x2.shape[1]
    Bt = Bt or B
    co, ci, ks, _ = w.shape
    wh, ws, cpad, kpad = pack_h2(w)
    Ho, Wo = (H + 2 * pad - ks) // stride + 1, (W + 2 * pad - ks) // stride + 1
    y = torch.empty((Bt, Ho, Wo, co), device="cuda")
    xd = to_h2(dev(nhwc(x)))
    x2d = to_h2(dev(nhwc(x2))) if x2 is not None else None
    bd = dev(b) if b is not None else None
    rd = dev(nhwc(resid)) if resid is not None else None
    gnd = torch.zeros((Bt, -(-Ho * Wo // 128), co, 2), dtype=torch.float64, device="cuda") if gn else None
    ovf = torch.zeros(1, dtype=torch.int32, device="cuda")
    wf = pack_frag(wh, cpad, kpad, C1 + C2) if (frag and ks in (3, 4)) else None
    chk(L().tcx_conv2d_h2_pro(xd.data_ptr(), x2d.data_ptr() if x2d is not None else None, Bt, bmod, H, W, C1, C2,
                              wh.data_ptr(), wf.data_ptr() if wf is not None else None, ws.data_ptr(),
                              bd.data_ptr() if bd is not None else None, None,
                              rd.data_ptr() if rd is not None else None, y.data_ptr(), int(out_h2), co, cpad, kpad, ks,
                              stride, pad, int(circular), act, gnd.data_ptr() if gnd is not None else None,
                              None, None, None, None, 0, ovf.data_ptr(), st()))
    if out_h2:
        y = from_h2(y)
    torch.cuda.synchronize()
    assert int(ovf.item()) == 0
    out = nchw(y.cpu().numpy())
    return (out, gnd.cpu().numpy()) if gn else out


def fp32_grade(got, fp32, ref):
    scale = max(1.0, float(np.abs(ref).max()))
    e_h2 = float(np.abs(got - ref).max())
    e_32 = float(np.abs(fp32 - ref).max())
    print(f"h2 err {e_h2 / scale:.2e}  fp32-mfma err {e_32 / scale:.2e} (of scale {scale:.2f})")
    close(got, ref)
    assert e_h2 <= 2.0 * e_32 + 2e-7 * scale


@pytest.mark.parametrize("B,Ci,Co,H,ks,stride,circ", [
    (2, 96, 96, 64, 3, 1, True), (3, 96, 192, 32, 3, 1, True), (2, 192, 192, 16, 3, 1, True),
    (2, 96, 96, 64, 4, 2, True), (2, 192, 192, 32, 4, 2, True), (2, 192, 576, 16, 1, 1, True),
    (2, 64, 40, 12, 3, 1, True),  # Cout not a multiple of 32, odd spatial size
    (2, 32, 64, 16, 3, 1, False), (2, 64, 128, 16, 4, 2, False),  # zero padding
    # halo-staged 3x3 kernel (conv3h.hip: Cout % 96 == 0, W in {16, 32, 64})
    (2, 64, 96, 32, 3, 1, False), (1, 32, 192, 64, 3, 1, True), (3, 96, 96, 16, 3, 1, False),
    # halo-staged 4x4/s2 kernel (conv4s2h.hip: Cout % 96 == 0, Cin % 16 == 0, Wo in {16, 32, 64});
    # the two ds cases above (96 @ 64^2, 192 @ 32^2) also run on it
    (2, 32, 96, 64, 4, 2, True),    # two 16-channel slices (the fewest the C1 % 32 rule allows)
    (3, 64, 192, 32, 4, 2, False),  # zero padding, two column blocks
    (1, 32, 96, 128, 4, 2, True),   # Wo = 64 (the 256^2 config's ds2)
])
@pytest.mark.parametrize("frag", [True, False], ids=["conv3g", "conv3p"])
def test_conv_h2_vs_oracle(B, Ci, Co, H, ks, stride, circ, frag):
    """frag: with the fragment-ordered weights the covered 3x3 shapes run on k_conv3g, without
    them on k_conv3p (both kernels are live: k_conv3p serves 16x16 rows and the training path)."""
    x = rng.standard_normal((B, Ci, H, H))
    w = rng.standard_normal((Co, Ci, ks, ks)) / np.sqrt(Ci * ks * ks)
    b = rng.standard_normal(Co)
    pad = 0 if ks == 1 else 1
    ref = nn_np.conv2d(x, w, b, stride=stride, padding=pad, mode="circular" if circ else "zeros")
    fp32_grade(run_conv_h2(x, w, b, stride, pad, circ, frag=frag), run_conv(x, w, b, stride, pad, circ), ref)


def run_conv_h2_pro(x, w, b, circular, tabs, x2=None, tabs2=None, gn=False, out_h2=False, expect_ovf=0):
    """tcx_conv2d_h2_pro: a source with tables (sc, sh [B][C]) is passed as FP32 and normalised +
    SiLU'd + split in the conv's halo staging (k_conv3g); a source without tables is h2."""
    B, C1, H, W = x.shape
    C2 = 0 if x2 is None else x2.shape[1]
    co, ci, ks, _ = w.shape
    wh, ws, cpad, kpad = pack_h2(w)
    y = torch.empty((B, H, W, co), device="cuda")
    src = lambda t, tb: dev(nhwc(t)) if tb is not None else to_h2(dev(nhwc(t)))  # noqa: E731
    xd = src(x, tabs)
    x2d = src(x2, tabs2) if x2 is not None else None
    tb = [dev(t) for t in tabs] if tabs is not None else [None, None]
    tb2 = [dev(t) for t in tabs2] if tabs2 is not None else [None, None]
    p = lambda t: t.data_ptr() if t is not None else None  # noqa: E731
    gnd = torch.zeros((B, H * W // 128, co, 2), dtype=torch.float64, device="cuda") if gn else None
    ovf = torch.zeros(1, dtype=torch.int32, device="cuda")
    wf = pack_frag(wh, cpad, kpad, C1 + C2)
    chk(L().tcx_conv2d_h2_pro(xd.data_ptr(), p(x2d), B, 0, H, W, C1, C2, wh.data_ptr(), p(wf), ws.data_ptr(),
                              dev(b).data_ptr(), None, None, y.data_ptr(), int(out_h2), co, cpad, kpad, 3, 1, 1,
                              int(circular), 0, p(gnd), p(tb[0]), p(tb[1]), p(tb2[0]), p(tb2[1]), 0, ovf.data_ptr(),
                              st()))
    if out_h2:
        y = from_h2(y)
    torch.cuda.synchronize()
    assert int(ovf.item()) == expect_ovf
    out = nchw(y.cpu().numpy())
    return (out, gnd.cpu().numpy()) if gn else out


def gn_silu_ref(x, tabs):
    sc, sh = tabs
    v = x * sc[:, :, None, None] + sh[:, :, None, None]
    return v / (1.0 + np.exp(-v))


def rand_tabs(B, C, seed):
    g = np.random.default_rng(seed)
    return (g.uniform(0.5, 2.0, (B, C)).astype(np.float32), g.standard_normal((B, C)).astype(np.float32))


@pytest.mark.parametrize("B,Ci,Co,H,circ,two", [
    (2, 96, 96, 64, True, False),    # up1_1 / down1_1 (64^2)
    (2, 192, 192, 32, True, False),  # down2_1 (32^2)
    (2, 96, 96, 32, True, False),    # up2_1
    (2, 192, 192, 16, True, False),  # mid_1 (16^2 rows)
    (2, 32, 96, 64, True, False),    # one chunk pair (the 16x16x32 form's untransformed last even chunk)
    (1, 384, 96, 32, True, False),   # the widest source the prologue tables hold
    (1, 96, 96, 128, True, False),   # config 5's 128^2 rows
    (2, 64, 96, 32, False, False),   # zero padding: the padded ring is 0 AFTER the transform
    (2, 96, 96, 64, True, True),     # concat: source 1 h2, source 2 fp32 + tables
])
def test_conv_h2_gn_silu_prologue_vs_oracle(B, Ci, Co, H, circ, two):
    """The GroupNorm+SiLU prologue (k_conv3m's 16x16x32 form at 16/32/64-px rows, k_conv3g at 128,
    k_conv3l for the mixed concat): conv(silu(x*sc + sh)) against the fp64 oracle of the
    same (SiLU in fp64), at the fp32 gate and within 2x the fp32-MFMA conv of the pre-normalised
    input (the fp32 path applies the tables in a separate pass)."""
    x = rng.standard_normal((B, Ci, H, H)) * 2.0
    x2 = rng.standard_normal((B, Ci, H, H)) * 1.5 if two else None
    w = rng.standard_normal((Co, Ci * (2 if two else 1), 3, 3)) / np.sqrt(Ci * 9)
    b = rng.standard_normal(Co)
    tabs = rand_tabs(B, Ci, 3)
    mode = "circular" if circ else "zeros"
    if two:
        xin = np.concatenate([x, gn_silu_ref(x2.astype(np.float32).astype(np.float64), tabs)], 1)
        got = run_conv_h2_pro(x, w, b, circ, None, x2=x2, tabs2=tabs)
    else:
        xin = gn_silu_ref(x.astype(np.float32).astype(np.float64), tabs)
        got = run_conv_h2_pro(x, w, b, circ, tabs)
    ref = nn_np.conv2d(xin, w, b, padding=1, mode=mode)
    fp32 = run_conv(xin, w, b, 1, 1, circ)
    fp32_grade(got, fp32, ref)


def test_conv_h2_gn_prologue_gn_stats_and_range_flag():
    """Prologue + fused GroupNorm partials of the output; a normalised value past the f16 range
    raises the overflow flag (the evaluator then recomputes in fp32)."""
    x = rng.standard_normal((2, 96, 64, 64))
    w = rng.standard_normal((96, 96, 3, 3)) / 30
    b = rng.standard_normal(96)
    tabs = rand_tabs(2, 96, 5)
    ref = nn_np.conv2d(gn_silu_ref(x.astype(np.float32).astype(np.float64), tabs), w, b, padding=1, mode="circular")
    got, part = run_conv_h2_pro(x, w, b, True, tabs, gn=True)
    close(got, ref)
    s = part.sum(axis=1)
    r = ref.reshape(2, 96, -1)
    np.testing.assert_allclose(s[..., 0], r.sum(-1), rtol=1e-5, atol=1e-3)
    np.testing.assert_allclose(s[..., 1], (r * r).sum(-1), rtol=1e-5, atol=1e-3)
    big = x.copy()
    big[1, 7, 9, 11] = 1e5  # silu(1e5 * sc + sh) > 65504
    run_conv_h2_pro(big, w, b, True, tabs, expect_ovf=1)


def test_conv_h2_pro_rejects_uncovered_shape():
    """A prologue on a shape k_conv3g does not cover (8x8 rows) is an error, not a silent drop."""
    from toycrystals_amd._lib import TcxError
    x = rng.standard_normal((2, 96, 8, 8))
    w = rng.standard_normal((96, 96, 3, 3)) / 30
    with pytest.raises(TcxError, match="prologue"):
        run_conv_h2_pro(x, w, np.zeros(96), True, rand_tabs(2, 96, 1))


def test_conv_h2_concat_out_h2_gn_stats():
    """Two sources (the U-Net skip concat), h2 output, fused GroupNorm partials."""
    x1 = rng.standard_normal((2, 96, 32, 32))
    x2 = rng.standard_normal((2, 96, 32, 32)) * 3.0
    w = rng.standard_normal((96, 192, 3, 3)) / 40
    b = rng.standard_normal(96)
    ref = nn_np.conv2d(np.concatenate([x1, x2], 1), w, b, padding=1, mode="circular")
    got, part = run_conv_h2(x1, w, b, 1, 1, True, x2=x2, gn=True, out_h2=True)
    fp32 = run_conv(x1, w, b, 1, 1, True, x2=x2)
    fp32_grade(got, fp32, ref)
    s = part.sum(axis=1)  # [B][C][2]
    r = ref.reshape(2, 96, -1)
    np.testing.assert_allclose(s[..., 0], r.sum(-1), rtol=1e-5, atol=1e-3)
    np.testing.assert_allclose(s[..., 1], (r * r).sum(-1), rtol=1e-5, atol=1e-3)


def test_conv_h2_ds_halo_out_h2_gn_stats():
    """The 4x4/s2 halo kernel with h2 output and fused GroupNorm partials (ds1's shape at B = 2)."""
    x = rng.standard_normal((2, 96, 64, 64)) * 2.0
    w = rng.standard_normal((96, 96, 4, 4)) / 40
    b = rng.standard_normal(96)
    ref = nn_np.conv2d(x, w, b, stride=2, padding=1, mode="circular")
    got, part = run_conv_h2(x, w, b, 2, 1, True, gn=True, out_h2=True)
    fp32 = run_conv(x, w, b, 2, 1, True)
    fp32_grade(got, fp32, ref)
    s = part.sum(axis=1)
    r = ref.reshape(2, 96, -1)
    np.testing.assert_allclose(s[..., 0], r.sum(-1), rtol=1e-5, atol=1e-3)
    np.testing.assert_allclose(s[..., 1], (r * r).sum(-1), rtol=1e-5, atol=1e-3)


def test_conv_h2_halo_bmod_resid_act():
    """The halo kernel's CFG batch aliasing (bmod), residual and SiLU epilogue."""
    x = rng.standard_normal((2, 32, 32, 32))
    w = rng.standard_normal((96, 32, 3, 3)) / 17
    b = rng.standard_normal(96)
    resid = rng.standard_normal((4, 96, 32, 32))
    xx = np.concatenate([x, x], 0)
    ref = nn_np.conv2d(xx, w, b, padding=1, mode="circular") + resid
    ref = ref / (1 + np.exp(-ref))
    got = run_conv_h2(x, w, b, 1, 1, True, resid=resid, bmod=2, Bt=4, act=3)
    fp32 = run_conv(x, w, b, 1, 1, True, resid=resid, bmod=2, Bt=4, act=3)
    fp32_grade(got, fp32, ref)


def test_conv_h2_bmod_resid_act():
    """CFG batch aliasing (bmod), residual add and SiLU epilogue."""
    x = rng.standard_normal((2, 64, 16, 16))
    w = rng.standard_normal((64, 64, 3, 3)) / 24
    b = rng.standard_normal(64)
    resid = rng.standard_normal((4, 64, 16, 16))
    xx = np.concatenate([x, x], 0)
    ref = nn_np.conv2d(xx, w, b, padding=1, mode="circular") + resid
    ref = ref / (1 + np.exp(-ref))
    got = run_conv_h2(x, w, b, 1, 1, True, resid=resid, bmod=2, Bt=4, act=3)
    fp32 = run_conv(x, w, b, 1, 1, True, resid=resid, bmod=2, Bt=4, act=3)
    fp32_grade(got, fp32, ref)


def test_weight_scale_extremes():
    """Tiny and large weights: the power-of-two scale keeps lo halves normal either way."""
    x = rng.standard_normal((1, 32, 16, 16))
    for mag in (1e-7, 1e3):
        w = rng.standard_normal((32, 32, 3, 3)) * mag
        ref = nn_np.conv2d(x, w, None, padding=1, mode="circular")
        got = run_conv_h2(x, w, None, 1, 1, True)
        assert float(np.abs(got - ref).max()) <= 2e-6 * float(np.abs(ref).max())


@pytest.mark.parametrize("B,Ci,Co,H,resid,out_h2", [
    (2, 192, 192, 16, True, False),   # proj: residual, fp32 out (k_lin1x1)
    (2, 192, 576, 16, False, True),   # qkv: h2 out (k_lin1x1)
    (4, 96, 288, 8, False, False),    # 3 chunks (odd count), 3 column blocks
    (2, 192, 384, 16, True, True),    # two 192-column tiles (8-wave form), residual and h2 out
    (1, 32, 96, 16, False, True),     # one chunk
    (3, 64, 96, 8, True, False),      # M = 192, not whole 128-row tiles: im2col kernel
])
def test_conv1x1_h2_vs_oracle(B, Ci, Co, H, resid, out_h2):
    """1x1 split convs (csrc/lin1x1.hip where M % 128 == 0 and Cout pads to 96k) against the fp64
    oracle at the fp32 conv's gate, with bias, residual and h2 output as the attention block uses them."""
    x = rng.standard_normal((B, Ci, H, H))
    w = rng.standard_normal((Co, Ci, 1, 1)) / np.sqrt(Ci)
    b = rng.standard_normal(Co)
    r = rng.standard_normal((B, Co, H, H)) if resid else None
    ref = nn_np.conv2d(x, w, b, stride=1, padding=0, mode="zeros")
    if resid:
        ref = ref + r
    got = run_conv_h2(x, w, b, 1, 0, False, resid=r, out_h2=out_h2)
    err = float(np.abs(got - ref).max()) / max(1.0, float(np.abs(ref).max()))
    print(f"1x1 h2 err {err:.2e}")
    assert err <= (2e-5 if not out_h2 else 2e-5 + 2.0 ** -21)


@pytest.mark.parametrize("inplace", [True, False])
def test_gn_apply_h2(inplace):
    B, HW, C = 2, 256, 96
    x = rng.standard_normal((B, HW, C)).astype(np.float32)
    sc = dev(rng.standard_normal((B, C)))
    sh = dev(rng.standard_normal((B, C)))
    t = dev(x)
    out = t if inplace else torch.empty_like(t)
    ovf = torch.zeros(1, dtype=torch.int32, device="cuda")
    chk(L().tcx_gn_apply_tab_h2(t.data_ptr(), out.data_ptr(), B, HW, C, sc.data_ptr(), sh.data_ptr(), 1,
                                ovf.data_ptr(), st()))
    got = from_h2(out).cpu().numpy()
    ref32 = torch.empty_like(t)
    chk(L().tcx_gn_apply_tab(dev(x).data_ptr(), ref32.data_ptr(), B, HW, C, sc.data_ptr(), sh.data_ptr(), 1, st()))
    r = ref32.cpu().numpy()
    # the h2 apply computes SiLU on the hardware exp2 / rcp (as the conv prologues), the fp32 reference
    # pass with IEEE expf and division: the h2 decode bound plus 8 fp32 ulps
    bad = np.argwhere(np.abs(got - r) > np.abs(r) * (2.0 ** -21 + 8 * 2.0 ** -23) + 2.0 ** -25)
    if len(bad):
        print("mismatches", len(bad), bad[:8].tolist(), got[tuple(bad[0])], r[tuple(bad[0])])
    dec_ok(got, r, fp32_ulps=8)
    assert int(ovf.item()) == 0


@pytest.mark.parametrize("B,H,W,C", [(2, 8, 8, 96), (2, 16, 16, 192), (2, 32, 32, 96), (1, 12, 20, 32), (1, 6, 64, 64),
                                     (2, 16, 128, 96), (1, 8, 64, 192), (1, 6, 48, 96), (1, 5, 7, 8)])
def test_upsample_h2(B, H, W, C):
    """h2 upsample (the banded LDS kernel where H % 2 == 0 and W C <= 3072 — us1 / us2 of the 64^2
    U-Net —; the column-segmented band for wider rows — config 5's us1 / us2 at 256^2, 16 / 8 source
    columns per segment —; else k_upsample2x_g8) against the fp32 upsample: the h2 decode bound."""
    x = dev(rng.standard_normal((B, H, W, C)))
    y = torch.empty((B, 2 * H, 2 * W, C), device="cuda")
    y32 = torch.empty_like(y)
    chk(L().tcx_upsample2x_h2(x.data_ptr(), y.data_ptr(), B, H, W, C, None, None, None, st()))
    chk(L().tcx_upsample2x(x.data_ptr(), y32.data_ptr(), B, H, W, C, None, None, st()))
    dec_ok(from_h2(y).cpu().numpy(), y32.cpu().numpy())


@pytest.mark.parametrize("B,H,W,C", [(2, 32, 32, 96), (2, 16, 16, 192), (1, 6, 64, 64), (2, 16, 128, 96),
                                     (1, 8, 64, 192)])
def test_upsample_h2_fused_gn_silu(B, H, W, C):
    """The evaluator's us1 input: GroupNorm+SiLU tables applied by the upsample while it stages its
    source (no apply pass), against the in-place fp32 apply pass (IEEE-division SiLU) followed by the
    fp32 upsample: the h2 decode bound plus 8 fp32 ulps for the hardware exp2 / rcp SiLU, and 2^-21 of
    the output scale (an output interpolated between SiLU values of opposite sign carries their
    absolute, not its own relative, rounding)."""
    x = rng.standard_normal((B, H, W, C)).astype(np.float32) * 2.0
    sc = dev(rng.uniform(0.5, 1.5, (B, C)))
    sh = dev(rng.standard_normal((B, C)))
    ovf = torch.zeros(1, dtype=torch.int32, device="cuda")
    y = torch.empty((B, 2 * H, 2 * W, C), device="cuda")
    chk(L().tcx_upsample2x_h2(dev(x).data_ptr(), y.data_ptr(), B, H, W, C, sc.data_ptr(), sh.data_ptr(),
                              ovf.data_ptr(), st()))
    a = dev(x)
    chk(L().tcx_gn_apply_tab(a.data_ptr(), a.data_ptr(), B, H * W, C, sc.data_ptr(), sh.data_ptr(), 1, st()))
    y32 = torch.empty_like(y)
    chk(L().tcx_upsample2x(a.data_ptr(), y32.data_ptr(), B, H, W, C, None, None, st()))
    got, ref = from_h2(y).cpu().numpy(), y32.cpu().numpy()
    bound = np.abs(ref) * (2.0 ** -21 + 8 * 2.0 ** -23) + 2.0 ** -25 + 2.0 ** -21 * float(np.abs(ref).max())
    assert np.all(np.abs(got - ref) <= bound), float(np.max(np.abs(got - ref) - bound))
    assert int(ovf.item()) == 0


@pytest.mark.parametrize("Bt,N,C,heads", [(2, 256, 192, 4), (1, 4096, 192, 4), (2, 1024, 64, 4)])
def test_attention_h2(Bt, N, C, heads):
    qkv = dev(rng.standard_normal((Bt, N, 3 * C)))
    o = torch.empty((Bt, N, C), device="cuda")
    o32 = torch.empty_like(o)
    chk(L().tcx_attention_h2(qkv.data_ptr(), o.data_ptr(), Bt, N, C, heads, None, st()))
    chk(L().tcx_attention(qkv.data_ptr(), o32.data_ptr(), Bt, N, C, heads, st()))
    dec_ok(from_h2(o).cpu().numpy(), o32.cpu().numpy())


@pytest.mark.parametrize("Bt,N,C,heads,amp", [(2, 256, 192, 4, 1.0), (2, 256, 192, 4, 3.0), (1, 4096, 192, 4, 1.0),
                                              (2, 512, 64, 4, 2.0), (1, 256, 128, 2, 1.0), (2, 256, 64, 2, 1.0)])
def test_attention_split_vs_oracle(Bt, N, C, heads, amp):
    """f16x3 attention (qkv and output h2, attention_split.hip) against the fp64 oracle on the same
    (h2-representable) inputs, at the fp32 attention's gate and within 2x its error.  amp scales
    q, k, v (amp 3: peaked softmax rows)."""
    from test_gpu_ops import close as close_ops
    qkv32 = dev(rng.standard_normal((Bt, N, 3 * C)) * amp)
    qh = to_h2(qkv32)
    qd = from_h2(qh)  # the values the h2 tensor represents
    o = torch.empty((Bt, N, C), device="cuda")
    o32 = torch.empty_like(o)
    chk(L().tcx_attention_split(qh.data_ptr(), o.data_ptr(), Bt, N, C, heads, st()))
    chk(L().tcx_attention(qd.data_ptr(), o32.data_ptr(), Bt, N, C, heads, st()))
    torch.cuda.synchronize()
    x = qd.double().cpu().numpy()
    d = C // heads
    sp = lambda a: a.reshape(Bt, N, heads, d).transpose(0, 2, 1, 3)  # noqa: E731
    ref = nn_np.sdpa(sp(x[:, :, :C]), sp(x[:, :, C:2 * C]), sp(x[:, :, 2 * C:])).transpose(0, 2, 1, 3).reshape(Bt, N, C)
    got = from_h2(o).double().cpu().numpy()
    e32 = float(np.abs(o32.double().cpu().numpy() - ref).max())
    err = close_ops(got, ref)
    scale = max(1.0, float(np.abs(ref).max()))
    # + 2^-21 of the scale: the h2 output itself carries 22 significant bits
    assert err <= 2 * e32 + (2e-7 + 2.0 ** -21) * scale, (err, e32)


def test_unet_range_fallback_to_fp32():
    """An activation beyond the f16 range raises the flag and the evaluator recomputes in fp32."""
    import warnings

    from toycrystals_amd.models.sde_score_model import CondUNetTiny
    torch.manual_seed(0)
    m = CondUNetTiny(4, 4, 32).cuda().eval()
    with torch.no_grad():
        m.ds1.weight.mul_(1e5)  # ds1 output (written as h2, consumed by down2) far beyond 65504
    x = torch.randn(2, 1, 64, 64, device="cuda")
    t = torch.full((2,), 0.3, device="cuda")
    yc = torch.tensor([0, 1], device="cuda")
    yv = torch.zeros(2, 4, device="cuda")
    with warnings.catch_warnings(record=True) as rec, torch.no_grad():
        warnings.simplefilter("always")
        e = m(x, t, yc, yv)
    assert any("f16 range" in str(r.message) for r in rec)
    from toycrystals_amd import _lib
    old = _lib.conv_precision()
    _lib.set_conv_precision("fp32")
    try:
        with torch.no_grad():
            e32 = m(x, t, yc, yv)
    finally:
        _lib.set_conv_precision(old)
    assert torch.equal(e, e32)


@pytest.mark.parametrize("H,Ci,Co", [(64, 96, 96), (32, 192, 192), (16, 192, 192), (64, 32, 96)])
def test_conv_h2_16x16_kernel_bmod_act_out_h2_gn(H, Ci, Co):
    """The h2-source 3x3 conv on v_mfma_f32_16x16x32_f16 (k_conv3m: rows of 16 / 32 / 64 px, one or
    several 16-channel chunk pairs) with CFG batch aliasing (bmod), SiLU epilogue, h2 output and fused
    GroupNorm partials, against the fp64 oracle at the fp32 conv's gate."""
    x = rng.standard_normal((2, Ci, H, H))
    w = rng.standard_normal((Co, Ci, 3, 3)) / np.sqrt(Ci * 9)
    b = rng.standard_normal(Co)
    xx = np.concatenate([x, x], 0)
    ref = nn_np.conv2d(xx, w, b, padding=1, mode="circular")
    ref = ref / (1 + np.exp(-ref))
    got, part = run_conv_h2(x, w, b, 1, 1, True, bmod=2, Bt=4, act=3, gn=True, out_h2=True)
    fp32 = run_conv(x, w, b, 1, 1, True, bmod=2, Bt=4, act=3)
    fp32_grade(got, fp32, ref)
    s = part.sum(axis=1)
    r = ref.reshape(4, Co, -1)
    np.testing.assert_allclose(s[..., 0], r.sum(-1), rtol=1e-5, atol=1e-3)
    np.testing.assert_allclose(s[..., 1], (r * r).sum(-1), rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("B,C1,Co,H,out_h2", [
    (2, 96, 96, 64, False),   # up1_0's shape (64^2 rows, 96 + 96 -> 96), fp32 output + GroupNorm partials
    (2, 96, 96, 32, False),   # 32^2 rows
    (1, 192, 96, 32, False),  # up2_0's shape (192 + 192 -> 96)
    (2, 96, 96, 64, True),    # h2 output
])
def test_quad_epilogue_equals_column_epilogue(B, C1, Co, H, out_h2):
    """k_conv3lg (the concat with a GroupNorm+SiLU prologue on source 2) stores through the quad-transposed
    epilogue (conv_epi_store_quad) without a residual and through the column epilogue
    (conv_epi_store_cols) with one.  A zero residual makes the two compute the same values: the outputs
    must be bit-equal, and the GroupNorm partials (summed per value in the quad form, as packed pairs in
    the column form: a different fp32 order) equal to fp32 rounding of the 128-pixel sums."""
    x1 = rng.standard_normal((B, C1, H, H))
    x2 = rng.standard_normal((B, C1, H, H)) * 1.5
    w = rng.standard_normal((Co, 2 * C1, 3, 3)) / np.sqrt(2 * C1 * 9)
    b = rng.standard_normal(Co)
    tabs = [dev(t) for t in rand_tabs(B, C1, 5)]
    wh, ws, cpad, kpad = pack_h2(w)
    wf = pack_frag(wh, cpad, kpad, 2 * C1)
    x1d = to_h2(dev(nhwc(x1)))
    x2d = dev(nhwc(x2))
    zero = torch.zeros((B, H, H, Co), device="cuda")
    bd = dev(b)
    outs = []
    for resid in (None, zero):
        y = torch.full((B, H, H, Co), float("nan"), device="cuda")
        gnd = None if out_h2 else torch.zeros((B, H * H // 128, Co, 2), dtype=torch.float64, device="cuda")
        ovf = torch.zeros(1, dtype=torch.int32, device="cuda")
        chk(L().tcx_conv2d_h2_pro(x1d.data_ptr(), x2d.data_ptr(), B, 0, H, H, C1, C1, wh.data_ptr(), wf.data_ptr(),
                                  ws.data_ptr(), bd.data_ptr(), None, resid.data_ptr() if resid is not None else None,
                                  y.data_ptr(), int(out_h2), Co, cpad, kpad, 3, 1, 1, 1, 0,
                                  gnd.data_ptr() if gnd is not None else None, None, None, tabs[0].data_ptr(),
                                  tabs[1].data_ptr(), 0, ovf.data_ptr(), st()))
        torch.cuda.synchronize()
        outs.append((y.cpu().numpy().view(np.uint32), None if gnd is None else gnd.cpu().numpy()))
    (ya, ga), (yb, gb) = outs
    assert np.array_equal(ya, yb), int(np.count_nonzero(ya != yb))
    if ga is not None:
        # 128 fp32 values per partial: the two orders agree to a few fp32 ulps of the sum of |values|
        np.testing.assert_allclose(ga, gb, rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("B,C1,C2,Co,H,ks", [
    (2, 96, 0, 96, 64, 4), (3, 192, 0, 192, 32, 4),  # ds1 / ds2: source 1 chunk-major (k_conv4s2g)
    (2, 96, 96, 96, 64, 3), (3, 192, 192, 96, 32, 3),  # up1.net.0 / up2.net.0: source 2 chunk-major (k_conv3m)
])
def test_chunk_major_source_equals_pixel_major(B, C1, C2, Co, H, ks):
    """tcx_conv2d_h2_pro with a chunk-major source ([C/8][B*H*W][32 B] record planes, bf16 arg bit 16 for
    source 1, bit 32 for source 2: the U-Net's skip tensors) gives bit-identical outputs and GroupNorm
    partials to the same records pixel-major: the kernels stage the same bytes into the same LDS slots."""
    cin = C1 + C2
    x1 = rng.standard_normal((B, C1, H, H))
    x2 = rng.standard_normal((B, C2, H, H)) if C2 else None
    w = rng.standard_normal((Co, cin, ks, ks)) / np.sqrt(cin * ks * ks)
    b = dev(rng.standard_normal(Co))
    wh, ws, cpad, kpad = pack_h2(w)
    wf = pack_frag(wh, cpad, kpad, cin)
    stride = 2 if ks == 4 else 1
    Ho = H // stride
    r1, r2 = to_h2(dev(nhwc(x1))), (to_h2(dev(nhwc(x2))) if C2 else None)

    def cm(r):  # pixel-major records [B][H][W][C/8][8 f32] -> chunk-major [C/8][B*H*W][8 f32]
        return r.reshape(-1, r.shape[-1] // 8, 8).permute(1, 0, 2).contiguous()

    def run(s1, s2, flag):
        y = torch.empty((B, Ho, Ho, Co), device="cuda")
        gnd = torch.zeros((B, Ho * Ho // 128, Co, 2), dtype=torch.float64, device="cuda")
        ovf = torch.zeros(1, dtype=torch.int32, device="cuda")
        chk(L().tcx_conv2d_h2_pro(s1.data_ptr(), s2.data_ptr() if s2 is not None else None, B, 0, H, H, C1, C2,
                                  wh.data_ptr(), wf.data_ptr(), ws.data_ptr(), b.data_ptr(), None, None, y.data_ptr(),
                                  0, Co, cpad, kpad, ks, stride, 1, 1, 0, gnd.data_ptr(), None, None, None, None, flag,
                                  ovf.data_ptr(), st()))
        torch.cuda.synchronize()
        return y.cpu().numpy(), gnd.cpu().numpy()

    ya, ga = run(r1, r2, 0)
    yb, gb = (run(cm(r1), None, 16) if C2 == 0 else run(r1, cm(r2), 32))
    assert np.array_equal(ya, yb) and np.array_equal(ga, gb)
    ref = nn_np.conv2d(np.concatenate([x1, x2], 1) if C2 else x1, w, b.cpu().numpy(), stride=stride, padding=1,
                       mode="circular")
    close(nchw(yb), ref)


def test_chunk_major_source_refused_off_its_kernels():
    """A chunk-major flag on a shape its kernels do not take fails loudly (no silent pixel-major read)."""
    x = to_h2(dev(nhwc(rng.standard_normal((1, 96, 16, 16)))))
    w = rng.standard_normal((96, 96, 3, 3)) / 30.0
    wh, ws, cpad, kpad = pack_h2(w)
    y = torch.empty((1, 16, 16, 96), device="cuda")
    rc = L().tcx_conv2d_h2_pro(x.data_ptr(), None, 1, 0, 16, 16, 96, 0, wh.data_ptr(), None, ws.data_ptr(), None,
                               None, None, y.data_ptr(), 0, 96, cpad, kpad, 3, 1, 1, 1, 0, None, None, None, None, None,
                               16, None, st())
    assert rc != 0


@pytest.mark.parametrize("B,HW,C", [(3, 4096, 96), (3, 1024, 192), (2, 256, 384)])
def test_gn_apply_chunk_major_equals_pixel_major(B, HW, C):
    """tcx_gn_apply_tab_h2_cm writes the same records as tcx_gn_apply_tab_h2 (GroupNorm + SiLU, f16x3
    split), bit for bit, in [C/8][B*HW][32 B] planes."""
    x = dev(rng.standard_normal((B, HW, C)).astype(np.float32) * 3)
    sc = dev(rng.standard_normal((B, C)))
    sh = dev(rng.standard_normal((B, C)))
    pm, cm = torch.empty_like(x), torch.full_like(x, float("nan"))
    ovf = torch.zeros(1, dtype=torch.int32, device="cuda")
    chk(L().tcx_gn_apply_tab_h2(x.data_ptr(), pm.data_ptr(), B, HW, C, sc.data_ptr(), sh.data_ptr(), 1,
                                ovf.data_ptr(), st()))
    chk(L().tcx_gn_apply_tab_h2_cm(x.data_ptr(), cm.data_ptr(), B, HW, C, sc.data_ptr(), sh.data_ptr(),
                                   ovf.data_ptr(), st()))
    torch.cuda.synchronize()
    want = pm.reshape(B * HW, C // 8, 8).permute(1, 0, 2).contiguous()
    a = want.view(torch.int32).cpu().numpy()
    b = cm.view(torch.int32).cpu().numpy().reshape(a.shape)
    nbad = int((a != b).sum())
    print(f"chunk-major apply: {nbad} of {a.size} words differ")
    assert nbad == 0 and int(ovf.item()) == 0


@pytest.mark.parametrize("B,Ci,Co,H,ks", [
    (2, 96, 96, 64, 3), (2, 192, 192, 32, 3), (2, 192, 192, 16, 3),  # k_conv3m (us1 / us2 convs write h2)
    (2, 96, 96, 64, 4), (2, 192, 192, 32, 4),  # k_conv4s2g (ds1 / ds2)
    (2, 192, 576, 16, 1),  # k_lin1x1 (qkv)
])
def test_conv_h2_output_equals_split_of_fp32_output(B, Ci, Co, H, ks):
    """An h2-output conv (16-B paired record stores, store_h2_pair) writes exactly tcx_f32_to_h2 of the
    same conv's fp32 output, word for word."""
    x = rng.standard_normal((B, Ci, H, H))
    w = rng.standard_normal((Co, Ci, ks, ks)) / np.sqrt(Ci * ks * ks)
    b = dev(rng.standard_normal(Co))
    wh, ws, cpad, kpad = pack_h2(w)
    wf = pack_frag(wh, cpad, kpad, Ci) if ks in (3, 4) else None
    stride, pad = (2, 1) if ks == 4 else (1, ks // 2)
    Ho = H // stride
    xd = to_h2(dev(nhwc(x)))

    def run(out_h2):
        y = torch.full((B, Ho, Ho, Co), float("nan"), device="cuda")
        ovf = torch.zeros(1, dtype=torch.int32, device="cuda")
        chk(L().tcx_conv2d_h2_pro(xd.data_ptr(), None, B, 0, H, H, Ci, 0, wh.data_ptr(),
                                  wf.data_ptr() if wf is not None else None, ws.data_ptr(), b.data_ptr(), None, None,
                                  y.data_ptr(), out_h2, Co, cpad, kpad, ks, stride, pad, 1, 0, None, None, None, None,
                                  None, 0, ovf.data_ptr(), st()))
        return y

    want = to_h2(run(0)).view(torch.int32).cpu().numpy()
    got = run(1).view(torch.int32).cpu().numpy()
    nbad = int((want != got).sum())
    print(f"h2 output vs split fp32 output: {nbad} of {want.size} words differ")
    assert nbad == 0
