"""GPU: the bf16 single-product path (config 5's "bf16 MFMA conv-as-GEMM", BASELINE.json configs[4]).

Records hold bf16 halves (hi = bf16(v), lo = bf16(v - hi)); every product is ONE
v_mfma_f32_32x32x16_bf16 of the hi halves with fp32 accumulation.  Checks:
  * the writers produce exactly torch's round-to-nearest-even bf16 of the value (hi) and of the
    residual (lo);
  * each bf16 kernel (k_conv3g at 16/32/64/128-pixel rows with and without the GroupNorm+SiLU prologue,
    the im2col kernel, k_conv4s2h, the split attention) against a float64 reference computed on the
    SAME bf16-rounded operands: then only the fp32 accumulation differs (5e-6 of the output scale);
    the attention additionally rounds P and its output to bf16 (1e-2);
  * the whole U-Net forward at 64² and 256² against the reference's fp32 goldens: bf16 operands
    carry 8 significant bits, so the stated gate is 3e-2 of the output scale (observed printed).
"""
import numpy as np
import pytest
import torch

from oracle import nn_np

from test_gpu_ops import L, chk, dev, nchw, nhwc, pack, st

pytestmark = pytest.mark.gpu

rng = np.random.default_rng(11)


def bf(a):
    """round to bf16 (nearest even) and back, as torch does on the CPU"""
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).to(torch.bfloat16).float().numpy()


def to_bf16_records(t):
    """fp32 NHWC [.., C] -> bf16 records via the GroupNorm-apply writer with scale 1, shift 0, no SiLU"""
    B = t.shape[0]
    C = t.shape[-1]
    HW = t.numel() // (B * C)
    one = torch.ones(B, C, device="cuda")
    zero = torch.zeros(B, C, device="cuda")
    y = torch.empty_like(t)
    chk(L().tcx_gn_apply_tab_bf16(t.data_ptr(), y.data_ptr(), B, HW, C, one.data_ptr(), zero.data_ptr(), 0, st()))
    return y


def decode(rec):
    """bf16 records [.., C] -> (hi, lo) float32 arrays [.., C]"""
    u = rec.contiguous().view(torch.int32).cpu().numpy().view(np.uint16)
    C = rec.shape[-1]
    g = u.reshape(-1, C // 8, 2, 8)
    hi = (g[:, :, 0, :].astype(np.uint32) << 16).view(np.float32).reshape(rec.shape)
    lo = (g[:, :, 1, :].astype(np.uint32) << 16).view(np.float32).reshape(rec.shape)
    return hi, lo


def test_bf16_writer_is_round_to_nearest_even():
    v = (rng.standard_normal((2, 8, 8, 32)) * 10.0 ** rng.uniform(-6, 6, (2, 8, 8, 32))).astype(np.float32)
    hi, lo = decode(to_bf16_records(dev(v)))
    assert np.array_equal(hi, bf(v))
    assert np.array_equal(lo, bf(v - bf(v)))


def pack_bf16(w):
    wpk, cpad, kpad = pack(w)
    wh = torch.empty_like(wpk)
    ws = torch.empty(4, device="cuda")
    chk(L().tcx_pack_conv_weight_bf16(wpk.data_ptr(), wh.data_ptr(), ws.data_ptr(), cpad, kpad, st()))
    return wh, ws, cpad, kpad


def pack_frag(wh, cpad, kpad, cin):
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


def run_conv_bf16(x, w, b, stride, pad, x2=None, frag=True, tabs=None):
    """tabs: (scale, shift) [B][C] for a GroupNorm+SiLU prologue on x (fp32 source, k_conv3g only)"""
    B, C1, H, W = x.shape
    C2 = 0 if x2 is None else x2.shape[1]
    co, ci, ks, _ = w.shape
    wh, ws, cpad, kpad = pack_bf16(w)
    Ho, Wo = (H + 2 * pad - ks) // stride + 1, (W + 2 * pad - ks) // stride + 1
    y = torch.empty((B, Ho, Wo, co), device="cuda")
    xd = dev(nhwc(x)) if tabs is not None else to_bf16_records(dev(nhwc(x)))
    x2d = to_bf16_records(dev(nhwc(x2))) if x2 is not None else None
    wf = pack_frag(wh, cpad, kpad, C1 + C2) if (frag and ks in (3, 4)) else None
    p = lambda t: t.data_ptr() if t is not None else None  # noqa: E731
    sc, sh = (dev(tabs[0]), dev(tabs[1])) if tabs is not None else (None, None)
    chk(L().tcx_conv2d_h2_pro(xd.data_ptr(), p(x2d), B, 0, H, W, C1, C2, wh.data_ptr(), p(wf), ws.data_ptr(),
                              dev(b).data_ptr(), None, None, y.data_ptr(), 0, co, cpad, kpad, ks, stride, pad, 1, 0,
                              None, p(sc), p(sh), None, None, 1, None, st()))
    return nchw(y.cpu().numpy())


def conv_ref(x, w, b, stride, pad):
    return nn_np.conv2d(x.astype(np.float64), w.astype(np.float64), b.astype(np.float64), stride, pad,
                        mode="circular")


@pytest.mark.parametrize("B,C1,C2,H,co,ks,stride,frag", [
    (2, 96, 0, 64, 96, 3, 1, True),      # k_conv3lb (LDS-DMA bf16), 64-px rows
    (2, 96, 96, 32, 96, 3, 1, True),     # k_conv3g, two sources, 32-px rows
    (1, 96, 0, 128, 96, 3, 1, True),     # k_conv3lb, 128-px rows
    (1, 96, 0, 256, 96, 3, 1, True),     # k_conv3lb, 256-px rows (one row per tile)
    (1, 96, 96, 256, 96, 3, 1, True),    # k_conv3lb, two sources (up1_0 at 256^2)
    (2, 192, 0, 64, 192, 3, 1, True),    # k_conv3lb, two n blocks (mid block at 256^2)
    (1, 192, 192, 128, 96, 3, 1, True),  # k_conv3lb, Cin = 384 over two sources (up2_0 at 256^2)
    (3, 96, 0, 128, 192, 3, 1, True),    # k_conv3lb, 96 -> 192, odd batch (down2_0 at 256^2)
    (2, 64, 0, 16, 96, 3, 1, True),      # k_conv3g, 16-px rows (mid block)
    (2, 64, 0, 16, 64, 3, 1, False),     # no fragment copy: the im2col kernel (no bf16 k_conv3p)
    (2, 96, 0, 64, 96, 4, 2, False),     # k_conv4s2h (ds1 at 64 -> 32)
    (2, 96, 0, 64, 96, 4, 2, True),      # k_conv4s2g (LDS-DMA, fragment-ordered 4x4 weights)
    (1, 96, 0, 128, 96, 4, 2, True),     # k_conv4s2g at Wo = 64 (config 5's ds2)
    (2, 192, 0, 16, 576, 1, 1, False),   # 1x1 (qkv): the im2col kernel
])
def test_bf16_convs_vs_float64_on_rounded_operands(B, C1, C2, H, co, ks, stride, frag):
    pad = 1 if ks in (3, 4) else 0
    x = rng.standard_normal((B, C1, H, H)).astype(np.float32)
    x2 = rng.standard_normal((B, C2, H, H)).astype(np.float32) if C2 else None
    w = (rng.standard_normal((co, C1 + C2, ks, ks)) / np.sqrt((C1 + C2) * ks * ks)).astype(np.float32)
    b = rng.standard_normal(co).astype(np.float32)
    y = run_conv_bf16(x, w, b, stride, pad, x2=x2, frag=frag)
    xin = bf(x) if x2 is None else np.concatenate([bf(x), bf(x2)], axis=1)
    ref = conv_ref(xin, bf(w), b, stride, pad)
    err = float(np.abs(y - ref).max()) / max(1.0, float(np.abs(ref).max()))
    print(f"bf16 conv B={B} C={C1}+{C2} {H}² co={co} k={ks} s={stride}: {err:.2e} vs float64 on bf16 operands")
    assert err < 5e-6


@pytest.mark.parametrize("Bt,H,C1,C2,co", [(8, 256, 96, 0, 96), (4, 256, 96, 96, 96), (16, 128, 96, 0, 192),
                                            (32, 64, 192, 0, 192)])
def test_bf16_conv3lb_repeats_bit_for_bit(Bt, H, C1, C2, co):
    """k_conv3lb with the quad-transposed epilogue repeats bit for bit (output and GroupNorm partials)
    into a NaN-filled output: the regression test of the store-data hazard (conv_common.hpp
    store_b128_guarded) that made one dword per 32 x 32 block come out old or new at random
    (profiles/r04_lbwhere.txt)."""
    g = torch.Generator(device="cuda").manual_seed(0)
    x1 = to_bf16_records(torch.randn((Bt, H, H, C1), device="cuda", generator=g))
    x2 = to_bf16_records(torch.randn((Bt, H, H, C2), device="cuda", generator=g)) if C2 else None
    w = (rng.standard_normal((co, C1 + C2, 3, 3)) / np.sqrt(9 * (C1 + C2))).astype(np.float32)
    wh, ws, cpad, kpad = pack_bf16(w)
    wf = pack_frag(wh, cpad, kpad, C1 + C2)
    b = dev(rng.standard_normal(co).astype(np.float32))
    y = torch.empty((Bt, H, H, co), device="cuda")
    gn = torch.zeros((Bt, H * H // 128, co, 2), dtype=torch.float64, device="cuda")

    def run():
        y.fill_(float("nan"))
        gn.zero_()
        chk(L().tcx_conv2d_h2_pro(x1.data_ptr(), x2.data_ptr() if x2 is not None else None, Bt, 0, H, H, C1, C2,
                                  wh.data_ptr(), wf.data_ptr(), ws.data_ptr(), b.data_ptr(), None, None, y.data_ptr(),
                                  0, co, cpad, kpad, 3, 1, 1, 1, 0, gn.data_ptr(), None, None, None, None, 1, None,
                                  st()))
        torch.cuda.synchronize()
        return y.clone(), gn.clone()
    y0, g0 = run()
    assert not bool(torch.isnan(y0).any())
    bad = 0
    for _ in range(6):
        y1, g1 = run()
        bad += int((y1 != y0).sum()) + int((g1 != g0).sum())
    print(f"k_conv3lb Bt={Bt} {H}² {C1}+{C2}->{co}: 6 repeats, {bad} differing values")
    assert bad == 0


@pytest.mark.parametrize("B,H", [(2, 64), (1, 256)])
def test_bf16_conv3g_gn_prologue_vs_float64(B, H):
    """the prologue applies silu(x*scale+shift) in fp32 and rounds the result to bf16 in registers
    (64-px rows: two halo units per thread; 256-px rows: the slim halo, 7 units per thread)"""
    C = 96
    x = rng.standard_normal((B, C, H, H)).astype(np.float32)
    sc = (0.5 + rng.random((B, C))).astype(np.float32)
    sh = rng.standard_normal((B, C)).astype(np.float32) * 0.2
    w = (rng.standard_normal((C, C, 3, 3)) / np.sqrt(9 * C)).astype(np.float32)
    b = rng.standard_normal(C).astype(np.float32)
    y = run_conv_bf16(x, w, b, 1, 1, tabs=(sc, sh))
    z = x * sc[:, :, None, None] + sh[:, :, None, None]
    a = z / (1.0 + np.exp(-z.astype(np.float64)))
    ref = conv_ref(bf(a.astype(np.float32)), bf(w), b, 1, 1)
    err = float(np.abs(y - ref).max()) / max(1.0, float(np.abs(ref).max()))
    print(f"bf16 conv3g with the GN+SiLU prologue: {err:.2e}")
    # the kernel's SiLU (hardware exp2 / rcp) may round to the neighbouring bf16 value: 2^-8 of one input
    assert err < 2e-3


def test_bf16_attention_split_vs_float64():
    Bt, N, C, heads = 2, 256, 192, 4
    D = C // heads
    qkv = (rng.standard_normal((Bt, N, 3 * C)) * 0.5).astype(np.float32)
    rec = to_bf16_records(dev(qkv))
    out = torch.empty(Bt, N, C, device="cuda")
    chk(L().tcx_attention_split_bf16(rec.data_ptr(), out.data_ptr(), Bt, N, C, heads, st()))
    hi, _ = decode(out)
    qb = bf(qkv).astype(np.float64)
    q, k, v = qb[..., :C], qb[..., C:2 * C], qb[..., 2 * C:]
    ref = np.empty((Bt, N, C))
    for b in range(Bt):
        for h in range(heads):
            sl = slice(h * D, (h + 1) * D)
            s = q[b, :, sl] @ k[b, :, sl].T / np.sqrt(D)
            p = np.exp(s - s.max(1, keepdims=True))
            ref[b, :, sl] = (p / p.sum(1, keepdims=True)) @ v[b, :, sl]
    err = float(np.abs(hi - ref).max()) / max(1.0, float(np.abs(ref).max()))
    print(f"bf16 split attention (P rounded to bf16, output as bf16): {err:.2e}")
    assert err < 1e-2


@pytest.mark.parametrize("name", ["unet96_b2", "unet96_b2_h256"])
def test_bf16_unet_forward_vs_reference(golden, name):
    """the whole evaluator in bf16 against the reference's fp32 forward: stated gate 3e-2 of the scale"""
    from toycrystals_amd import _lib
    from test_gpu_models import cu, rel_err, unet
    g = golden(name)
    m = unet(96)
    old = _lib.conv_precision()
    try:
        _lib.set_conv_precision("bf16")
        with torch.no_grad():
            e_bf = m(cu(g["x_t"]), cu(g["t"]), cu(g["y_cat"]), cu(g["y_cont"])).cpu().numpy()
        _lib.set_conv_precision("f16x3")
        with torch.no_grad():
            e_h2 = m(cu(g["x_t"]), cu(g["t"]), cu(g["y_cat"]), cu(g["y_cont"])).cpu().numpy()
    finally:
        _lib.set_conv_precision(old)
    e1, e2 = rel_err(e_bf, g["eps"]), rel_err(e_h2, g["eps"])
    print(f"{name}: bf16 {e1:.2e}, f16x3 {e2:.2e} of the output scale vs the reference fp32 forward")
    assert e2 < 2e-5
    assert e1 < 3e-2 and e1 > 10 * e2  # really the bf16 path (8-bit operands), within its gate


@pytest.fixture
def bf16():
    from toycrystals_amd import _lib
    old = _lib.conv_precision()
    _lib.set_conv_precision("bf16")
    yield
    _lib.set_conv_precision(old)


def test_bf16_sde_256px_vs_reference(golden, bf16):
    """Config 5's sampler at 256x256 in bf16 (2 reverse-SDE steps + projection, CFG 1.5, base 96)
    against the reference's fp32 run of the same draws (sde96_2step_h256).  Stated gates for 8-bit
    operands: x0_hat within 3e-2 of max(1, |x0_hat|max) (observed 3.7e-3), image mean-abs 5e-3; the
    image is (x0_hat + 1)/2 clamped, so its max-abs gate is half the x0_hat gate in absolute terms
    (this untrained net's x0_hat reaches tens, so single pixels move by ~0.2, observed printed)."""
    from test_gpu_models import run_sde, unet
    from toycrystals_amd.models.sde_score_model import host_noise
    g = golden("sde96_2step_h256")
    m = unet(96)
    B = int(g["B"])
    shape = (B, 1, 256, 256)
    torch.manual_seed(int(g["noise_seed"]))
    noise = host_noise(shape, int(g["steps"]) + 1)
    out, x0 = run_sde(m, g, noise.cuda(), shape)
    img = float(np.abs(out - g["out"]).max())
    x0e = float(np.abs(x0 - g["x0_unclamped"]).max()) / max(1.0, float(np.abs(g["x0_unclamped"]).max()))
    print(f"bf16 sde96_2step_h256: image max-abs {img:.3e} mean-abs {float(np.abs(out - g['out']).mean()):.3e}, "
          f"x0_hat rel {x0e:.3e}")
    scale = max(1.0, float(np.abs(g["x0_unclamped"]).max()))
    assert x0e < 3e-2 and float(np.abs(out - g["out"]).mean()) < 5e-3 and img <= 0.5 * 3e-2 * scale
    assert np.abs(np.clip((x0 + 1.0) * 0.5, 0.0, 1.0) - out).max() < 1e-6


def test_bf16_trained_sde300_trajectory_drift(golden):
    """The bf16 path's 300-step reverse SDE (CFG 1.5, t_end 0.005) on the trained base-96 model
    (trained96_ema, B = 8, the reference's recorded draws; /root/reference/src/toycrystals/models/
    sde_score_model.py:507-569) against the reference's fp32 run, gated by an ERROR MODEL: the
    reference's own run of the same trajectory with every conv operand and the attention's q, k, v, P
    rounded to bf16 and fp32 accumulation (tests/golden/make_goldens.py gen_bf16_emulated,
    sde96_trained_300_bf16emu.npz) drifts from its fp32 run by image mean-abs 3.0e-3, p99 3.4e-2,
    max 0.25, 6.7 % of the pixels off by more than 1e-2: per-step bf16 rounding (~7e-3 of a forward)
    is absorbed on most of the image and amplified at a few unstable pixels of the stochastic
    trajectory.  Gate: each of those four statistics of the bf16 path vs the fp32 reference at most
    2x the emulated reference's (printed), and the fp32-grade f16x3 path on the same run within 1e-4."""
    from test_gpu_models import run_sde, unet
    from toycrystals_amd import _lib
    from toycrystals_amd.models.sde_score_model import host_noise
    g = golden("sde96_trained_300")
    emu = golden("sde96_trained_300_bf16emu")
    m = unet(96, golden("trained96_ema"))
    B, steps = int(g["B"]), int(g["steps"])
    assert int(emu["B"]) == B and int(emu["noise_seed"]) == int(g["noise_seed"]) and int(emu["steps"]) == steps
    torch.manual_seed(int(g["noise_seed"]))
    noise = host_noise((B, 1, 64, 64), steps + 1).cuda()
    old = _lib.conv_precision()
    try:
        _lib.set_conv_precision("f16x3")
        out_h2, x0_h2 = run_sde(m, g, noise, (B, 1, 64, 64))
        _lib.set_conv_precision("bf16")
        out_bf, x0_bf = run_sde(m, g, noise, (B, 1, 64, 64))
    finally:
        _lib.set_conv_precision(old)

    def stats(img):
        d = np.abs(img - g["out"])
        return {"mean": float(d.mean()), "p99": float(np.quantile(d, 0.99)), "max": float(d.max()),
                "off": float((d > 1e-2).mean())}
    model, got = stats(emu["out"]), stats(out_bf)
    for k in model:
        print(f"bf16 300-step vs fp32 reference, {k}: bf16 path {got[k]:.3e}, bf16-emulated reference "
              f"{model[k]:.3e} (gate {2 * model[k]:.3e})")
    d_emu = np.abs(out_bf - emu["out"])
    print(f"bf16 path vs the bf16-emulated reference: mean {float(d_emu.mean()):.3e} max {float(d_emu.max()):.3e}")
    for k in model:
        assert got[k] <= 2.0 * model[k], (k, got[k], model[k])
    # outer caps: round 3's fixed bounds (mean 5e-3, 8 % of pixels off by > 1e-2), and the distance to the
    # emulated run itself (observed mean 4.6e-3; both are draws of the same 8-bit noise around fp32)
    assert got["mean"] <= 5e-3 and got["off"] <= 0.08, got
    assert float(d_emu.mean()) <= 1e-2
    assert float(np.abs(out_h2 - g["out"]).max()) < 1e-4  # the fp32-grade path on the same run
    assert float(np.abs(out_bf - out_h2).max()) > 1e-5  # really the bf16 path


def test_bf16_256px_b64_workload(bf16):
    """Config 5's per-GPU workload: 256x256, B = 64 (512 over 8 GPUs), 300 reverse-SDE steps, CFG 1.5,
    bf16, in-kernel Philox.  With CFG the 128 rows exceed the 84-row pass cap (2 GiB activations),
    so every evaluation runs two passes (42 + 22 images).  The images are finite and in [0, 1], and
    each checked image equals itself sampled alone at its Philox element offset, bit for bit (first
    and last of each pass).  This random-init net saturates the clamped image, so the same check runs
    on the unclamped x0_hat too (every pixel of the trajectory)."""
    from test_gpu_models import unet
    from toycrystals_amd.models.sde_score_model import VPSDE, sample_reverse_sde_euler_maruyama
    m = unet(96)
    sde = VPSDE(0.1, 30.0)
    B, S = 64, 256
    y_cat = (torch.arange(B) % 4).cuda()
    y_cont = torch.zeros(B, 4, device="cuda")
    y_cont[:, 1] = torch.linspace(0.0, np.pi / 3, B, device="cuda")
    kw = dict(n_steps=300, guidance_scale=1.5, t_end=0.005, seed=77)
    x = sample_reverse_sde_euler_maruyama(m, sde, y_cat, y_cont, (B, 1, S, S), **kw)
    assert bool(torch.isfinite(x).all()) and float(x.min()) >= 0.0 and float(x.max()) <= 1.0
    print(f"bf16 256px B=64: mean {float(x.mean()):.4f}, unsaturated {float(((x > 0) & (x < 1)).float().mean()):.3f}")
    x0 = sample_reverse_sde_euler_maruyama(m, sde, y_cat, y_cont, (B, 1, S, S), return_x0_hat=True, **kw)
    assert bool(torch.isfinite(x0).all())
    assert torch.equal(torch.clamp((x0 + 1.0) * 0.5, 0.0, 1.0), x)
    for i in (0, 41, 42, 63):
        xi = sample_reverse_sde_euler_maruyama(m, sde, y_cat[i:i + 1], y_cont[i:i + 1], (1, 1, S, S),
                                               elem_offset=i * S * S, return_x0_hat=True, **kw)
        assert torch.equal(xi[0], x0[i]), (i, float((xi[0] - x0[i]).abs().max()))


# ---------------------------------------------------------------- 2-byte bf16 ("b2", config 5 at 256^2)
# The U-Net evaluator at precision bf16 and 256^2 keeps its tensors as plain NHWC bf16 (csrc/h2.hpp "b2"):
# the records' hi halves, which are all a bf16 product reads.  The kernels read the same bf16 values into
# the same MFMA operands in the same order, so against the 4-byte record path the results are equal BIT FOR
# BIT (fp32 outputs), and a b2 output is the round-to-nearest-even of the fp32 value.

def to_b2(t):
    """fp32 NHWC [.., C] -> 2-byte bf16 (torch int16 storage) via the b2 apply writer (scale 1, shift 0)"""
    B, C = t.shape[0], t.shape[-1]
    HW = t.numel() // (B * C)
    y = torch.empty(t.shape, dtype=torch.int16, device="cuda")
    one = torch.ones(B, C, device="cuda")
    zero = torch.zeros(B, C, device="cuda")
    chk(L().tcx_gn_apply_tab_b2(t.data_ptr(), y.data_ptr(), B, HW, C, one.data_ptr(), zero.data_ptr(), 0, 0, st()))
    return y


def b2_float(t):
    return t.view(torch.bfloat16).float()


def test_b2_writer_is_round_to_nearest_even_and_the_record_hi():
    v = (rng.standard_normal((2, 8, 8, 32)) * 10.0 ** rng.uniform(-6, 6, (2, 8, 8, 32))).astype(np.float32)
    y = to_b2(dev(v))
    assert np.array_equal(b2_float(y).cpu().numpy(), bf(v))
    hi, _ = decode(to_bf16_records(dev(v)))
    assert np.array_equal(b2_float(y).cpu().numpy(), hi)


def test_b2_apply_in_place_equals_the_record_apply():
    """GroupNorm+SiLU of a b2 tensor in place (the pre-norm conv outputs of config 5) == the record writer
    applied to the same bf16 values held in fp32, bit for bit"""
    B, HW, C = 3, 512, 96
    x = torch.from_numpy(bf(rng.standard_normal((B, HW, C)).astype(np.float32) * 3)).cuda()
    sc = torch.rand(B, C, device="cuda") + 0.5
    sh = torch.randn(B, C, device="cuda")
    y = to_b2(x)
    chk(L().tcx_gn_apply_tab_b2(y.data_ptr(), y.data_ptr(), B, HW, C, sc.data_ptr(), sh.data_ptr(), 1, 1, st()))
    rec = torch.empty_like(x)
    chk(L().tcx_gn_apply_tab_bf16(x.data_ptr(), rec.data_ptr(), B, HW, C, sc.data_ptr(), sh.data_ptr(), 1, st()))
    hi, _ = decode(rec)
    assert np.array_equal(b2_float(y).cpu().numpy(), hi)


@pytest.mark.parametrize("B,H,W,C,tabs", [(2, 128, 128, 96, True), (2, 64, 64, 192, False)])
def test_b2_upsample_equals_the_record_upsample(B, H, W, C, tabs):
    """config 5's us1 (GroupNorm+SiLU of the source applied while staging) and us2, segmented band form"""
    x = torch.randn(B, H, W, C, device="cuda")
    sc = torch.rand(B, C, device="cuda") + 0.5 if tabs else None
    sh = torch.randn(B, C, device="cuda") if tabs else None
    p = lambda t: t.data_ptr() if t is not None else None  # noqa: E731
    y = torch.empty((B, 2 * H, 2 * W, C), dtype=torch.int16, device="cuda")
    chk(L().tcx_upsample2x_b2(x.data_ptr(), y.data_ptr(), B, H, W, C, p(sc), p(sh), st()))
    rec = torch.empty((B, 2 * H, 2 * W, C), device="cuda")
    chk(L().tcx_upsample2x_bf16(x.data_ptr(), rec.data_ptr(), B, H, W, C, p(sc), p(sh), st()))
    hi, _ = decode(rec)
    assert np.array_equal(b2_float(y).cpu().numpy(), hi)


def test_b2_attention_vs_the_record_attention_and_float64():
    """the b2 attention (config 5: 2-byte bf16 qkv and output) against the 4-byte record form of the same kernel
    (8 waves x 128-key tiles, deferred running max) and against float64 on the same bf16 operands.  The b2 output
    is rounded to bf16, so the two agree to bf16 rounding of the output; each is gated against float64 as
    test_bf16_attention_split_vs_float64 (1e-2 of the scale: P and the output are bf16).  (A 4-wave x 64-key
    form measured in round 6 was slower and removed, profiles/r06_h_attn_q4_ab.txt.)"""
    Bt, N, C, heads = 2, 1024, 192, 4
    D = C // heads
    qkv_np = (rng.standard_normal((Bt, N, 3 * C)) * 0.5).astype(np.float32)
    qkv = torch.from_numpy(qkv_np).cuda()
    out_r = torch.empty(Bt, N, C, device="cuda")
    chk(L().tcx_attention_split_bf16(to_bf16_records(qkv).data_ptr(), out_r.data_ptr(), Bt, N, C, heads, st()))
    out_b = torch.empty((Bt, N, C), dtype=torch.int16, device="cuda")
    chk(L().tcx_attention_split_b2(to_b2(qkv).data_ptr(), out_b.data_ptr(), Bt, N, C, heads, st()))
    hi, _ = decode(out_r)
    yb = b2_float(out_b).cpu().numpy()
    qb = bf(qkv_np).astype(np.float64)
    q, k, v = qb[..., :C], qb[..., C:2 * C], qb[..., 2 * C:]
    ref = np.empty((Bt, N, C))
    for b in range(Bt):
        for h in range(heads):
            sl = slice(h * D, (h + 1) * D)
            sc = q[b, :, sl] @ k[b, :, sl].T / np.sqrt(D)
            pr = np.exp(sc - sc.max(1, keepdims=True))
            ref[b, :, sl] = (pr / pr.sum(1, keepdims=True)) @ v[b, :, sl]
    scale = max(1.0, float(np.abs(ref).max()))
    eb, er = float(np.abs(yb - ref).max()) / scale, float(np.abs(hi - ref).max()) / scale
    d = float(np.abs(yb - hi).max()) / scale
    print(f"b2 attention vs float64 {eb:.2e}, records {er:.2e}; b2 vs records {d:.2e}")
    assert eb < 1e-2 and er < 1e-2 and d < 1e-2


def _conv_fmt(x1, x2, w, b, ks, stride, fmt, out_b2, gn=False):
    """the conv over fp32 NHWC sources held as records (fmt 1) or b2 (fmt 2); out_b2: 2-byte output"""
    B, H, W, C1 = x1.shape
    C2 = x2.shape[-1] if x2 is not None else 0
    co = w.shape[0]
    wh, ws, cpad, kpad = pack_bf16(w)
    wf = pack_frag(wh, cpad, kpad, C1 + C2)
    cv = to_b2 if fmt == 2 else to_bf16_records
    s1 = cv(x1)
    s2 = cv(x2) if x2 is not None else None
    pad = 1 if ks in (3, 4) else 0
    Ho, Wo = (H + 2 * pad - ks) // stride + 1, (W + 2 * pad - ks) // stride + 1
    y = torch.empty((B, Ho, Wo, co), dtype=torch.int16 if out_b2 else torch.float32, device="cuda")
    g = torch.zeros((B, Ho * Wo // 128, co, 2), dtype=torch.float64, device="cuda") if gn else None
    p = lambda t: t.data_ptr() if t is not None else None  # noqa: E731
    chk(L().tcx_conv2d_h2_pro(s1.data_ptr(), p(s2), B, 0, H, W, C1, C2, wh.data_ptr(), p(wf), ws.data_ptr(),
                              dev(b).data_ptr(), None, None, y.data_ptr(), int(out_b2), co, cpad, kpad, ks, stride,
                              pad, 1, 0, p(g), None, None, None, None, fmt, None, st()))
    torch.cuda.synchronize()
    return y, g


@pytest.mark.parametrize("B,C1,C2,H,co,ks,stride", [
    (1, 96, 0, 256, 96, 3, 1),     # k_conv3lb at 256-px rows (down1_1 / up1_1)
    (1, 96, 96, 256, 96, 3, 1),    # two b2 sources (up1_0)
    (2, 96, 0, 128, 192, 3, 1),    # 128-px rows, two n blocks (down2_0)
    (1, 192, 192, 128, 96, 3, 1),  # Cin 384 over two sources (up2_0)
    (2, 192, 0, 64, 192, 3, 1),    # 64-px rows (the mid block)
    (1, 192, 0, 128, 192, 4, 2),   # k_conv4s2g, slim slots at Wo = 64 (ds2)
    (2, 192, 0, 64, 576, 1, 1),    # k_lin1x1 (qkv at 256^2: 4,096 tokens per image)
])
def test_b2_conv_equals_the_record_conv(B, C1, C2, H, co, ks, stride):
    """fp32 outputs and GroupNorm partials against the 4-byte record sources: bit for bit where both run one
    kernel (4x4/s2, 1x1); for the 3x3 convs both run k_conv3lb by default (TCX_CONV3MB=1/2: the b2 sources on
    k_conv3mb's 16x16x32 tap pairs — the same bf16 products summed in fp32 in another order), so within 5e-6 of
    the output scale.  The b2 output is the round-to-nearest-even of the same kernel's fp32 output."""
    g_ = torch.Generator(device="cuda").manual_seed(1)
    x1 = torch.randn((B, H, H, C1), device="cuda", generator=g_)
    x2 = torch.randn((B, H, H, C2), device="cuda", generator=g_) if C2 else None
    w = (rng.standard_normal((co, C1 + C2, ks, ks)) / np.sqrt((C1 + C2) * ks * ks)).astype(np.float32)
    b = rng.standard_normal(co).astype(np.float32)
    gn = ks == 3
    yr, gr = _conv_fmt(x1, x2, w, b, ks, stride, 1, False, gn)
    yb, gb = _conv_fmt(x1, x2, w, b, ks, stride, 2, False, gn)
    if ks == 3:
        scale = max(1.0, float(yr.abs().max()))
        err = float((yr - yb).abs().max()) / scale
        print(f"b2 vs records (3x3) {C1}+{C2}->{co} at {H}^2: {err:.2e}")
        assert err < 5e-6
        np.testing.assert_allclose(gb.cpu().numpy(), gr.cpu().numpy(), rtol=1e-5, atol=1e-3)
    else:
        assert torch.equal(yr, yb)
        if gn:
            assert torch.equal(gr, gb)
    y2, _ = _conv_fmt(x1, x2, w, b, ks, stride, 2, True)
    assert torch.equal(b2_float(y2), yb.to(torch.bfloat16).float())


def test_b2_ds1_wo128_vs_float64_on_rounded_operands():
    """config 5's ds1 (256^2 -> 128^2, 96 channels) on k_conv4s2g's slim b2 slots (the 4-byte records take
    the im2col kernel there): against float64 on the same bf16 operands"""
    B, C, H = 1, 96, 256
    x = rng.standard_normal((B, C, H, H)).astype(np.float32)
    w = (rng.standard_normal((C, C, 4, 4)) / np.sqrt(16 * C)).astype(np.float32)
    b = rng.standard_normal(C).astype(np.float32)
    y, _ = _conv_fmt(dev(nhwc(x)), None, w, b, 4, 2, 2, False)
    ref = conv_ref(bf(x), bf(w), b, 2, 1)
    err = float(np.abs(nchw(y.cpu().numpy()) - ref).max()) / max(1.0, float(np.abs(ref).max()))
    print(f"b2 ds1 Wo=128: {err:.2e} vs float64 on bf16 operands")
    assert err < 5e-6


B2_CHILD = r"""
import sys, numpy as np, torch
sys.path[:0] = [sys.argv[1], sys.argv[1] + "/tests", sys.argv[1] + "/vae-diffusion-toy-crystals_amd"]
from toycrystals_amd import _lib
from test_gpu_models import cu, unet
g = dict(np.load(sys.argv[1] + "/tests/golden/unet96_b2_h256.npz"))
m = unet(96)
_lib.set_conv_precision("bf16")
with torch.no_grad():
    e = m(cu(g["x_t"]), cu(g["t"]), cu(g["y_cat"]), cu(g["y_cont"])).cpu().numpy()
np.save(sys.argv[2], e)
"""


def test_b2_256px_forward_vs_records_and_reference(tmp_path, golden):
    """the whole 256^2 bf16 forward with b2 tensors (default) and with 4-byte records (TCX_BF_B2=0), each in
    its own process: both within the stated 3e-2 gate of the reference's fp32 forward; the b2 form adds the
    bf16 rounding of the pre-GroupNorm conv outputs (printed: its distance to the record form)"""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = {}
    for v in ("1", "0"):
        path = str(tmp_path / f"e{v}.npy")
        env = dict(os.environ, TCX_BF_B2=v)
        r = subprocess.run([sys.executable, "-c", B2_CHILD, root, path], capture_output=True, text=True, timeout=300,
                           env=env)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
        out[v] = np.load(path)
    g = golden("unet96_b2_h256")
    scale = max(1.0, float(np.abs(g["eps"]).max()))
    e_b2 = float(np.abs(out["1"] - g["eps"]).max()) / scale
    e_rec = float(np.abs(out["0"] - g["eps"]).max()) / scale
    d = float(np.abs(out["1"] - out["0"]).max()) / scale
    print(f"256^2 bf16 forward vs reference: b2 {e_b2:.2e}, records {e_rec:.2e}; b2 vs records {d:.2e}")
    assert e_b2 < 3e-2 and e_rec < 3e-2
    assert d > 0.0  # the b2 path really ran (its pre-norm rounding)


def test_b2_head_rejects_misaligned_out_w():
    """config 5 (256^2 bf16, b2 tensors): up1_1 writes 2-byte bf16 that only the register-weight head reads,
    whose constant loads need out_w 16-byte aligned.  A C-ABI caller's misaligned out_w is an error with a
    message, never a fall-through to a head that reads the b2 tensor as fp32"""
    from toycrystals_amd import _lib
    from toycrystals_amd.models.sde_score_model import CondUNetTiny
    torch.manual_seed(0)
    m = CondUNetTiny(4, 4, 96).cuda().eval()
    B, H = 1, 256
    x = torch.randn(B, 1, H, H, device="cuda")
    t = torch.full((B,), 0.5, device="cuda")
    yc = torch.zeros(B, dtype=torch.long, device="cuda")
    yv = torch.zeros(B, 4, device="cuda")
    prev = _lib.conv_precision()
    _lib.set_conv_precision("bf16")
    try:
        with torch.no_grad():
            good = m(x, t, yc, yv)  # aligned (the pack's own copy): runs
            pk = m.tcx_pack(x.device)
            keep = pk.net.out_w
            buf = torch.zeros(96 * 9 + 4, device="cuda")  # the head weights' size, one float past 16 B
            pk.net.out_w = buf.data_ptr() + 4
            try:
                with pytest.raises(_lib.TcxError, match="aligned"):
                    m(x, t, yc, yv)
            finally:
                pk.net.out_w = keep
            again = m(x, t, yc, yv)
    finally:
        _lib.set_conv_precision(prev)
    assert torch.equal(good, again)  # the library state is intact after the rejected call


def _b2_cm(t):
    """b2 NHWC [B, H, W, C] (int16 storage) -> chunk-major b2 planes [C/8][B*H*W][8]"""
    C = t.shape[-1]
    return t.reshape(-1, C // 8, 8).permute(1, 0, 2).contiguous()


@pytest.mark.parametrize("B,HW,C", [(2, 65536, 96), (3, 16384, 192)])
def test_b2_apply_chunk_major_equals_in_place(B, HW, C):
    """config 5's skip tensors (round 6): tcx_gn_apply_tab_b2_cm (b2 pre-norm source -> GroupNorm + SiLU ->
    chunk-major b2 planes) holds exactly the values of the in-place b2 apply, transposed into planes"""
    x = torch.from_numpy(bf(rng.standard_normal((B, HW, C)).astype(np.float32) * 3)).cuda()
    sc = torch.rand(B, C, device="cuda") + 0.5
    sh = torch.randn(B, C, device="cuda")
    y = to_b2(x)
    cm = torch.full((C // 8, B * HW, 8), -1, dtype=torch.int16, device="cuda")
    chk(L().tcx_gn_apply_tab_b2_cm(y.data_ptr(), cm.data_ptr(), B, HW, C, sc.data_ptr(), sh.data_ptr(), st()))
    chk(L().tcx_gn_apply_tab_b2(y.data_ptr(), y.data_ptr(), B, HW, C, sc.data_ptr(), sh.data_ptr(), 1, 1, st()))
    torch.cuda.synchronize()
    assert torch.equal(_b2_cm(y.reshape(B, HW, 1, C)), cm)


@pytest.mark.parametrize("B,C1,C2,H,co,ks,stride", [
    (2, 96, 0, 256, 96, 4, 2),     # ds1: k_conv4s2g slim, Wo = 128, source 1 chunk-major
    (2, 192, 0, 128, 192, 4, 2),   # ds2: Wo = 64 (RT = 2)
    (1, 96, 96, 256, 96, 3, 1),    # up1.net.0: k_conv3lb at 256-px rows, source 2 chunk-major
    (2, 192, 192, 128, 96, 3, 1),  # up2.net.0: 128-px rows, Cin 384
])
def test_b2_chunk_major_source_equals_pixel_major(B, C1, C2, H, co, ks, stride):
    """config 5 (round 6): tcx_conv2d_h2_pro with bf16 = 2 and a chunk-major b2 source (+16 source 1 on the
    downsample, +32 source 2 on the concat conv) gives bit-identical outputs and GroupNorm partials to the same
    b2 tensor pixel-major: the kernels stage the same bytes into the same LDS slots"""
    x1 = dev(nhwc(rng.standard_normal((B, C1, H, H))))
    x2 = dev(nhwc(rng.standard_normal((B, C2, H, H)))) if C2 else None
    w = (rng.standard_normal((co, C1 + C2, ks, ks)) / np.sqrt(ks * ks * (C1 + C2))).astype(np.float32)
    b = rng.standard_normal(co).astype(np.float32)
    wh, ws, cpad, kpad = pack_bf16(w)
    wf = pack_frag(wh, cpad, kpad, C1 + C2)
    s1, s2 = to_b2(x1), (to_b2(x2) if C2 else None)
    Ho = H // stride
    bd = dev(b)

    def run(a1, a2, flag):
        y = torch.empty((B, Ho, Ho, co), dtype=torch.int16, device="cuda")
        g = torch.zeros((B, Ho * Ho // 128, co, 2), dtype=torch.float64, device="cuda")
        p = lambda t: t.data_ptr() if t is not None else None  # noqa: E731
        chk(L().tcx_conv2d_h2_pro(a1.data_ptr(), p(a2), B, 0, H, H, C1, C2, wh.data_ptr(), p(wf), ws.data_ptr(),
                                  bd.data_ptr(), None, None, y.data_ptr(), 1, co, cpad, kpad, ks, stride, 1, 1, 0,
                                  g.data_ptr(), None, None, None, None, flag, None, st()))
        torch.cuda.synchronize()
        return y, g

    ya, ga = run(s1, s2, 2)
    yb, gb = run(_b2_cm(s1), None, 2 + 16) if C2 == 0 else run(s1, _b2_cm(s2), 2 + 32)
    nd = int((ya != yb).sum())
    print(f"b2 chunk-major {C1}+{C2}->{co} {ks}x{ks}/s{stride} at {H}^2: {nd} outputs differ")
    assert nd == 0 and torch.equal(ga, gb)


def test_b2_256px_forward_chunk_major_skips_bit_identical(tmp_path):
    """the whole 256^2 bf16 forward with the chunk-major b2 skip tensors (default, round 6) and with pixel-major
    skips (TCX_SKIP_CM=0), each in its own process: bit-identical eps (the skip layout changes where bytes
    come from, never the arithmetic)"""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = {}
    for v in ("3", "0"):
        path = str(tmp_path / f"e{v}.npy")
        env = dict(os.environ, TCX_SKIP_CM=v)
        r = subprocess.run([sys.executable, "-c", B2_CHILD, root, path], capture_output=True, text=True, timeout=300,
                           env=env)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
        out[v] = np.load(path)
    assert np.array_equal(out["3"], out["0"]), float(np.abs(out["3"] - out["0"]).max())



@pytest.fixture
def conv3mb_everywhere():
    """k_conv3mb on every b2 3x3 shape it covers (the default runs k_conv3lb everywhere)"""
    prev = L().tcx_debug_conv3mb(2)
    yield
    L().tcx_debug_conv3mb(prev)


@pytest.mark.parametrize("B,C1,C2,H,co", [
    (1, 96, 0, 256, 96),     # 256-px rows, one row per tile (down1_1 / up1_1 / us1)
    (1, 96, 96, 256, 96),    # two b2 sources (up1.net.0)
    (3, 96, 0, 128, 192),    # 128-px rows, two n blocks, odd batch (down2.net.0)
    (1, 192, 192, 128, 96),  # Cin 384 over two sources (up2.net.0)
    (2, 192, 0, 64, 192),    # 64-px rows (the mid block)
    (2, 192, 0, 128, 192),   # Cin 192: an even number of 9-pair periods (down2_1, us2)
])
def test_b2_conv3mb_vs_float64_on_rounded_operands(B, C1, C2, H, co, conv3mb_everywhere):
    """k_conv3mb (round 6: config 5's 3x3 convs on v_mfma_f32_16x16x32_bf16 tap pairs, three-slot weight
    ring) on b2 sources against float64 on the same bf16-rounded operands: only the fp32 accumulation
    differs (5e-6 of the output scale, as the k_conv3lb gate); GroupNorm partials against float64 sums of
    the fp32 output; the b2 output is the round-to-nearest-even of the fp32 output"""
    x1 = rng.standard_normal((B, C1, H, H)).astype(np.float32)
    x2 = rng.standard_normal((B, C2, H, H)).astype(np.float32) if C2 else None
    w = (rng.standard_normal((co, C1 + C2, 3, 3)) / np.sqrt(9 * (C1 + C2))).astype(np.float32)
    b = rng.standard_normal(co).astype(np.float32)
    y, g = _conv_fmt(dev(nhwc(x1)), dev(nhwc(x2)) if C2 else None, w, b, 3, 1, 2, False, gn=True)
    xin = bf(x1) if x2 is None else np.concatenate([bf(x1), bf(x2)], axis=1)
    ref = conv_ref(xin, bf(w), b, 1, 1)
    yn = nchw(y.cpu().numpy())
    err = float(np.abs(yn - ref).max()) / max(1.0, float(np.abs(ref).max()))
    yd = y.double().cpu().numpy().reshape(B, H * H // 128, 128, co)
    gs = np.stack([yd.sum(2), (yd * yd).sum(2)], -1)
    gerr = float(np.abs(g.cpu().numpy() - gs).max()) / max(1.0, float(np.abs(gs).max()))
    print(f"k_conv3mb B={B} {C1}+{C2}->{co} at {H}^2: {err:.2e} vs float64, GroupNorm partials {gerr:.2e}")
    assert err < 5e-6 and gerr < 1e-6
    y2, _ = _conv_fmt(dev(nhwc(x1)), dev(nhwc(x2)) if C2 else None, w, b, 3, 1, 2, True)
    assert torch.equal(b2_float(y2), y.to(torch.bfloat16).float())


@pytest.mark.parametrize("Bt,H,C1,C2,co", [(8, 256, 96, 0, 96), (4, 256, 96, 96, 96), (16, 128, 96, 0, 192),
                                            (32, 64, 192, 0, 192)])
def test_b2_conv3mb_repeats_bit_for_bit(Bt, H, C1, C2, co, conv3mb_everywhere):
    """k_conv3mb repeats bit for bit (b2 output and GroupNorm partials) into a NaN-filled output, six times"""
    g = torch.Generator(device="cuda").manual_seed(0)
    s1 = to_b2(torch.randn((Bt, H, H, C1), device="cuda", generator=g))
    s2 = to_b2(torch.randn((Bt, H, H, C2), device="cuda", generator=g)) if C2 else None
    w = (rng.standard_normal((co, C1 + C2, 3, 3)) / np.sqrt(9 * (C1 + C2))).astype(np.float32)
    wh, ws, cpad, kpad = pack_bf16(w)
    wf = pack_frag(wh, cpad, kpad, C1 + C2)
    bd = dev(rng.standard_normal(co).astype(np.float32))
    y = torch.empty((Bt, H, H, co), dtype=torch.int16, device="cuda")
    gn = torch.zeros((Bt, H * H // 128, co, 2), dtype=torch.float64, device="cuda")

    def run():
        y.fill_(-1)
        gn.zero_()
        chk(L().tcx_conv2d_h2_pro(s1.data_ptr(), s2.data_ptr() if s2 is not None else None, Bt, 0, H, H, C1, C2,
                                  wh.data_ptr(), wf.data_ptr(), ws.data_ptr(), bd.data_ptr(), None, None, y.data_ptr(),
                                  1, co, cpad, kpad, 3, 1, 1, 1, 0, gn.data_ptr(), None, None, None, None, 2, None,
                                  st()))
        torch.cuda.synchronize()
        return y.clone(), gn.clone()
    y0, g0 = run()
    assert not bool(torch.isnan(b2_float(y0)).any())
    bad = 0
    for _ in range(6):
        y1, g1 = run()
        bad += int((y1 != y0).sum()) + int((g1 != g0).sum())
    print(f"k_conv3mb Bt={Bt} {H}^2 {C1}+{C2}->{co}: 6 repeats, {bad} differing values")
    assert bad == 0



@pytest.mark.parametrize("B,C1,C2,H,co,ob2", [(1, 96, 0, 256, 96, 1), (1, 96, 96, 256, 96, 1), (2, 192, 0, 128, 192, 1),
                                              (1, 192, 192, 128, 96, 1), (2, 96, 0, 128, 96, 0), (2, 192, 0, 64, 192, 0)])
def test_b2_conv3mb_equals_conv3lb_bit_for_bit(B, C1, C2, H, co, ob2):
    """k_conv3mb (16x16x32 tap pairs) and k_conv3lb (32x32x16 taps) on the same b2 sources: the MFMAs sum the
    same bf16 products in the same k order (tap, then channel) into fp32, so the outputs are bit-identical —
    which is what lets the library pick either per layer; the GroupNorm partials are summed per lane in fp32 over
    different accumulator layouts (16x16 vs 32x32 blocks) before the fp64 fold: equal to fp32 rounding of those
    partial sums (the gate of test_b2_conv_equals_the_record_conv)"""
    x1 = dev(nhwc(rng.standard_normal((B, C1, H, H))))
    x2 = dev(nhwc(rng.standard_normal((B, C2, H, H)))) if C2 else None
    w = (rng.standard_normal((co, C1 + C2, 3, 3)) / np.sqrt(9 * (C1 + C2))).astype(np.float32)
    b = rng.standard_normal(co).astype(np.float32)
    out = {}
    for mode in (2, 0):
        prev = L().tcx_debug_conv3mb(mode)
        try:
            out[mode] = _conv_fmt(x1, x2, w, b, 3, 1, 2, bool(ob2), gn=True)
        finally:
            L().tcx_debug_conv3mb(prev)
    assert torch.equal(out[2][0], out[0][0])
    np.testing.assert_allclose(out[2][1].cpu().numpy(), out[0][1].cpu().numpy(), rtol=1e-5, atol=1e-3)
