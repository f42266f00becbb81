"""GPU: the configuration bench.py TIMES, pinned.

bench.py's `value` comes from the 300-step reverse SDE at base_ch 96, B = 128, CFG 1.5, t_end 0.005,
in-kernel Philox noise, on FOUR concurrent sampling lanes (tcx_set_sample_lanes(4): the batch as four
per-stream chains whose kernels co-run).  The golden / oracle sampler tests pin the one-lane sampler;
here the timed mode must reproduce it bit for bit at the full headline size, and the convs whose
only round-4 defect appeared under co-run (a 16-B store whose data VGPR hipcc rewrote across a
branch join, conv_common.hpp store_b128_guarded) must repeat bit for bit while other kernels run on
other streams (the scenario tools/determinism_probe.py --corun diagnosed).

Reference of the sampler: /root/reference/src/toycrystals/models/sde_score_model.py:507-569."""
import math

import numpy as np
import pytest
import torch

from test_gpu_h2 import pack_frag, pack_h2, to_h2
from test_gpu_ops import L, chk, dev, st

pytestmark = pytest.mark.gpu


def _bench_model_and_inputs(B=128):
    from toycrystals_amd.models.sde_score_model import CondUNetTiny, VPSDE
    torch.manual_seed(0)
    model = CondUNetTiny(n_types=4, y_cont_dim=4, base_ch=96).cuda().eval()
    y_cat = (torch.arange(B) % 4).cuda()
    y_cont = torch.zeros(B, 4)
    y_cont[:, 1] = torch.linspace(0.0, math.pi / 3.0, B)
    return model, VPSDE(beta_min=0.1, beta_max=30.0), y_cat, y_cont.cuda()


@pytest.mark.parametrize("x0_hat", [False, True], ids=["image", "x0_hat"])
def test_bench_sampler_four_lanes_equal_one_lane(x0_hat):
    """bench.py's run(): the timed 4-lane sampler equals the 1-lane sampler bit for bit, on the image
    the metric counts and on the unclamped projection (which sees every pixel of an untrained net)."""
    from toycrystals_amd._lib import conv_precision, used_conv_precision
    from toycrystals_amd.models.sde_score_model import sample_reverse_sde_euler_maruyama
    assert conv_precision() == "f16x3"  # bench.py's default precision
    model, sde, y_cat, y_cont = _bench_model_and_inputs()
    outs = {}
    try:
        for lanes in (4, 1):
            L().tcx_set_sample_lanes(lanes)
            outs[lanes] = sample_reverse_sde_euler_maruyama(model, sde, y_cat, y_cont, (128, 1, 64, 64), n_steps=300,
                                                            guidance_scale=1.5, t_end=0.005, seed=1_000_003,
                                                            elem_offset=0, return_x0_hat=x0_hat)
            assert used_conv_precision() == "f16x3"
    finally:
        L().tcx_set_sample_lanes(0)
    a, b = outs[4], outs[1]
    assert bool(torch.isfinite(a).all())
    n_diff = int((a != b).sum())
    print(f"300-step B=128 base-96 sampler ({'x0_hat' if x0_hat else 'image'}): 4 lanes vs 1 lane, "
          f"{n_diff} of {a.numel()} values differ; mean {float(a.mean()):.4f}")
    assert n_diff == 0


def _conv_setup(Bt, H, C1, C2, Co, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    x1 = to_h2(torch.randn((Bt, H, H, C1), device="cuda", generator=g))
    x2 = to_h2(torch.randn((Bt, H, H, C2), device="cuda", generator=g)) if C2 else None
    xf = torch.randn((Bt, H, H, C1), device="cuda", generator=g)
    w = (np.random.default_rng(seed + 1).standard_normal((Co, C1 + C2, 3, 3)) / np.sqrt(9 * (C1 + C2))).astype(np.float32)
    wh, ws, cpad, kpad = pack_h2(w)
    wf = pack_frag(wh, cpad, kpad, C1 + C2)
    b = dev(np.random.default_rng(seed + 2).standard_normal(Co).astype(np.float32))
    sc = torch.rand((Bt, C1), device="cuda", generator=g) + 0.5
    sh = torch.randn((Bt, C1), device="cuda", generator=g)
    return dict(x1=x1, x2=x2, xf=xf, wh=wh, ws=ws, wf=wf, cpad=cpad, kpad=kpad, b=b, sc=sc, sh=sh)


def _launch(s, Bt, H, C1, C2, Co, pro, y, gn, stream):
    """one sampler-shaped 3x3 conv: h2 sources (k_conv3m) or one fp32 source with the GroupNorm+SiLU
    prologue (the prologue conv of the evaluator)"""
    x1 = s["xf"] if pro else s["x1"]
    x2 = s["x2"] if (s["x2"] is not None and not pro) else None
    chk(L().tcx_conv2d_h2_pro(x1.data_ptr(), x2.data_ptr() if x2 is not None else None, Bt, 0, H, H, C1,
                              0 if pro else C2, s["wh"].data_ptr(), s["wf"].data_ptr(), s["ws"].data_ptr(),
                              s["b"].data_ptr(), None, None, y.data_ptr(), 0, Co, s["cpad"], s["kpad"], 3, 1, 1, 1, 0,
                              gn.data_ptr(), s["sc"].data_ptr() if pro else None, s["sh"].data_ptr() if pro else None,
                              None, None, 0, None, stream))


# the evaluator's layer shapes at Bt = 128 (one lane of bench.py's four carries 64 images = 128 rows):
# (H, C1, C2, Cout, prologue)
CORUN_SHAPES = [(64, 96, 0, 96, False), (64, 96, 96, 96, False), (32, 96, 0, 192, False),
                (32, 192, 192, 96, False), (16, 192, 0, 192, False),
                (64, 96, 0, 96, True), (32, 192, 0, 192, True), (32, 96, 0, 96, True), (16, 192, 0, 192, True)]


@pytest.mark.parametrize("H,C1,C2,Co,pro", CORUN_SHAPES,
                         ids=[f"{h}px_{a}+{b}to{c}{'_pro' if p else ''}" for h, a, b, c, p in CORUN_SHAPES])
def test_conv_repeats_bit_for_bit_under_corun(H, C1, C2, Co, pro):
    """The conv launched on one stream while a GroupNorm-prologue conv, a 4x4/s2 downsample and an h2
    conversion pass run on three other streams (what the sampler's lanes do to each other), ten
    times: output and GroupNorm partials equal to a solo launch bit for bit."""
    Bt = 128
    s = _conv_setup(Bt, H, C1, C2, Co)
    o = _conv_setup(Bt, 64, 96, 0, 96, seed=7)  # the co-running kernels' operands
    w4 = (np.random.default_rng(3).standard_normal((96, 96, 4, 4)) / np.sqrt(16 * 96)).astype(np.float32)
    wh4, ws4, cpad4, kpad4 = pack_h2(w4)
    wf4 = pack_frag(wh4, cpad4, kpad4, 96)
    ref = torch.empty((Bt, H, H, Co), device="cuda")
    refg = torch.zeros((Bt, H * H // 128 if H * H >= 128 else 1, Co, 2), dtype=torch.float64, device="cuda")
    _launch(s, Bt, H, C1, C2, Co, pro, ref, refg, st())
    torch.cuda.synchronize()
    assert bool(torch.isfinite(ref).all())
    s0, s1, s2, s3 = (torch.cuda.Stream() for _ in range(4))
    y, gg = torch.empty_like(ref), torch.zeros_like(refg)
    yp = torch.empty((Bt, 64, 64, 96), device="cuda")
    gp = torch.zeros((Bt, 32, 96, 2), dtype=torch.float64, device="cuda")
    yd = torch.empty((Bt, 32, 32, 96), device="cuda")
    xo = torch.empty_like(o["xf"])
    bad = 0
    for _ in range(10):
        y.fill_(float("nan"))
        torch.cuda.synchronize()
        for _ in range(2):
            _launch(o, Bt, 64, 96, 0, 96, True, yp, gp, s1.cuda_stream)
            chk(L().tcx_conv2d_h2_pro(o["x1"].data_ptr(), None, Bt, 0, 64, 64, 96, 0, wh4.data_ptr(), wf4.data_ptr(),
                                      ws4.data_ptr(), o["b"].data_ptr(), None, None, yd.data_ptr(), 0, 96, cpad4, kpad4,
                                      4, 2, 1, 1, 0, None, None, None, None, None, 0, None, s2.cuda_stream))
            chk(L().tcx_f32_to_h2(o["xf"].data_ptr(), xo.data_ptr(), o["xf"].numel(), None, s3.cuda_stream))
        _launch(s, Bt, H, C1, C2, Co, pro, y, gg, s0.cuda_stream)
        torch.cuda.synchronize()
        bad += int((y != ref).sum()) + int((gg != refg).sum())
    print(f"conv {H}x{H} {C1}+{C2}->{Co} {'prologue' if pro else 'h2'}: 10 co-run repeats, differing {bad}")
    assert bad == 0


@pytest.mark.parametrize("sampler,lanes", [("sde", 4), ("sde", 1), ("ode", 4)])
def test_sampler_error_path_then_correct_next_call(sampler, lanes):
    """An evaluation failing mid-loop (tcx_debug_fail_eval: the k-th evaluation after arming returns
    TCX_EINVAL) surfaces as an error of the sampling call; every lane stream has been joined back, so
    the same workspace serves the next call, which must equal a clean run bit for bit.  The
    conditioning tables live in the caller's workspace (tcx_sde/ode_workspace_size): the library
    allocates nothing."""
    from toycrystals_amd._lib import TcxError
    from toycrystals_amd.models.sde_score_model import (CondUNetTiny, VPSDE, sample_probability_flow_ode,
                                                        sample_reverse_sde_euler_maruyama)
    torch.manual_seed(0)
    m = CondUNetTiny(4, 4, 32).cuda().eval()
    B, steps = 8, 6
    y_cat = (torch.arange(B) % 4).cuda()
    y_cont = torch.rand(B, 4, generator=torch.Generator().manual_seed(2)).cuda()
    fn = sample_reverse_sde_euler_maruyama if sampler == "sde" else sample_probability_flow_ode
    kw = dict(img_shape=(B, 1, 64, 64), n_steps=steps, guidance_scale=1.5, t_end=0.005, seed=31, return_x0_hat=True)
    try:
        L().tcx_set_sample_lanes(lanes)
        clean = fn(m, VPSDE(0.1, 30.0), y_cat, y_cont, **kw)
        torch.cuda.synchronize()
        L().tcx_debug_fail_eval(3 * lanes + 2)  # mid-loop: step 3 (SDE) / stage 2 of step 1 (ODE)
        with pytest.raises(TcxError, match="injected failure"):
            fn(m, VPSDE(0.1, 30.0), y_cat, y_cont, **kw)
        torch.cuda.synchronize()
        again = fn(m, VPSDE(0.1, 30.0), y_cat, y_cont, **kw)
        torch.cuda.synchronize()
    finally:
        L().tcx_debug_fail_eval(0)
        L().tcx_set_sample_lanes(0)
    assert bool(torch.isfinite(clean).all())
    assert torch.equal(clean, again)


def test_sampler_workspace_is_sized_by_the_query_and_checked():
    """tcx_sde_workspace_size covers the U-Net workspace AND the conditioning tables (grows with the
    step count); one byte less is TCX_EWS (-4), before anything is launched."""
    import ctypes
    from toycrystals_amd.models.sde_score_model import CondUNetTiny, VPSDE, step_table
    torch.manual_seed(0)
    m = CondUNetTiny(4, 4, 32).cuda().eval()
    pk = m.tcx_pack()
    B, H = 4, 64
    n10 = int(L().tcx_sde_workspace_size(ctypes.byref(pk.net), B, H, H, 10, 1.5))
    n300 = int(L().tcx_sde_workspace_size(ctypes.byref(pk.net), B, H, H, 300, 1.5))
    unet = int(L().tcx_unet_workspace_size(ctypes.byref(pk.net), 2 * B, H, H))
    assert n300 > n10 > unet
    assert int(L().tcx_ode_workspace_size(ctypes.byref(pk.net), B, H, H, 10, 1.5)) > n10
    ws = torch.empty(n10, dtype=torch.uint8, device="cuda")
    x = torch.randn(B, 1, H, H, device="cuda")
    tab = step_table(VPSDE(0.1, 30.0), 10, 0.005).cuda()
    yc = torch.zeros(B, dtype=torch.int64, device="cuda")
    yv = torch.zeros(B, 4, device="cuda")
    rc = L().tcx_sde_sample_shard(ctypes.byref(pk.net), x.data_ptr(), yc.data_ptr(), yv.data_ptr(), B, H, H, 10, 1.5,
                                  tab.data_ptr(), None, 1, 0, 0, ws.data_ptr(), n10 - 1, st())
    assert rc == -4
    rc = L().tcx_sde_sample_shard(ctypes.byref(pk.net), x.data_ptr(), yc.data_ptr(), yv.data_ptr(), B, H, H, 10, 1.5,
                                  tab.data_ptr(), None, 1, 0, 0, ws.data_ptr(), n10, st())
    torch.cuda.synchronize()
    assert rc == 0 and bool(torch.isfinite(x).all())
