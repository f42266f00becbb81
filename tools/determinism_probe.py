#!/usr/bin/env python3
"""Bitwise determinism of the split-path convs and the sampler (diagnostic): the same launch repeated
must give identical bytes; the sampler's images for a batch must not depend on the batch they are
sampled in (shard semantics).  usage (GPU box): python tools/determinism_probe.py"""
import math
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "vae-diffusion-toy-crystals_amd")]
from test_gpu_h2 import pack_frag, pack_h2, to_h2  # noqa: E402
from test_gpu_ops import L, chk, dev, st  # noqa: E402


def conv_repeat(Bt, H, C1, C2, Co, reps=30):
    g = torch.Generator(device="cuda").manual_seed(0)
    x1 = to_h2(torch.randn((Bt, H, H, C1), device="cuda", generator=g))
    x2 = to_h2(torch.randn((Bt, H, H, C2), device="cuda", generator=g)) if C2 else None
    w = (np.random.default_rng(1).standard_normal((Co, C1 + C2, 3, 3)) / np.sqrt(9 * (C1 + C2))).astype(np.float32)
    wh, ws, cpad, kpad = pack_h2(w)
    wf = pack_frag(wh, cpad, kpad, C1 + C2)
    b = dev(np.random.default_rng(2).standard_normal(Co).astype(np.float32))
    outs = []
    for _ in range(reps):
        y = torch.full((Bt, H, H, Co), float("nan"), device="cuda")
        gn = torch.zeros((Bt, H * H // 128, Co, 2), dtype=torch.float64, device="cuda")
        chk(L().tcx_conv2d_h2_pro(x1.data_ptr(), x2.data_ptr() if x2 is not None else None, Bt, 0, H, H, C1, C2,
                                  wh.data_ptr(), wf.data_ptr(), ws.data_ptr(), b.data_ptr(), None, None, y.data_ptr(),
                                  0, Co, cpad, kpad, 3, 1, 1, 1, 0, gn.data_ptr(), None, None, None, None, 0, None,
                                  st()))
        outs.append((y.clone(), gn.clone()))
    torch.cuda.synchronize()
    bad = sum(int((o[0] != outs[0][0]).sum()) for o in outs[1:])
    badg = sum(int((o[1] != outs[0][1]).sum()) for o in outs[1:])
    nan = int(torch.isnan(outs[0][0]).sum())
    print(f"conv Bt={Bt} {H}x{H} {C1}+{C2}->{Co}: {reps} repeats, differing outputs {bad}, gn {badg}, NaN {nan}", flush=True)
    return bad + badg + nan


def conv_streams(Bt, H, C1, C2, Co, nstreams=4, reps=10):
    """the same conv launched on several streams at once (the sampler's lanes), each against a
    single-stream reference"""
    g = torch.Generator(device="cuda").manual_seed(0)
    x1 = to_h2(torch.randn((Bt, H, H, C1), device="cuda", generator=g))
    x2 = to_h2(torch.randn((Bt, H, H, C2), device="cuda", generator=g)) if C2 else None
    w = (np.random.default_rng(1).standard_normal((Co, C1 + C2, 3, 3)) / np.sqrt(9 * (C1 + C2))).astype(np.float32)
    wh, ws, cpad, kpad = pack_h2(w)
    wf = pack_frag(wh, cpad, kpad, C1 + C2)
    b = dev(np.random.default_rng(2).standard_normal(Co).astype(np.float32))

    def launch(y, gn, stream):
        chk(L().tcx_conv2d_h2_pro(x1.data_ptr(), x2.data_ptr() if x2 is not None else None, Bt, 0, H, H, C1, C2,
                                  wh.data_ptr(), wf.data_ptr(), ws.data_ptr(), b.data_ptr(), None, None, y.data_ptr(),
                                  0, Co, cpad, kpad, 3, 1, 1, 1, 0, gn.data_ptr(), None, None, None, None, 0, None,
                                  stream))
    ref = torch.empty((Bt, H, H, Co), device="cuda")
    refg = torch.zeros((Bt, H * H // 128, Co, 2), dtype=torch.float64, device="cuda")
    launch(ref, refg, st())
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream() for _ in range(nstreams)]
    ys = [torch.empty_like(ref) for _ in streams]
    gs = [torch.zeros_like(refg) for _ in streams]
    bad = 0
    for _ in range(reps):
        for s_, y, gg in zip(streams, ys, gs):
            launch(y, gg, s_.cuda_stream)
        torch.cuda.synchronize()
        bad += sum(int((y != ref).sum()) + int((gg != refg).sum()) for y, gg in zip(ys, gs))
    print(f"conv Bt={Bt} {H}x{H} {C1}+{C2}->{Co} on {nstreams} concurrent streams x {reps}: differing {bad}", flush=True)
    return bad


def conv_corun(reps=10, Bt=128, H=64, C=96, C2=0, Co=96):
    """k_conv3m (64x64, 96 -> 96) on one stream while OTHER kernels run on three more streams: the GN-prologue
    3x3 conv (k_conv3lg PRO 1), the 4x4/s2 conv (k_conv4s2g) and an h2 conversion pass"""
    g = torch.Generator(device="cuda").manual_seed(0)
    x1 = to_h2(torch.randn((Bt, H, H, C), device="cuda", generator=g))
    x2 = to_h2(torch.randn((Bt, H, H, C2), device="cuda", generator=g)) if C2 else None
    xf = torch.randn((Bt, H, H, C), device="cuda", generator=g)
    w = (np.random.default_rng(1).standard_normal((Co, C + C2, 3, 3)) / np.sqrt(9 * (C + C2))).astype(np.float32)
    wp = (np.random.default_rng(5).standard_normal((C, C, 3, 3)) / np.sqrt(9 * C)).astype(np.float32)
    w4 = (np.random.default_rng(3).standard_normal((C, C, 4, 4)) / np.sqrt(16 * C)).astype(np.float32)
    wh, ws, cpad, kpad = pack_h2(w)
    wf = pack_frag(wh, cpad, kpad, C + C2)
    whp, wsp, cpadp, kpadp = pack_h2(wp)
    wfp = pack_frag(whp, cpadp, kpadp, C)
    wh4, ws4, cpad4, kpad4 = pack_h2(w4)
    wf4 = pack_frag(wh4, cpad4, kpad4, C)
    b = dev(np.random.default_rng(2).standard_normal(C).astype(np.float32))
    sc = torch.rand((Bt, C), device="cuda") + 0.5
    sh = torch.randn((Bt, C), device="cuda")

    bo = dev(np.random.default_rng(2).standard_normal(Co).astype(np.float32))

    def conv3m(y, gn, stream):
        chk(L().tcx_conv2d_h2_pro(x1.data_ptr(), x2.data_ptr() if x2 is not None else None, Bt, 0, H, H, C, C2,
                                  wh.data_ptr(), wf.data_ptr(), ws.data_ptr(), bo.data_ptr(), None, None, y.data_ptr(),
                                  0, Co, cpad, kpad, 3, 1, 1, 1, 0, gn.data_ptr(), None, None, None, None, 0, None,
                                  stream))

    def pro(y, stream):
        chk(L().tcx_conv2d_h2_pro(xf.data_ptr(), None, Bt, 0, H, H, C, 0, whp.data_ptr(), wfp.data_ptr(), wsp.data_ptr(),
                                  b.data_ptr(), None, None, y.data_ptr(), 0, C, cpadp, kpadp, 3, 1, 1, 1, 0, None,
                                  sc.data_ptr(), sh.data_ptr(), None, None, 0, None, stream))

    def ds(y, stream):
        chk(L().tcx_conv2d_h2_pro(x1.data_ptr(), None, Bt, 0, H, H, C, 0, wh4.data_ptr(), wf4.data_ptr(),
                                  ws4.data_ptr(), b.data_ptr(), None, None, y.data_ptr(), 0, C, cpad4, kpad4, 4, 2, 1, 1,
                                  0, None, None, None, None, None, 0, None, stream))
    ref = torch.empty((Bt, H, H, Co), device="cuda")
    refg = torch.zeros((Bt, H * H // 128, Co, 2), dtype=torch.float64, device="cuda")
    conv3m(ref, refg, st())
    torch.cuda.synchronize()
    s0, s1, s2, s3 = (torch.cuda.Stream() for _ in range(4))
    y, gg = torch.empty_like(ref), torch.zeros_like(refg)
    yp = torch.empty((Bt, H, H, C), device="cuda")
    yd = torch.empty((Bt, H // 2, H // 2, C), device="cuda")
    xo = torch.empty_like(xf)
    bad = 0
    for _ in range(reps):
        for _ in range(3 if H > 16 else 1):
            pro(yp, s1.cuda_stream)
            ds(yd, s2.cuda_stream)
            chk(L().tcx_f32_to_h2(xf.data_ptr(), xo.data_ptr(), xf.numel(), None, s3.cuda_stream))
        conv3m(y, gg, s0.cuda_stream)
        torch.cuda.synchronize()
        d = (y != ref)
        nb_ = int(d.sum())
        bad += nb_ + int((gg != refg).sum())
        if nb_:
            idx = torch.nonzero(d.reshape(-1, Co))  # [pixel, channel]
            pix, ch = idx[:, 0], idx[:, 1]
            tile = pix // 256
            wv = (pix % 256) // 64
            rb = (pix % 64) // 16
            err = float((y - ref).abs().max())
            for t_ in torch.unique(tile)[:3].tolist():
                sel = tile == t_
                pl = (pix[sel] % 256).tolist()
                cl = ch[sel].tolist()
                pairs = sorted(set(zip(pl, cl)))
                print(f"    tile {t_}: {len(pairs)} elements; pixels {sorted(set(pl))}; channels {sorted(set(cl))}")
            print(f"  rep: {nb_} differing, tiles {torch.unique(tile).numel()} (first {torch.unique(tile)[:8].tolist()}), "
                  f"waves {torch.bincount(wv, minlength=4).tolist()}, row blocks {torch.bincount(rb, minlength=4).tolist()}, "
                  f"16-ch blocks {torch.bincount(ch // 16, minlength=6).tolist()}, max err {err:.3e}, "
                  f"pixels per differing tile {nb_ / max(1, torch.unique(tile).numel()) / Co:.1f}", flush=True)
    print(f"conv3m Bt={Bt} {H}x{H} {C}+{C2}->{Co} beside k_conv3lg-PRO1 / k_conv4s2g / h2 conversion on other streams x {reps}: differing {bad}",
          flush=True)
    return bad


def sampler_batches(lanes=1):
    from toycrystals_amd.models.sde_score_model import CondUNetTiny, VPSDE, sample_reverse_sde_euler_maruyama
    prev = L().tcx_set_sample_lanes(lanes)
    torch.manual_seed(0)
    m = CondUNetTiny(4, 4, 96).cuda().eval()
    sde = VPSDE(0.1, 30.0)
    G = 256
    yc = (torch.arange(G) % 4).cuda()
    yv = torch.zeros(G, 4)
    yv[:, 1] = torch.linspace(0, math.pi / 3, G)
    yv = yv.cuda()
    kw = dict(n_steps=3, guidance_scale=1.5, t_end=0.005, seed=1_000_003, return_x0_hat=True)
    full = sample_reverse_sde_euler_maruyama(m, sde, yc, yv, (G, 1, 64, 64), **kw)
    full2 = sample_reverse_sde_euler_maruyama(m, sde, yc, yv, (G, 1, 64, 64), **kw)
    half = torch.cat([sample_reverse_sde_euler_maruyama(m, sde, yc[r * 128:(r + 1) * 128], yv[r * 128:(r + 1) * 128],
                                                         (128, 1, 64, 64), elem_offset=r * 128 * 4096, **kw)
                      for r in range(2)])
    d1 = int((full != full2).sum())
    d2 = int((full != half).sum())
    per_img = (full != half).reshape(G, -1).sum(1)
    L().tcx_set_sample_lanes(prev)
    print(f"sampler x0_hat, {lanes} lanes: B=256 twice {d1} differing; B=256 vs 2 x 128 shards {d2} differing; "
          f"images affected {int((per_img > 0).sum())}: {torch.nonzero(per_img).flatten().tolist()[:40]}", flush=True)
    return d1 + d2


if __name__ == "__main__":
    n = 0
    if len(sys.argv) > 1 and sys.argv[1] == "--corun":
        n = 0
        for shp in ((128, 64, 96, 0, 96), (128, 64, 96, 96, 96), (128, 32, 96, 0, 192), (128, 32, 192, 192, 192),
                    (128, 16, 192, 0, 192)):
            n += conv_corun(20, *shp)
        print("deterministic" if n == 0 else "NONDETERMINISTIC")
        raise SystemExit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "--sampler-only":
        n = sampler_batches(4)
        print("deterministic" if n == 0 else "NONDETERMINISTIC")
        raise SystemExit(0)
    for shape in ((256, 64, 96, 0, 96), (256, 64, 96, 96, 96), (256, 32, 192, 192, 192), (256, 16, 192, 0, 192)):
        n += conv_repeat(*shape)
        n += conv_streams(*shape)
    n += sampler_batches(1)
    n += sampler_batches(4)
    print("deterministic" if n == 0 else "NONDETERMINISTIC")
