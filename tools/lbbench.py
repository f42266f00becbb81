#!/usr/bin/env python3
"""Time config 5's bf16 3x3 conv (k_conv3lb) at its 256^2 / 128^2 / 64^2 layer shapes (HIP events,
median of REPS) and the repeatability of each launch (NaN-filled output, bytes compared; WHERE=1 prints
where differences fall in the tile).  usage (GPU box): python tools/lbbench.py"""
import os
import statistics
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "vae-diffusion-toy-crystals_amd")]
from test_gpu_bf16 import pack_bf16, pack_frag, to_bf16_records  # noqa: E402
from test_gpu_ops import L, chk, dev, st  # noqa: E402

BT = int(os.environ.get("BT", "44"))
REPS = int(os.environ.get("REPS", "10"))
# name, H, C1, C2, Co
SHAPES = [("down1_1 256", 256, 96, 0, 96), ("up1_0 256", 256, 96, 96, 96), ("down2_0 128", 128, 96, 0, 192),
          ("down2_1 128", 128, 192, 0, 192), ("down3 64", 64, 192, 0, 192)]


def run(name, H, C1, C2, Co):
    g = torch.Generator(device="cuda").manual_seed(0)
    x1 = to_bf16_records(torch.randn((BT, H, H, C1), device="cuda", generator=g))
    x2 = to_bf16_records(torch.randn((BT, H, H, C2), device="cuda", generator=g)) if C2 else None
    w = (np.random.default_rng(1).standard_normal((Co, C1 + C2, 3, 3)) / np.sqrt(9 * (C1 + C2))).astype(np.float32)
    wh, ws, cpad, kpad = pack_bf16(w)
    wf = pack_frag(wh, cpad, kpad, C1 + C2)
    b = dev(np.zeros(Co, np.float32))
    y = torch.empty((BT, H, H, Co), device="cuda")
    gn = torch.zeros((BT, H * H // 128, Co, 2), dtype=torch.float64, device="cuda") if os.environ.get("GN", "1") == "1" else None

    def launch():
        chk(L().tcx_conv2d_h2_pro(x1.data_ptr(), x2.data_ptr() if x2 is not None else None, BT, 0, H, H, C1, C2,
                                  wh.data_ptr(), wf.data_ptr(), ws.data_ptr(), b.data_ptr(), None, None, y.data_ptr(),
                                  0, Co, cpad, kpad, 3, 1, 1, 1, 0, gn.data_ptr() if gn is not None else None, None, None, None, None, 1, None,
                                  st()))
    launch()
    torch.cuda.synchronize()
    ts = []
    for _ in range(REPS):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        launch()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    us = statistics.median(ts)
    # repeatability: the same launch into a NaN-filled output, bytes compared with the first
    ref = gn.clone() if gn is not None else None
    y.fill_(float("nan"))
    launch()
    y0 = y.clone()
    g0 = gn.clone() if gn is not None else None
    bad = 0
    for _ in range(int(os.environ.get("DET", "8"))):
        y.fill_(float("nan"))
        if gn is not None:
            gn.zero_()
        launch()
        torch.cuda.synchronize()
        dy = (y != y0)
        nb_ = int(dy.sum())
        bad += nb_ + (int((gn != g0).sum()) if gn is not None else 0)
        if nb_ and os.environ.get("WHERE", "0") == "1":
            idx = torch.nonzero(dy.reshape(-1, Co))
            pix, ch = idx[:, 0], idx[:, 1]
            tl = pix // 256
            pt = pix % 256
            rel = float((y - y0).abs().max() / y0.abs().max())
            print(f"   {nb_} differing (gn {int((gn != g0).sum()) if gn is not None else 0}), rel {rel:.2e}, tiles "
                  f"{torch.unique(tl).numel()}: wave {torch.bincount(pt // 64, minlength=4).tolist()} rt "
                  f"{torch.bincount((pt % 64) // 32, minlength=2).tolist()} row%32 "
                  f"{torch.bincount(pt % 32, minlength=32).tolist()} n {torch.bincount(ch // 32, minlength=Co // 32).tolist()} "
                  f"ch%32 {torch.bincount(ch % 32, minlength=32).tolist()}", flush=True)
            t0 = int(tl[0])
            sel = tl == t0
            print(f"   tile {t0}: pixels {sorted(set(pt[sel].tolist()))[:40]} channels {sorted(set(ch[sel].tolist()))[:40]}", flush=True)
    nan = int(torch.isnan(y0).sum())
    del ref
    fl = 2.0 * BT * H * H * Co * 9 * (C1 + C2)
    print(f"{name:14s} Bt={BT} {C1}+{C2}->{Co}: {us:8.1f} us  {fl / us / 1e6:7.1f} TFLOP/s  "
          f"{fl / us / 1e6 / 2500:.3f} of bf16 peak; repeat differing {bad}, NaN {nan}", flush=True)


if __name__ == "__main__":
    print("GN", os.environ.get("GN", "1"))
    for s in SHAPES:
        run(*s)
