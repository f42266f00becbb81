#!/usr/bin/env python3
"""Time config 5's 3x3 convs on 2-byte bf16 (b2) sources and outputs at their 256^2 / 128^2 / 64^2 layer shapes
(HIP events, median of REPS), on the kernel the library picks (k_conv3mb by default, k_conv3lb with
TCX_CONV3MB=0; TCX_CONV3MB=2 forces k_conv3mb on every shape), with the fraction of the 2.5 PFLOP/s dense bf16 peak.  usage (GPU box): python tools/mbbench.py"""
import os
import statistics
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "vae-diffusion-toy-crystals_amd")]
from test_gpu_bf16 import pack_bf16, pack_frag, to_b2  # noqa: E402
from test_gpu_ops import L, chk, dev, st  # noqa: E402

BT = int(os.environ.get("BT", "84"))
REPS = int(os.environ.get("REPS", "10"))
# name, H, C1, C2, Co, b2 output
SHAPES = [("down1_1 256", 256, 96, 0, 96, 1), ("up1_0 256", 256, 96, 96, 96, 1), ("down2_0 128", 128, 96, 0, 192, 1),
          ("down2_1 128", 128, 192, 0, 192, 1), ("up2_0 128", 128, 192, 192, 96, 1), ("up2_1 128 fp32", 128, 96, 0, 96, 0),
          ("mid_0 64", 64, 192, 0, 192, 1), ("mid_1 64 fp32", 64, 192, 0, 192, 0)]


def run(name, H, C1, C2, Co, ob2):
    g = torch.Generator(device="cuda").manual_seed(0)
    x1 = to_b2(torch.randn((BT, H, H, C1), device="cuda", generator=g))
    x2 = to_b2(torch.randn((BT, H, H, C2), device="cuda", generator=g)) if C2 else None
    w = (np.random.default_rng(1).standard_normal((Co, C1 + C2, 3, 3)) / np.sqrt(9 * (C1 + C2))).astype(np.float32)
    wh, ws, cpad, kpad = pack_bf16(w)
    wf = pack_frag(wh, cpad, kpad, C1 + C2)
    b = dev(np.zeros(Co, np.float32))
    y = torch.empty((BT, H, H, Co), dtype=torch.int16 if ob2 else torch.float32, device="cuda")
    gn = torch.zeros((BT, H * H // 128, Co, 2), dtype=torch.float64, device="cuda")

    def launch():
        chk(L().tcx_conv2d_h2_pro(x1.data_ptr(), x2.data_ptr() if x2 is not None else None, BT, 0, H, H, C1, C2,
                                  wh.data_ptr(), wf.data_ptr(), ws.data_ptr(), b.data_ptr(), None, None, y.data_ptr(),
                                  ob2, Co, cpad, kpad, 3, 1, 1, 1, 0, gn.data_ptr(), None, None, None, None, 2, None,
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
    fl = 2.0 * BT * H * H * Co * 9 * (C1 + C2)
    print(f"{name:16s} Bt={BT} {C1}+{C2}->{Co}: {us:8.1f} us  {fl / us / 1e6:7.1f} TFLOP/s  "
          f"{fl / us / 1e6 / 2500:.3f} of bf16 peak", flush=True)


if __name__ == "__main__":
    print("TCX_CONV3MB", os.environ.get("TCX_CONV3MB", "1"), "TCX_LB_RING", os.environ.get("TCX_LB_RING", "3"))
    for s in SHAPES:
        run(*s)
