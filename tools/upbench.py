#!/usr/bin/env python3
"""Micro-benchmark of the h2 upsample forms at the sampler's us1 / us2 shapes (Bt = 256): µs per call
(HIP events, median of REPS).  TCX_UPB selects the form (csrc/norm.hip); us1 also times the separate
fp32 GroupNorm apply pass + plain upsample it replaces."""
import os, statistics, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vae-diffusion-toy-crystals_amd"))
import torch
from toycrystals_amd._lib import lib, check

L = lib()
st = torch.cuda.current_stream().cuda_stream
reps = int(os.environ.get("REPS", "30"))


def t(fn):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); fn(); e1.record(); e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    return statistics.median(ts)


for name, B, H, C, tabs in [("us1", 256, 32, 96, True), ("us2", 256, 16, 192, False)]:
    x = torch.randn(B, H, H, C, device="cuda")
    y = torch.empty(B, 2 * H, 2 * H, C, device="cuda")
    sc = torch.rand(B, C, device="cuda") + 0.5
    sh = torch.randn(B, C, device="cuda")
    ovf = torch.zeros(4, dtype=torch.int32, device="cuda")
    s_, h_ = (sc.data_ptr(), sh.data_ptr()) if tabs else (None, None)
    us = t(lambda: check(L.tcx_upsample2x_h2(x.data_ptr(), y.data_ptr(), B, H, H, C, s_, h_, ovf.data_ptr(), st)))
    mb = (x.numel() + y.numel()) * 4 / 1e6
    print(f"{name} UPB={os.environ.get('TCX_UPB', 'default')} tables={tabs}: {us:8.1f} us  {mb / us:6.2f} TB/s", flush=True)
    if tabs:
        def sep():
            check(L.tcx_gn_apply_tab(x.data_ptr(), x.data_ptr(), B, H * H, C, sc.data_ptr(), sh.data_ptr(), 1, st))
            check(L.tcx_upsample2x_h2(x.data_ptr(), y.data_ptr(), B, H, H, C, None, None, ovf.data_ptr(), st))
        print(f"{name} UPB={os.environ.get('TCX_UPB', 'default')} apply pass + upsample: {t(sep):8.1f} us", flush=True)
