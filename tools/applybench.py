#!/usr/bin/env python3
"""HBM rate of the GroupNorm+SiLU apply pass that writes bf16 / h2 records (config 5's 256^2 shape by
default), in place and out of place, beside a torch float4 copy of the same bytes.
usage (GPU box): python tools/applybench.py [BT=44 HW=65536 C=96]"""
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "vae-diffusion-toy-crystals_amd")]
from test_gpu_ops import L, chk, st  # noqa: E402

BT = int(os.environ.get("BT", "44"))
HW = int(os.environ.get("HW", "65536"))
C = int(os.environ.get("C", "96"))
REPS = int(os.environ.get("REPS", "10"))


def timed(fn):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(REPS):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    return statistics.median(ts)


if __name__ == "__main__":
    x = torch.randn(BT, HW, C, device="cuda")
    y = torch.empty_like(x)
    sc = torch.rand(BT, C, device="cuda") + 0.5
    sh = torch.randn(BT, C, device="cuda")
    nb = 2 * x.numel() * 4
    for name, fn in (
            ("apply bf16 out of place", lambda: chk(L().tcx_gn_apply_tab_bf16(x.data_ptr(), y.data_ptr(), BT, HW, C, sc.data_ptr(),
                                                                               sh.data_ptr(), 1, st()))),
            ("apply bf16 in place", lambda: chk(L().tcx_gn_apply_tab_bf16(y.data_ptr(), y.data_ptr(), BT, HW, C, sc.data_ptr(),
                                                                           sh.data_ptr(), 1, st()))),
            ("torch copy", lambda: y.copy_(x))):
        us = timed(fn)
        print(f"{name:26s} Bt={BT} HW={HW} C={C}: {us:8.1f} us  {nb / us / 1e6:6.2f} TB/s (read + write)", flush=True)
