#!/usr/bin/env python3
"""Timeline of one k_conv3m launch from its in-kernel stamps (tcx_debug_conv_stamps): per-workgroup
phase durations (prologue, tap loop, epilogue stores, GroupNorm partials), the in-kernel clock, the
dispatch rounds and how much of the launch the slots spend outside the tap loop.
usage (GPU box): python tools/conv3m_stamps.py [--layer down1_1|up1_0|up2_0|mid_0]"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "vae-diffusion-toy-crystals_amd")]
from test_gpu_h2 import pack_frag, pack_h2, to_h2  # noqa: E402
from test_gpu_ops import L, chk, dev, st  # noqa: E402

LAYERS = {  # Bt, H, C1, C2, Cout: the sampler's k_conv3m layers at B = 128 (CFG: Bt = 256)
    "down1_1": (256, 64, 96, 0, 96), "up1_0": (256, 64, 96, 96, 96), "down2_0": (256, 32, 96, 0, 192),
    "up2_0": (256, 32, 192, 192, 192), "mid_0": (256, 16, 192, 0, 192)}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--layer", default="down1_1", choices=sorted(LAYERS))
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    Bt, H, C1, C2, Co = LAYERS[a.layer]
    g = torch.Generator(device="cuda").manual_seed(0)
    x1 = to_h2(torch.randn((Bt, H, H, C1), device="cuda", generator=g))
    x2 = to_h2(torch.randn((Bt, H, H, C2), device="cuda", generator=g)) if C2 else None
    w = (np.random.default_rng(1).standard_normal((Co, C1 + C2, 3, 3)) / np.sqrt(9 * (C1 + C2))).astype(np.float32)
    wh, ws, cpad, kpad = pack_h2(w)
    wf = pack_frag(wh, cpad, kpad, C1 + C2)
    b = dev(np.zeros(Co, np.float32))
    y = torch.empty((Bt, H, H, Co), device="cuda")
    gn = torch.zeros((Bt, H * H // 128, Co, 2), dtype=torch.float64, device="cuda")
    ovf = torch.zeros(1, dtype=torch.int32, device="cuda")
    nwg = Bt * H * H // 256 * (cpad // 96)
    stamps = torch.zeros((nwg, 8), dtype=torch.int64, device="cuda")

    def launch():
        chk(L().tcx_conv2d_h2_pro(x1.data_ptr(), x2.data_ptr() if x2 is not None else None, Bt, 0, H, H, C1, C2,
                                  wh.data_ptr(), wf.data_ptr(), ws.data_ptr(), b.data_ptr(), None, None, y.data_ptr(),
                                  0, Co, cpad, kpad, 3, 1, 1, 1, 0, gn.data_ptr(), None, None, None, None, 0,
                                  ovf.data_ptr(), st()))
    for _ in range(20):
        launch()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(10):
        launch()
    ev1.record()
    torch.cuda.synchronize()
    ms = ev0.elapsed_time(ev1) / 10
    chk(L().tcx_debug_conv_stamps(ctypes.c_void_p(stamps.data_ptr()), nwg))
    launch()
    torch.cuda.synchronize()
    chk(L().tcx_debug_conv_stamps(None, 0))
    s = stamps.cpu().numpy().astype(np.int64)
    t0 = s[:, 0].min()
    rt = (s[:, :5] - t0) / 100.0  # us
    clk = (s[:, 6] - s[:, 5]) / ((s[:, 2] - s[:, 0]) / 100.0) / 1e3  # GHz (shader clock over the loop)
    pro, loop, epi, gnp = rt[:, 1] - rt[:, 0], rt[:, 2] - rt[:, 1], rt[:, 3] - rt[:, 2], rt[:, 4] - rt[:, 3]
    span = rt[:, 4].max()
    flop = 2.0 * Bt * H * H * Co * 9 * (C1 + C2)
    out = [f"layer {a.layer}: Bt {Bt}, {H}x{H}, Cin {C1}+{C2} -> {Co}; {nwg} workgroups; event time {ms * 1e3:.1f} us "
           f"({flop / ms / 1e9:.0f} TFLOP/s fp32-equivalent, {flop / ms / 1e9 / 833.3:.3f} of 833)",
           f"stamped launch span {span:.1f} us; in-loop clock median {np.median(clk):.3f} GHz",
           "phase (us)      p10      p50      p90     mean"]
    for nm, v in (("prologue", pro), ("tap loop", loop), ("epi stores", epi), ("gn partials", gnp),
                  ("whole WG", rt[:, 4] - rt[:, 0])):
        out.append(f"{nm:12s} {np.percentile(v, 10):8.2f} {np.percentile(v, 50):8.2f} {np.percentile(v, 90):8.2f} "
                   f"{v.mean():8.2f}")
    busy = (rt[:, 4] - rt[:, 0]).sum()
    out.append(f"slot occupancy: sum of WG lifetimes / (512 slots x span) = {busy / (512 * span):.3f}; "
               f"tap-loop share of lifetimes {loop.sum() / busy:.3f}")
    st_ = np.sort(rt[:, 0])
    gaps = np.diff(st_)
    out.append(f"start times: first {st_[0]:.2f}, 512th {st_[min(511, len(st_) - 1)]:.2f}, last {st_[-1]:.2f} us; "
               f"end of first round (min exit) {rt[:, 4].min():.2f} us")
    # co-residence: workgroups on one CU (HW_ID cu / sh / se bits + XCC)
    hw = s[:, 7]
    cu_key = ((hw >> 16) << 16) | (hw & 0xff00)
    keys, inv = np.unique(cu_key, return_inverse=True)
    out.append(f"distinct CUs seen {len(keys)}; workgroups per CU p50 {np.median(np.bincount(inv)):.0f}")
    # phase alignment of the two resident workgroups: for each CU, sort by start; pair consecutive
    dif = []
    for k in range(len(keys)):
        idx = np.where(inv == k)[0]
        starts = np.sort(rt[idx, 0])
        if len(starts) >= 4:
            dif.extend(np.diff(starts)[:6].tolist())
    if dif:
        out.append(f"start-to-start of consecutive WGs on one CU: p10 {np.percentile(dif, 10):.2f} p50 "
                   f"{np.percentile(dif, 50):.2f} p90 {np.percentile(dif, 90):.2f} us")
    txt = "\n".join(out)
    print(txt)
    if a.out:
        open(a.out, "w").write(txt + "\n")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
