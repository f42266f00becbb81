#!/usr/bin/env python3
"""Per-layer micro-benchmark of libtcx's implicit-GEMM conv at the U-Net's shapes (Bt=256).
Prints µs and algorithmic TFLOP/s per layer (HIP events, median of N reps).
H2=1: the f16x3 split conv (tcx_conv2d_h2) over h2 operands instead of the fp32-MFMA conv; with PRO=1
the single-source 3x3 layers at W >= 32 read fp32 + GroupNorm tables (k_conv3g's prologue).
LAYER=name selects one layer, REPS the repetitions; TCX_CONV3G=0 selects k_conv3p for the 3x3 layers."""
import ctypes, os, sys, statistics
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vae-diffusion-toy-crystals_amd"))
import torch
from toycrystals_amd._lib import lib, check

L = lib()
st = torch.cuda.current_stream().cuda_stream
Bt = int(os.environ.get("BT", "256"))
C = 96
# name, H(in), Cin1, Cin2, Cout, ks, stride, pad, ups
LAYERS = [("conv0", 64, 1, 0, C, 3, 1, 1, 0), ("down1_1", 64, C, 0, C, 3, 1, 1, 0), ("ds1", 64, C, 0, C, 4, 2, 1, 0),
          ("down2_0", 32, C, 0, 2 * C, 3, 1, 1, 0), ("down2_1", 32, 2 * C, 0, 2 * C, 3, 1, 1, 0),
          ("ds2", 32, 2 * C, 0, 2 * C, 4, 2, 1, 0), ("mid", 16, 2 * C, 0, 2 * C, 3, 1, 1, 0),
          ("qkv", 16, 2 * C, 0, 6 * C, 1, 1, 0, 0), ("proj", 16, 2 * C, 0, 2 * C, 1, 1, 0, 0),
          ("us2(ups)", 16, 2 * C, 0, 2 * C, 3, 1, 1, 1), ("us2(pre)", 32, 2 * C, 0, 2 * C, 3, 1, 1, 0),
          ("up2_0", 32, 2 * C, 2 * C, C, 3, 1, 1, 0), ("up2_1", 32, C, 0, C, 3, 1, 1, 0),
          ("us1(ups)", 32, C, 0, C, 3, 1, 1, 1), ("up1_0", 64, C, C, C, 3, 1, 1, 0), ("up1_1", 64, C, 0, C, 3, 1, 1, 0)]


def rup(v, a=32):
    return (v + a - 1) // a * a


def bench(name, H, C1, C2, Co, ks, s, pad, ups, reps=20, gn=os.environ.get("GN", "1") == "1"):
    Cin = C1 + C2
    kpad, cpad = rup(ks * ks * Cin), rup(Co)
    x1 = torch.randn(Bt, H, H, C1, device="cuda")
    x2 = torch.randn(Bt, H, H, C2, device="cuda") if C2 else None
    w = torch.randn(Co, Cin, ks, ks, device="cuda") / (Cin * ks * ks) ** 0.5
    wpk = torch.empty(cpad, kpad, device="cuda")
    check(L.tcx_pack_conv_weight(w.data_ptr(), wpk.data_ptr(), Co, Cin, ks, cpad, kpad, st))
    b = torch.randn(Co, device="cuda")
    Hi = 2 * H if ups else H
    Ho = (Hi + 2 * pad - ks) // s + 1
    y = torch.empty(Bt, Ho, Ho, Co, device="cuda")
    use_gn = gn and (Ho * Ho) % 128 == 0 and ks == 3
    use_pro = os.environ.get("PRO", "1") == "1" and Cin % 32 == 0 and C1 % 32 == 0 and not ups and (Ho * Ho) % 128 == 0
    tabs = [torch.rand(Bt, C1, device="cuda") + 0.5, torch.randn(Bt, C1, device="cuda")] if use_pro else []
    pro = [t.data_ptr() for t in tabs] + [None, None] if use_pro else [None] * 4
    g = torch.empty(Bt, max(1, Ho * Ho // 128), Co, 2, dtype=torch.float64, device="cuda") if use_gn else None
    if H2:
        if ups or C1 % 32:
            return None
        def h2(t):
            o = torch.empty_like(t)
            check(L.tcx_f32_to_h2(t.data_ptr(), o.data_ptr(), t.numel(), None, st))
            return o
        # PRO=1 (H2 mode): source 1 stays fp32 and k_conv3g applies GroupNorm+SiLU tables while staging
        h2pro = os.environ.get("PRO", "0") == "1" and ks == 3 and s == 1 and C2 == 0 and H >= 16
        hp = [t.data_ptr() for t in tabs[:2]] if (h2pro and use_pro) else [None, None]
        if hp[0] is None:
            x1 = h2(x1)
        x2 = h2(x2) if x2 is not None else None
        wh = torch.empty_like(wpk)
        ws = torch.empty(4, device="cuda")
        check(L.tcx_pack_conv_weight_h2(wpk.data_ptr(), wh.data_ptr(), ws.data_ptr(), cpad, kpad, st))

        nfb = int(L.tcx_conv_weight_h2_frag_bytes(cpad, Cin)) if (ks == 3 and os.environ.get("TCX_CONV3G", "1") != "0") else 0
        if ks == 4 and os.environ.get("FRAG4", "1") == "1":
            nfb = int(L.tcx_conv_weight_h2_frag4_bytes(cpad, Cin))
        wf = torch.empty(max(nfb // 4, 4), device="cuda")
        if nfb:
            pk = L.tcx_pack_conv_weight_h2_frag4 if ks == 4 else L.tcx_pack_conv_weight_h2_frag
            check(pk(wh.data_ptr(), wf.data_ptr(), cpad, kpad, Cin, st))
        wfp = wf.data_ptr() if nfb else None

        def run():
            check(L.tcx_conv2d_h2_pro(x1.data_ptr(), x2.data_ptr() if x2 is not None else None, Bt, 0, H, H, C1, C2,
                                      wh.data_ptr(), wfp, ws.data_ptr(), b.data_ptr(), None, None, y.data_ptr(), 0, Co,
                                      cpad, kpad, ks, s, pad, 1, 0, g.data_ptr() if g is not None else None, hp[0],
                                      hp[1], None, None, 0, None, st))
    else:
      def run():
        check(L.tcx_conv2d(x1.data_ptr(), x2.data_ptr() if x2 is not None else None, Bt, 0, H, H, C1, C2,
                           wpk.data_ptr(), b.data_ptr(), None, None, y.data_ptr(), Co, cpad, kpad, ks, s, pad, 1,
                           ups, 0, g.data_ptr() if g is not None else None, *pro, st))
    for _ in range(3):
        run()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); run(); e1.record(); e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    us = statistics.median(ts)
    fl = 2.0 * Bt * Ho * Ho * Co * ks * ks * Cin
    print(f"{name:10s} {H:3d}->{Ho:3d} {Cin:4d}->{Co:4d} k{ks}s{s} {us:9.1f} us {fl / us / 1e6:7.1f} TF", flush=True)
    return us, fl


H2 = os.environ.get("H2", "0") == "1"
only = os.environ.get("LAYER")
reps = int(os.environ.get("REPS", "20"))
tot_us = tot_fl = 0
for l in LAYERS:
    if only and l[0] != only:
        continue
    r = bench(*l, reps=reps)
    if r is None:
        continue
    us, fl = r
    if l[0] not in ("us2(pre)",):
        tot_us += us; tot_fl += fl
if tot_us:
    print(f"TOTAL {tot_us:.1f} us  {tot_fl / tot_us / 1e6:.1f} TF (mid counted once)")
