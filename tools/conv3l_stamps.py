#!/usr/bin/env python3
"""Per-workgroup phase timing of k_conv3l at the up1_1 shape (Bt=256, 64x64, 96 -> 96, h2 source):
run with TCX_CONV3L_DBG=1 (stamps) or 2 (stamps, no output stores).  Prints the launch span, the
per-workgroup prologue / tap-loop / epilogue durations and how much of each CU slot's time lies
between workgroups (dispatch gaps)."""
import ctypes
import os
import statistics
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vae-diffusion-toy-crystals_amd"))
import torch  # noqa: E402
from toycrystals_amd._lib import lib, check  # noqa: E402

L = lib()
st = torch.cuda.current_stream().cuda_stream
Bt, H, C = int(os.environ.get("BT", "256")), 64, 96
Cin = int(os.environ.get("CIN", "96"))
kpad, cpad = 9 * Cin, 96


def h2(t):
    o = torch.empty_like(t)
    check(L.tcx_f32_to_h2(t.data_ptr(), o.data_ptr(), t.numel(), None, st))
    return o


x1 = h2(torch.randn(Bt, H, H, Cin, device="cuda"))
w = torch.randn(C, Cin, 3, 3, device="cuda") / (Cin * 9) ** 0.5
wpk = torch.empty(cpad, kpad, device="cuda")
check(L.tcx_pack_conv_weight(w.data_ptr(), wpk.data_ptr(), C, Cin, 3, cpad, kpad, st))
wh = torch.empty_like(wpk)
ws = torch.empty(4, device="cuda")
check(L.tcx_pack_conv_weight_h2(wpk.data_ptr(), wh.data_ptr(), ws.data_ptr(), cpad, kpad, st))
wf = torch.empty(int(L.tcx_conv_weight_h2_frag_bytes(cpad, Cin)) // 4, device="cuda")
check(L.tcx_pack_conv_weight_h2_frag(wh.data_ptr(), wf.data_ptr(), cpad, kpad, Cin, st))
b = torch.randn(C, device="cuda")
y = torch.empty(Bt, H, H, C, device="cuda")
g = torch.empty(Bt, H * H // 128, C, 2, dtype=torch.float64, device="cuda")


def run():
    check(L.tcx_conv2d_h2_pro(x1.data_ptr(), None, Bt, 0, H, H, Cin, 0, wh.data_ptr(), wf.data_ptr(), ws.data_ptr(),
                              b.data_ptr(), None, None, y.data_ptr(), 0, C, cpad, kpad, 3, 1, 1, 1, 0, g.data_ptr(),
                              None, None, None, None, 0, None, st))


for _ in range(5):
    run()
ts = []
for _ in range(10):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(); run(); e1.record(); e1.synchronize()
    ts.append(e0.elapsed_time(e1) * 1e3)
print(f"launch {statistics.median(ts):.1f} us (median of 10, events)")
n = Bt * H * H // 256
buf = (ctypes.c_ulonglong * (n * 5))()
check(L.tcx_conv3l_stamps(ctypes.cast(buf, ctypes.c_void_p), n))
S = [[buf[i * 5 + k] for k in range(5)] for i in range(n)]
t0 = min(s[0] for s in S)
us = lambda v: (v - t0) / 100.0  # noqa: E731  (100 MHz ticks -> us)
span = max(s[3] for s in S) - t0
print(f"stamped span {span / 100:.1f} us over {n} workgroups")
pro = [(s[1] - s[0]) / 100 for s in S]
loop = [(s[2] - s[1]) / 100 for s in S]
epi = [(s[3] - s[2]) / 100 for s in S]
for nm, v in (("prologue", pro), ("taps", loop), ("epilogue", epi)):
    v = sorted(v)
    print(f"{nm:9s} median {v[len(v) // 2]:7.2f} us  p10 {v[len(v) // 10]:7.2f}  p90 {v[9 * len(v) // 10]:7.2f}")
# per CU (xcc, se, sh, cu): workgroups in start order; busy = sum of workgroup lifetimes over 2 slots
cus = defaultdict(list)
for s in S:
    hw, xcc = s[4] & 0xffffffff, s[4] >> 32
    key = (xcc, (hw >> 13) & 7, (hw >> 12) & 1, (hw >> 8) & 15)
    cus[key].append(s)
occ, gaps, rounds = [], [], []
for key, L_ in cus.items():
    L_.sort(key=lambda s: s[0])
    life = sum(s[3] - s[0] for s in L_)
    first, last = min(s[0] for s in L_), max(s[3] for s in L_)
    occ.append(life / (2 * (last - first)))
    rounds.append(len(L_))
    # gap between a workgroup's exit and the start of the next workgroup on this CU
    ends = sorted(s[3] for s in L_)
    starts = sorted(s[0] for s in L_)[2:]
    for st_ in starts:
        prev = max([e for e in ends if e <= st_] or [st_])
        gaps.append((st_ - prev) / 100)
print(f"CUs {len(cus)}  workgroups per CU {min(rounds)}-{max(rounds)}  slot occupancy median {statistics.median(occ):.3f}")
if gaps:
    gaps.sort()
    print(f"dispatch gap median {gaps[len(gaps) // 2]:.2f} us  p90 {gaps[9 * len(gaps) // 10]:.2f}")
# phase alignment of the two slots of a CU: |start difference| of consecutive workgroups
d = []
for L_ in cus.values():
    st_ = sorted(s[0] for s in L_)
    d += [(st_[i + 1] - st_[i]) / 100 for i in range(0, len(st_) - 1, 2)]
d.sort()
print(f"start offset of paired slots median {d[len(d) // 2]:.2f} us  p90 {d[9 * len(d) // 10]:.2f}")
# timeline: how many workgroups are in their tap loop vs elsewhere, in 2-us bins
nb = int(span / 200) + 1
inloop, other = [0] * nb, [0] * nb
for s in S:
    for k in range(nb):
        a, b_ = t0 + k * 200, t0 + (k + 1) * 200
        ov = max(0, min(b_, s[2]) - max(a, s[1]))
        inloop[k] += ov / 200
        ov2 = max(0, min(b_, s[3]) - max(a, s[0])) - ov
        other[k] += ov2 / 200
print("2-us bins: mean workgroups in the tap loop / in prologue+epilogue (512 slots)")
print(" ".join(f"{a:.0f}/{o:.0f}" for a, o in zip(inloop, other)))
