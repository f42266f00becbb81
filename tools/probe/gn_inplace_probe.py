"""Probe: GroupNorm-apply (h2 writer) in place vs out of place on a 64^2 x 96 x 256 activation."""
import os, sys, statistics
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "vae-diffusion-toy-crystals_amd"))
import torch
from toycrystals_amd._lib import lib, check
L = lib()
st = torch.cuda.current_stream().cuda_stream
Bt, HW, C = 256, 4096, 96
x = torch.randn(Bt * HW * C, device="cuda")
y = torch.empty_like(x)
sc = torch.rand(Bt, C, device="cuda") + 0.5
sh = torch.randn(Bt, C, device="cuda")
def run(out):
    check(L.tcx_gn_apply_tab_h2(x.data_ptr(), out.data_ptr(), Bt, HW, C, sc.data_ptr(), sh.data_ptr(), 1, None, st))
for name, out in (("inplace", x), ("outofplace", y), ("inplace", x), ("outofplace", y)):
    for _ in range(3):
        run(out)
    ts = []
    for _ in range(20):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); run(out); e1.record(); e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    us = statistics.median(ts)
    print(f"{name:10s} {us:8.1f} us  {2 * x.numel() * 4 / us / 1e6:6.2f} TB/s", flush=True)
