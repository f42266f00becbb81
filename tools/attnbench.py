#!/usr/bin/env python3
"""Micro-benchmark of the config-5 split attention (2-byte bf16 qkv / output, csrc/attention_split.hip) at one
84-row pass: Bt = 84, N = 4,096 tokens, C = 192, 4 heads (d = 48).  µs per launch (HIP events on the launch
stream, median of REPS).  TCX_ATTN_DEFER / TCX_ATTN_XCD select the variant (read once per process)."""
import os, statistics, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vae-diffusion-toy-crystals_amd"))
import torch
from toycrystals_amd._lib import lib, check

L = lib()
st = torch.cuda.current_stream().cuda_stream
reps = int(os.environ.get("REPS", "20"))
Bt, N, C, heads = 84, 4096, 192, 4
g = torch.Generator(device="cuda").manual_seed(0)
qkv = (torch.randn(Bt, N, 3 * C, device="cuda", generator=g) * 0.5).to(torch.bfloat16).view(torch.int16)
out = torch.empty(Bt, N, C, dtype=torch.int16, device="cuda")


def run():
    check(L.tcx_attention_split_b2(qkv.data_ptr(), out.data_ptr(), Bt, N, C, heads, st))


for _ in range(3):
    run()
ts = []
for _ in range(reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(); run(); e1.record(); e1.synchronize()
    ts.append(e0.elapsed_time(e1) * 1e3)
o = out.view(torch.bfloat16).float()
print(f"attn_b2 defer={os.environ.get('TCX_ATTN_DEFER', 'default')} pf2={os.environ.get('TCX_ATTN_PF2', 'default')} {statistics.median(ts):.1f} us "
      f"(min {min(ts):.1f}); out sum {o.sum().item():.6e} absmax {o.abs().max().item():.4f}")
