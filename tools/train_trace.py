#!/usr/bin/env python3
"""Which convolutions of one score training step (CondUNetTiny(96), B = 128) run on the fp32 kernels
instead of the split path, and where the step's device copies come from.

Wraps functional._conv_fwd / _conv_wgrad / _conv_dgrad / tcx_conv_transpose2x to log shapes and
the path taken, then runs one step under torch.profiler and prints the aten copy-like ops with
their Python call sites.  usage: python tools/train_trace.py
"""
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vae-diffusion-toy-crystals_amd"))

import torch  # noqa: E402

from toycrystals_amd import functional as TF  # noqa: E402
from toycrystals_amd.optim import Adam, ema_update  # noqa: E402

LOG = []


def wrap(name, fn, describe):
    def w(*a, **k):
        LOG.append((name, describe(*a, **k)))
        return fn(*a, **k)
    return w


def d_fwd(x1, x2, wpk, kpad, cpad, b, bias_b, resid, Cout, ks, stride, pad, circular, out_hw=None, keep=None,
          xh=None):
    B, H, W, C1 = x1.shape
    C2 = 0 if x2 is None else x2.shape[3]
    Ho = (H + 2 * pad - ks) // stride + 1
    Wo = (W + 2 * pad - ks) // stride + 1
    split = TF._split_ok(x1, x2, C1, C2, ks, kpad, float(B) * Ho * Wo * Cout * ks * ks * (C1 + C2))
    return f"B{B} {H}x{W} C{C1}+{C2} -> {Cout} k{ks}s{stride} circ{circular} {'split' if split else 'FP32'}"


def d_wgrad(x1, x2, dy, Cout, ks, stride, pad, circular, xrec=None, dyrec=None):
    B, H, W, C1 = x1.shape
    C2 = 0 if x2 is None else x2.shape[3]
    split = TF._WGRAD_SPLIT and xrec is not None and Cout % 8 == 0
    return f"B{B} {H}x{W} C{C1}+{C2} -> {Cout} k{ks}s{stride} {'split' if split else 'FP32'}"


def d_dgrad(dy, w, C_lo, n_ci, stride, pad, circular, H, W, keep=None):
    return f"dy{tuple(dy.shape)} w{tuple(w.shape)} ci[{C_lo},{C_lo + n_ci}) s{stride}"


TF._conv_fwd = wrap("fwd", TF._conv_fwd, d_fwd)
TF._conv_wgrad = wrap("wgrad", TF._conv_wgrad, d_wgrad)
TF._conv_dgrad = wrap("dgrad", TF._conv_dgrad, d_dgrad)


def main():
    from toycrystals_amd.models.sde_score_model import CondUNetTiny, VPSDE, diffusion_loss_eps
    torch.manual_seed(0)
    B = 128
    model = CondUNetTiny(4, 4, 96).cuda().train()
    ema = CondUNetTiny(4, 4, 96).cuda()
    ema.load_state_dict(model.state_dict())
    sde = VPSDE(0.1, 30.0)
    opt = Adam(model.parameters(), lr=1e-4)
    x0 = torch.rand(B, 1, 64, 64, device="cuda")
    y_cat = (torch.arange(B, device="cuda") % 4).to(torch.int64)
    y_cont = torch.zeros(B, 4, device="cuda")

    def step():
        loss = diffusion_loss_eps(model, sde, x0, y_cat, y_cont, p_uncond=0.1)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
        ema_update(ema, model, 0.999)

    for _ in range(2):
        step()
    torch.cuda.synchronize()
    LOG.clear()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU], with_stack=True, record_shapes=True) as prof:
        step()
        torch.cuda.synchronize()
    print("== conv calls of one step (in order)")
    for name, d in LOG:
        print(f"  {name:6s} {d}")
    print("== aten ops of one step (count, self CPU us)")
    ev = prof.key_averages()
    rows = sorted(ev, key=lambda e: -e.count)
    for e in rows[:40]:
        print(f"  {e.count:5d}  {e.self_cpu_time_total:9.0f}  {e.key}")
    print("== call sites of copy-like ops")
    sites = collections.Counter()
    for e in prof.events():
        if e.name in ("aten::copy_", "aten::clone", "aten::contiguous", "aten::cat", "aten::to", "aten::_to_copy",
                      "aten::zeros", "aten::zero_", "aten::fill_", "aten::index", "aten::where", "aten::mul",
                      "aten::add", "aten::add_", "aten::sub", "aten::div"):
            st = [s for s in (e.stack or []) if "toycrystals_amd" in s or "train_trace" in s]
            sites[(e.name, st[0] if st else "?")] += 1
    for (n, s), c in sites.most_common(60):
        print(f"  {c:4d}  {n:18s} {s}")


if __name__ == "__main__":
    main()
