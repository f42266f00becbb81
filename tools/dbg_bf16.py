#!/usr/bin/env python3
"""Bisect helper for the bf16 256x256 forward (tests/test_gpu_bf16.py::test_bf16_unet_forward_vs_reference):
runs the evaluator in bf16 three times against the committed golden, prints the error, whether the
runs agree bit for bit, and where the largest deviations sit.  usage (GPU box):
    python tools/dbg_bf16.py [--lib path/to/libtcx_variant.so] [--name unet96_b2_h256]"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vae-diffusion-toy-crystals_amd"), os.path.join(ROOT, "tests")]


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default="")
    ap.add_argument("--name", default="unet96_b2_h256")
    a = ap.parse_args()
    from toycrystals_amd import _lib
    if a.lib:
        _lib.LIB_PATH = os.path.abspath(a.lib)
    from test_gpu_models import cu, rel_err, unet
    g = dict(np.load(os.path.join(ROOT, "tests", "golden", a.name + ".npz"), allow_pickle=False))
    m = unet(96)
    _lib.set_conv_precision("bf16")
    outs = []
    for _ in range(3):
        with torch.no_grad():
            outs.append(m(cu(g["x_t"]), cu(g["t"]), cu(g["y_cat"]), cu(g["y_cont"])).cpu().numpy())
    ref = g["eps"]
    for i, e in enumerate(outs):
        d = np.abs(e - ref)
        idx = np.unravel_index(np.argmax(d), d.shape)
        big = np.argwhere(d > 0.05 * max(1.0, np.abs(ref).max()))
        print(f"run {i}: rel err {rel_err(e, ref):.3e}; max at {tuple(int(v) for v in idx)}; "
              f"{len(big)} elements > 5e-2; equal to run 0: {np.array_equal(e, outs[0])}")
        if len(big):
            ys, xs = big[:, 2], big[:, 3]
            print(f"   rows {ys.min()}..{ys.max()}, cols {xs.min()}..{xs.max()}, batches {sorted(set(big[:, 0].tolist()))}; "
                  f"row histogram (32-row bins) {np.bincount(ys // 32, minlength=8).tolist()}; "
                  f"col histogram {np.bincount(xs // 32, minlength=8).tolist()}")
    print("used", _lib.LIB_PATH)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
