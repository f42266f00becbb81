#!/usr/bin/env python3
"""Per-kernel roofline of one headline U-Net evaluation (base 96, 64x64, Bt = 256 = CFG-doubled B = 128:
the one-lane pass bench.py times) from a rocpd_layers.py table.

Each position is matched to its layer of CondUNetTiny.forward (sde_score_model.py:243-266) and given its
algorithmic work: 2 MACs per multiply-add for the convs (fp32-equivalent FLOP, priced against the f16x3
ceiling of 833 TFLOP/s = 2.5 PF / 3 products), and the bytes a pass must move at least (every tensor read
and written once, at its stored width) for the bandwidth kernels, priced against 8 TB/s.

usage: layer_roofline.py profiles/r05_g_layers.txt [out.txt]"""
import re
import sys

BT, C, C2 = 256, 96, 192
P0, P1, P2 = 64 * 64, 32 * 32, 16 * 16
F16X3_PEAK = 2500.0 / 3  # TFLOP/s fp32-equivalent
HBM_PEAK = 8.0  # TB/s


def conv(px, cin, cout, taps):
    return ("mfma", 2.0 * BT * px * cin * cout * taps)


def mem(nbytes):
    return ("hbm", float(nbytes))


E4 = 4  # fp32 / h2 record bytes per element
# (layer, work) in launch order; 'fin' = GroupNorm finalize (fp64 partials -> [Bt][C] tables)
LAYERS = [
    ("first: acf statistics", mem(BT * P0 * 4 // 2)),  # x_t is [B][H][W]: B = Bt/2 images read
    ("first: GroupNorm 0 sums", None),
    ("fin 0", None),
    ("down1.net.0 conv 1->96 + GN0 + SiLU -> records", mem(BT * P0 * C * E4)),
    ("down1.net.3 conv (down1_1)", conv(P0, C, C, 9)),
    ("fin 1", None),
    ("apply GN1+SiLU -> h2 (skip h1, chunk-major)", mem(2 * BT * P0 * C * E4)),
    ("ds1 4x4/s2", conv(P1, C, C, 16)),
    ("down2.net.0 conv (down2_0)", conv(P1, C, C2, 9)),
    ("fin 2", None),
    ("down2.net.3 conv, GN2 prologue (down2_1)", conv(P1, C2, C2, 9)),
    ("fin 3", None),
    ("apply GN3+SiLU -> h2 (skip h2, chunk-major)", mem(2 * BT * P1 * C2 * E4)),
    ("ds2 4x4/s2", conv(P2, C2, C2, 16)),
    ("mid.net.0 conv (mid_0)", conv(P2, C2, C2, 9)),
    ("fin 4", None),
    ("mid.net.3 conv, GN4 prologue (mid_1)", conv(P2, C2, C2, 9)),
    ("fin 5", None),
    ("apply GN5+SiLU (attention input, fp32)", mem(2 * BT * P2 * C2 * E4)),
    ("attn.norm statistics", mem(BT * P2 * C2 * E4)),
    ("fin 6", None),
    ("apply attn.norm -> h2", mem(2 * BT * P2 * C2 * E4)),
    ("attn qkv 1x1", conv(P2, C2, 3 * C2, 1)),
    ("attention (4 heads, d 48, N 256)", ("mfma", 2.0 * 2 * BT * 4 * P2 * P2 * (C2 // 4))),
    ("attn proj 1x1 + residual", conv(P2, C2, C2, 1)),
    ("us2 bilinear x2 -> h2", mem(BT * (P2 + P1) * C2 * E4)),
    ("us2 conv", conv(P1, C2, C2, 9)),
    ("up2.net.0 conv on cat (up2_0)", conv(P1, 2 * C2, C, 9)),
    ("fin 7", None),
    ("up2.net.3 conv, GN7 prologue (up2_1)", conv(P1, C, C, 9)),
    ("fin 8", None),
    ("us1 GN8+SiLU + bilinear x2 -> h2", mem(BT * (P1 + P0) * C * E4)),
    ("us1 conv", conv(P0, C, C, 9)),
    ("up1.net.0 conv on cat (up1_0)", conv(P0, 2 * C, C, 9)),
    ("fin 9", None),
    ("up1.net.3 conv, GN9 prologue (up1_1)", conv(P0, C, C, 9)),
    ("fin 10", None),
    ("head: GN10+SiLU + out conv channel sums", mem(BT * P0 * C * E4 + BT * 9 * P0 * 4)),
    ("sampler step (9-tap gather, CFG, EM, noise)", mem(BT * 9 * P0 * 4 + 3 * (BT // 2) * P0 * 4)),
]


# round 5: k_attn_prep replaces positions 18-21 (apply GN5, attn.norm statistics, finalize, apply)
ATTN4 = slice(18, 22)
ATTN_PREP = ("mid GN+SiLU + attn.norm stats/tables + records", mem(3 * BT * P2 * C2 * E4))


def main() -> int:
    rows = []
    for line in open(sys.argv[1]):
        m = re.match(r"\s*(\d+) (\S+).*?\s([\d.]+) us$", line.rstrip())
        if m:
            rows.append((int(m.group(1)), m.group(2), float(m.group(3))))
    global LAYERS
    if any(r[1].startswith("k_attn_prep") for r in rows):
        LAYERS = LAYERS[:ATTN4.start] + [ATTN_PREP] + LAYERS[ATTN4.stop:]
    if len(rows) != len(LAYERS):
        print(f"expected {len(LAYERS)} kernels per evaluation, got {len(rows)}", file=sys.stderr)
        return 1
    out = open(sys.argv[2], "w") if len(sys.argv) > 2 else sys.stdout
    conv_us = other_us = 0.0
    print(f"{'#':>2} {'layer':48s} {'kernel':28s} {'us':>7s} {'work':>12s} {'achieved':>14s} {'frac':>6s}", file=out)
    for (i, kname, us), (layer, work) in zip(rows, LAYERS):
        if work is None:
            ws, ach, frac = "-", "-", ""
        elif work[0] == "mfma":
            tf = work[1] / (us * 1e-6) / 1e12
            ws, ach, frac = f"{work[1] / 1e9:.1f} GFLOP", f"{tf:.0f} TFLOP/s", f"{tf / F16X3_PEAK:.3f}"
        else:
            tb = work[1] / (us * 1e-6) / 1e12
            ws, ach, frac = f"{work[1] / 1e6:.0f} MB", f"{tb:.2f} TB/s", f"{tb / HBM_PEAK:.3f}"
        is_conv = work is not None and work[0] == "mfma" and "attention" not in layer
        if is_conv:
            conv_us += us
        else:
            other_us += us
        print(f"{i:2d} {layer:48s} {kname[:28]:28s} {us:7.1f} {ws:>12s} {ach:>14s} {frac:>6s}", file=out)
    print(f"conv kernels {conv_us:.1f} us, everything else {other_us:.1f} us per evaluation", file=out)
    return 0


if __name__ == "__main__":
    sys.exit(main())
