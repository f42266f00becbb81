"""numpy restatements of the ATen ops the reference's hot path calls (oracle; test-only).

Layout is NCHW like the reference.  `dt` is the compute dtype (np.float32 mirrors the
reference, np.float64 gives the fp64 restatement used to bound fp32 noise).
"""
from __future__ import annotations

import numpy as np
from numpy.lib.stride_tricks import sliding_window_view


def linear(x, w, b=None):
    """torch.nn.Linear: y = x W^T + b."""
    y = x @ w.T
    if b is not None:
        y = y + b
    return y


def silu(x):
    return x / (1.0 + np.exp(-x))


def relu(x):
    return np.maximum(x, 0)


def sigmoid(x):
    return 1.0 / (1.0 + np.exp(-x))


def conv2d(x, w, b, stride: int = 1, padding: int = 0, mode: str = "zeros"):
    """nn.Conv2d (groups=1, dilation=1).  mode 'circular' wraps (padding_mode='circular'),
    'zeros' zero-pads.  x [B,C,H,W], w [Co,C,kh,kw]."""
    if padding:
        pad = ((0, 0), (0, 0), (padding, padding), (padding, padding))
        x = np.pad(x, pad, mode="wrap" if mode == "circular" else "constant")
    kh, kw = w.shape[2], w.shape[3]
    win = sliding_window_view(x, (kh, kw), axis=(2, 3))[:, :, ::stride, ::stride]  # [B,C,Ho,Wo,kh,kw]
    B, C, Ho, Wo = win.shape[:4]
    cols = np.ascontiguousarray(win.transpose(0, 2, 3, 1, 4, 5)).reshape(B * Ho * Wo, C * kh * kw)
    y = cols @ w.reshape(w.shape[0], -1).T
    if b is not None:
        y = y + b
    return y.reshape(B, Ho, Wo, -1).transpose(0, 3, 1, 2)


def conv_transpose2d(x, w, b, stride: int = 2, padding: int = 1):
    """nn.ConvTranspose2d (groups=1, output_padding=0).  w [Cin,Cout,kh,kw].
    Restated as a zero-inserted input correlated with the flipped, transposed kernel."""
    B, C, H, W = x.shape
    kh = w.shape[2]
    up = np.zeros((B, C, (H - 1) * stride + 1, (W - 1) * stride + 1), dtype=x.dtype)
    up[:, :, ::stride, ::stride] = x
    p = kh - 1 - padding
    up = np.pad(up, ((0, 0), (0, 0), (p, p), (p, p)))
    wf = np.ascontiguousarray(w[:, :, ::-1, ::-1].transpose(1, 0, 2, 3))
    return conv2d(up, wf, b, stride=1, padding=0)


def group_norm(x, groups: int, weight, bias, eps: float = 1e-5):
    B, C = x.shape[:2]
    xr = x.reshape(B, groups, -1)
    mean = xr.mean(axis=2, keepdims=True)
    var = ((xr - mean) ** 2).mean(axis=2, keepdims=True)
    y = ((xr - mean) / np.sqrt(var + eps)).reshape(x.shape)
    shape = (1, C) + (1,) * (x.ndim - 2)
    return y * weight.reshape(shape) + bias.reshape(shape)


def layer_norm(x, weight, bias, eps: float = 1e-5):
    mean = x.mean(axis=-1, keepdims=True)
    var = ((x - mean) ** 2).mean(axis=-1, keepdims=True)
    return (x - mean) / np.sqrt(var + eps) * weight + bias


def upsample_bilinear2x(x):
    """nn.Upsample(scale_factor=2, mode='bilinear', align_corners=False):
    src = (dst + 0.5) / 2 - 0.5 clamped at 0, edge-clamped neighbour."""
    B, C, H, W = x.shape

    def axis_weights(n):
        dst = np.arange(2 * n)
        src = np.maximum((dst + 0.5) / 2.0 - 0.5, 0.0)
        i0 = np.floor(src).astype(np.int64)
        i1 = np.minimum(i0 + 1, n - 1)
        l1 = (src - i0).astype(x.dtype)
        return i0, i1, (1 - l1).astype(x.dtype), l1

    y0, y1, hy0, hy1 = axis_weights(H)
    x0, x1, wx0, wx1 = axis_weights(W)
    top = x[:, :, y0, :]
    bot = x[:, :, y1, :]
    rows = hy0[None, None, :, None] * (wx0 * top[:, :, :, x0] + wx1 * top[:, :, :, x1]) + \
        hy1[None, None, :, None] * (wx0 * bot[:, :, :, x0] + wx1 * bot[:, :, :, x1])
    return rows


def sdpa(q, k, v):
    """F.scaled_dot_product_attention without mask: softmax(q k^T / sqrt(d)) v."""
    d = q.shape[-1]
    s = (q @ np.swapaxes(k, -1, -2)) * (1.0 / np.sqrt(d)).astype(q.dtype)
    s = s - s.max(axis=-1, keepdims=True)
    p = np.exp(s)
    p = p / p.sum(axis=-1, keepdims=True)
    return p @ v
