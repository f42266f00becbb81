"""Autograd Functions over libtcx: the training path of the three models.

Each Function's forward and backward run HIP kernels from libtcx (include/tcx.h); torch only
allocates tensors, orders work on the current stream and chains the Functions (autograd).
Activations are NHWC fp32 contiguous ([B, H, W, C]); parameters keep the reference's layouts
(nn.Conv2d [Cout][Cin][k][k], nn.ConvTranspose2d [Cin][Cout][k][k], nn.Linear [out][in]) so the
gradients land in `.grad` exactly where torch.optim / the reference's checkpoints expect them.

Reference ops mirrored (file:line in /root/reference):
  nn.Conv2d circular / zero       src/toycrystals/models/sde_score_model.py:102-105,133-134,208-225; models/vae.py:19-26
  nn.ConvTranspose2d              models/vae.py:35-42
  nn.GroupNorm (+ SiLU)           sde_score_model.py:103-105,150
  nn.Upsample bilinear x2         sde_score_model.py:217-222
  SDPA                            sde_score_model.py:150-157
  nn.Linear / SiLU / ReLU / Sigmoid / nn.Embedding / nn.LayerNorm / FiLM   (all three models)
  F.mse_loss                      sde_score_model.py:399
"""
from __future__ import annotations

import ctypes
import math
import os
from typing import Optional

import torch

from ._lib import check, lib, ptr, stream_ptr

ACT_RELU, ACT_SIGMOID, ACT_SILU = 1, 2, 3

_WS = {}


def _ws(device: torch.device, nbytes: int) -> torch.Tensor:
    """Grow-only per-device scratch (stream-ordered reuse: every user runs on the current stream)."""
    key = torch.device(device)
    t = _WS.get(key)
    if t is None or t.numel() < nbytes:
        t = torch.empty(max(int(nbytes), 1 << 20), dtype=torch.uint8, device=key)
        _WS[key] = t
    return t


def _rup(v: int, a: int = 32) -> int:
    return (v + a - 1) // a * a


def _st(t: torch.Tensor) -> int:
    return stream_ptr(t.device)


def _empty(shape, like: torch.Tensor) -> torch.Tensor:
    return torch.empty(shape, device=like.device, dtype=torch.float32)


def _c(t: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
    return None if t is None else t.contiguous()


# ---------------------------------------------------------------- GEMM helper
def gemm(M, N, K, A, sa_m, sa_k, B, sb_k, sb_n, C, sc_m, sc_n, alpha=1.0, beta=0.0, bias=None, batch=1, bdiv=1,
         a_hl=(0, 0), b_hl=(0, 0), c_hl=(0, 0), a_off=0, b_off=0, c_off=0):
    """C = alpha A B + beta C (+ bias) through tcx_gemm_ws (split-K scratch when the shape wants it);
    offsets are in floats."""
    L = lib()
    nb = int(L.tcx_gemm_workspace(M, N, K, batch))
    ws = _ws(C.device, nb) if nb else None
    check(L.tcx_gemm_ws(M, N, K, float(alpha), ptr(A) + 4 * a_off, sa_m, sa_k, ptr(B) + 4 * b_off, sb_k, sb_n,
                        float(beta), ptr(C) + 4 * c_off, sc_m, sc_n, ptr(bias), batch, bdiv, a_hl[0], a_hl[1], b_hl[0],
                        b_hl[1], c_hl[0], c_hl[1], ptr(ws) if ws is not None else None, nb, _st(C)), "tcx_gemm")


def _colsum_total(x: torch.Tensor, rows: int, C: int) -> torch.Tensor:
    L = lib()
    out = _empty((C,), x)
    nb = int(L.tcx_colsum_workspace(1, rows, C))
    ws = _ws(x.device, nb)
    check(L.tcx_colsum(ptr(x), 1, rows, C, None, ptr(out), 0.0, ptr(ws), ws.numel(), _st(x)), "tcx_colsum")
    return out


def _colsum_per_batch(x: torch.Tensor, B: int, HW: int, C: int) -> torch.Tensor:
    L = lib()
    out = _empty((B, C), x)
    nb = int(L.tcx_colsum_workspace(B, HW, C))
    ws = _ws(x.device, nb)
    check(L.tcx_colsum(ptr(x), B, HW, C, ptr(out), None, 0.0, ptr(ws), ws.numel(), _st(x)), "tcx_colsum")
    return out


# ---------------------------------------------------------------- convolution
def _pack_conv(w: torch.Tensor):
    Cout, Cin, ks, _ = w.shape
    kpad, cpad = _rup(ks * ks * Cin), _rup(Cout)
    wpk = _empty((cpad, kpad), w)
    check(lib().tcx_pack_conv_weight(ptr(w), ptr(wpk), Cout, Cin, ks, cpad, kpad, _st(w)), "pack conv")
    return wpk, kpad, cpad


# Training convs on the f16x3 split path (csrc/h2.hpp) when the conv precision is f16x3 and the
# shape allows it (source channels % 32, a concat of equal halves, k*k <= 16): the operand (an
# activation in the forward, dY in the stride-1 data gradient) is converted to h2 after an exact
# power-of-two scaling from its max |value| (gradients sit far below the f16 normal range,
# activations can exceed its maximum), the weight is packed to h2 with its own power-of-two scale,
# and the conv epilogue applies the product of both inverse scales.  The weight gradient of the same
# convs runs split too (tcx_conv_wgrad_h2: x and dY scaled and converted).  TCX_TRAIN_SPLIT=0 keeps
# all of them on fp32 MFMA.
_TRAIN_SPLIT = os.environ.get("TCX_TRAIN_SPLIT", "1") != "0"


_SPLIT_MIN_MACS = 4e9  # below this the scaling / conversion launches cost more than the MFMA saves
_WGRAD_SPLIT = os.environ.get("TCX_WGRAD_FP32", "0") == "0"  # TCX_WGRAD_FP32=1: weight gradients on fp32 MFMA
_FRAG_TRAIN = os.environ.get("TCX_TRAIN_FRAG", "1") != "0"  # TCX_TRAIN_FRAG=0: training convs without the fragment copy (A/B)


def _split_ok(x1, x2, C1, C2, ks, kpad, macs) -> bool:
    from ._lib import conv_precision
    return (_TRAIN_SPLIT and conv_precision() == "f16x3" and macs >= _SPLIT_MIN_MACS and C1 % 32 == 0
            and C2 in (0, C1) and ks * ks <= 16 and kpad == ks * ks * (C1 + C2) and x1.numel() % 8 == 0
            and max(x1.numel(), 0 if x2 is None else x2.numel()) * 4 < (1 << 31))


_SLOT_INIT = {}
_SLOT_POOL = {}  # device -> [chunk of fresh slots, next free index]
_SLOT_CHUNK = 256


def _scale_slot(device) -> torch.Tensor:
    """A fresh [bits = 0][1.0][1/s] slot (int32 x 12, fields 16 B apart).  Slots are handed out of
    chunks of 256 initialised by one launch (a copy per slot cost 58 launches per score step); each
    slot is used once, and a chunk lives while any slot view of it does."""
    e = _SLOT_POOL.get(device)
    if e is None or e[1] >= _SLOT_CHUNK:
        t = _SLOT_INIT.get(device)
        if t is None:
            h = torch.zeros(12, dtype=torch.int32)
            h[4:5].view(torch.float32).fill_(1.0)
            t = _SLOT_INIT[device] = h.to(device)
        e = _SLOT_POOL[device] = [t.repeat(_SLOT_CHUNK), 0]
    i = e[1]
    e[1] = i + 1
    return e[0][12 * i:12 * i + 12]


def _absmax_slot_for(x: torch.Tensor, C: int) -> torch.Tensor | None:
    """A slot for a producer kernel to raise with max |x| (tcx_gn_apply_tab_absmax / tcx_gn_bwd_absmax)
    when a split training conv may consume x (f16x3, channels % 32, a conv above the split threshold)."""
    from ._lib import conv_precision
    if not (_TRAIN_SPLIT and C % 32 == 0 and 9.0 * x.numel() * C >= _SPLIT_MIN_MACS
            and conv_precision() == "f16x3"):
        return None
    return _scale_slot(x.device)


def _tag_absmax(x: torch.Tensor, sl) -> None:
    # consumed by _h2_scaled only while x is unchanged (same storage, same version counter: autograd's
    # in-place gradient accumulation bumps it)
    if sl is not None:
        x._tcx_amax = (sl, x._version, x.data_ptr())


def _tagged_slot(t: torch.Tensor):
    a = getattr(t, "_tcx_amax", None)
    if a is not None and a[1] == t._version and a[2] == t.data_ptr():
        return a[0]
    return None


def _h2_scaled(ts, mul=None):
    """fp32 tensors sharing ONE power-of-two scale s (max |s v| in [2^13, 2^14)) -> their h2 records
    and a 1-element float tensor holding 1/s (tcx_absmax + tcx_f32_to_h2_scaled).  A single tensor
    whose producer already reported its max |value| (_tag_absmax) skips the absmax pass.
    mul: a 1-element float tensor m; the returned scalar is then m / s, written by the conversion
    itself (the conv epilogue's combined scale without a separate multiply launch)."""
    L = lib()
    st = _st(ts[0])
    sl = _tagged_slot(ts[0]) if len(ts) == 1 else None
    pre = sl is not None
    if not pre:
        sl = _scale_slot(ts[0].device)  # [bits][1.0][1/s], 16 B apart
    elif mul is not None:
        # the producer's slot may still be read as 1/s by records made earlier: keep it, multiply apart
        hs, inv_t = _h2_scaled(ts)
        return hs, inv_t * mul
    bits, one, inv = ptr(sl), ptr(sl) + 16, ptr(sl) + 32
    for t in ts if not pre else ():
        check(L.tcx_absmax(ptr(t), t.numel(), bits, st), "tcx_absmax")
    hs = []
    for i, t in enumerate(ts):
        h = torch.empty_like(t)
        num = (ptr(mul) if mul is not None else one) if i == 0 else None
        check(L.tcx_f32_to_h2_scaled(ptr(t), ptr(h), t.numel(), bits, num, inv if i == 0 else None, st), "to h2")
        hs.append(h)
    return hs, sl[8:9].view(torch.float32)


def _conv_fwd_split(x1, x2, wpk, kpad, cpad, b, bias_b, resid, Cout, ks, stride, pad, circular, y, xh=None):
    """xh: (x1h, x2h, 1/s_x) already converted (the backward reuses the forward's / dgrad's records);
    returns y and the operand records for reuse."""
    L = lib()
    st = _st(x1)
    B, H, W, C1 = x1.shape
    C2 = 0 if x2 is None else x2.shape[3]
    if xh is None:
        hs, xinv = _h2_scaled([x1] if x2 is None else [x1, x2])
        xh = (hs[0], hs[1] if x2 is not None else None, xinv)
    x1h, x2h, xinv = xh
    # h2 of the packed weight (the layout of tcx_pack_conv_weight_h2) and comb = 1 / (s_w s_x), the
    # scale the conv epilogue applies, written by the weight's conversion launch
    (wh,), comb = _h2_scaled([wpk], mul=xinv)
    # fragment-ordered copy of the weight (round 3): the 3x3 convs then run on the LDS-DMA kernels of
    # the sampler (k_conv3lg / k_conv3g) and the 4x4/s2 ones on k_conv4s2g instead of the register-
    # staged k_conv3p / k_conv4s2h (the library picks; a shape they do not cover ignores the copy)
    wf = None
    if _FRAG_TRAIN and stride in (1, 2) and ks in (3, 4) and (ks == 3) == (stride == 1):
        Cin = C1 + C2
        nb = int(L.tcx_conv_weight_h2_frag_bytes(cpad, Cin) if ks == 3 else L.tcx_conv_weight_h2_frag4_bytes(cpad, Cin))
        if nb and kpad == ks * ks * Cin:
            wf = torch.empty(nb // 4, dtype=torch.float32, device=x1.device)
            pk = L.tcx_pack_conv_weight_h2_frag if ks == 3 else L.tcx_pack_conv_weight_h2_frag4
            check(pk(ptr(wh), ptr(wf), cpad, kpad, Cin, st), "pack frag")
    check(L.tcx_conv2d_h2_pro(ptr(x1h), ptr(x2h), B, 0, H, W, C1, C2, ptr(wh), ptr(wf), ptr(comb), ptr(b), ptr(bias_b),
                              ptr(resid), ptr(y), 0, Cout, cpad, kpad, ks, stride, pad, circular, 0, None, None, None,
                              None, None, 0, None, st), "tcx_conv2d_h2")
    return y, xh


def _conv_fwd(x1, x2, wpk, kpad, cpad, b, bias_b, resid, Cout, ks, stride, pad, circular, out_hw=None, keep=None,
              xh=None):
    """keep: a list that receives the split path's operand records (x1h, x2h, 1/s_x) when it runs;
    xh: records converted by the caller."""
    B, H, W, C1 = x1.shape
    C2 = 0 if x2 is None else x2.shape[3]
    Ho = (H + 2 * pad - ks) // stride + 1
    Wo = (W + 2 * pad - ks) // stride + 1
    y = _empty((B, Ho, Wo, Cout), x1)
    if _split_ok(x1, x2, C1, C2, ks, kpad, float(B) * Ho * Wo * Cout * ks * ks * (C1 + C2)):
        y, rec = _conv_fwd_split(x1, x2, wpk, kpad, cpad, b, bias_b, resid, Cout, ks, stride, pad, circular, y, xh)
        if keep is not None:
            keep.append(rec)
        return y
    check(lib().tcx_conv2d(ptr(x1), ptr(x2), B, 0, H, W, C1, C2, ptr(wpk), ptr(b), ptr(bias_b), ptr(resid), ptr(y),
                           Cout, cpad, kpad, ks, stride, pad, circular, 0, 0, None, None, None, None, None, _st(x1)),
          "tcx_conv2d")
    return y


def _conv_dgrad(dy, w, C_lo, n_ci, stride, pad, circular, H, W, keep=None):
    """Gradient w.r.t. input channels [C_lo, C_lo + n_ci) of a Conv2d with weight w [Cout][Cin][k][k].
    keep: [] to receive / [rec] to reuse dY's split-path records (dyh, None, 1/s_dy)."""
    L = lib()
    Cout, Cin, ks, _ = w.shape
    B = dy.shape[0]
    st = _st(dy)
    if stride == 1:
        kpad, cpad = _rup(ks * ks * Cout), _rup(n_ci)
        wpk = _empty((cpad, kpad), dy)
        check(L.tcx_pack_conv_dgrad_weight(ptr(w), ptr(wpk), Cout, Cin, ks, C_lo, n_ci, cpad, kpad, st), "pack dgrad")
        xh = keep[0] if keep else None
        dx = _conv_fwd(dy, None, wpk, kpad, cpad, None, None, None, n_ci, ks, 1, ks - 1 - pad, circular,
                       keep=keep if (keep is not None and not keep) else None, xh=xh)
        assert dx.shape[1] == H and dx.shape[2] == W
        return dx
    if stride == 2 and ks == 4 and pad == 1 and C_lo == 0 and n_ci == Cin:
        # adjoint of a stride-2 4x4 conv = ConvTranspose2d(4,2,1) with the same weight read as [in=Cout][out=Cin]
        kpad, cpad = _rup(4 * Cout), _rup(Cin)
        wpk = _empty((4, cpad, kpad), dy)
        check(L.tcx_pack_convT_weight(ptr(w), ptr(wpk), Cout, Cin, cpad, kpad, st), "pack convT")
        Hy, Wy = dy.shape[1], dy.shape[2]
        dx = _empty((B, 2 * Hy, 2 * Wy, Cin), dy)
        if _split_ok(dy, None, Cout, 0, 2, kpad, float(B) * 4 * Hy * Wy * Cin * 4 * Cout):
            # f16x3 (round 6): dY's records (made here or by an earlier data gradient, and reused by the
            # weight gradient) and the phase weights' records, comb = 1 / (s_w s_dy) from the conversion
            if keep:
                xh = keep[0]
            else:
                hs, inv = _h2_scaled([dy])
                xh = (hs[0], None, inv)
                if keep is not None:
                    keep.append(xh)
            (wh,), comb = _h2_scaled([wpk], mul=xh[2])
            check(L.tcx_conv_transpose2x_h2(ptr(xh[0]), B, Hy, Wy, Cout, ptr(wh), ptr(comb), None, ptr(dx), Cin, cpad,
                                            kpad, 0, circular, st), "tcx_conv_transpose2x_h2")
        else:
            check(L.tcx_conv_transpose2x(ptr(dy), B, Hy, Wy, Cout, ptr(wpk), None, ptr(dx), Cin, cpad, kpad, 0,
                                         circular, st), "tcx_conv_transpose2x")
        assert dx.shape[1] == H and dx.shape[2] == W
        return dx
    raise NotImplementedError(f"conv data gradient for stride={stride}, k={ks}, pad={pad}")


def _conv_wgrad(x1, x2, dy, Cout, ks, stride, pad, circular, xrec=None, dyrec=None):
    """xrec / dyrec: the split-path records (h2, h2 or None, 1/s) of x and dY when the forward / the
    data gradient made them: the weight gradient then runs f16x3 (tcx_conv_wgrad_h2) on them."""
    L = lib()
    B, H, W, C1 = x1.shape
    C2 = 0 if x2 is None else x2.shape[3]
    Ho, Wo = dy.shape[1], dy.shape[2]
    dw = _empty((Cout, C1 + C2, ks, ks), dy)
    nb = int(L.tcx_conv_wgrad_workspace(B, Ho, Wo, C1 + C2, Cout, ks))
    ws = _ws(dy.device, nb)
    if _WGRAD_SPLIT and xrec is not None and Cout % 8 == 0 and dy.numel() * 4 < (1 << 31):
        if dyrec is None:
            (dyh,), comb = _h2_scaled([dy], mul=xrec[2])
        else:
            dyh, _, dyinv = dyrec
            comb = xrec[2] * dyinv
        check(L.tcx_conv_wgrad_h2(ptr(xrec[0]), ptr(xrec[1]), B, H, W, C1, C2, ptr(dyh), Cout, ks, stride, pad,
                                  circular, 0.0, ptr(comb), ptr(dw), ptr(ws), ws.numel(), _st(dy)),
              "tcx_conv_wgrad_h2")
        return dw
    check(L.tcx_conv_wgrad(ptr(x1), ptr(x2), B, H, W, C1, C2, ptr(dy), Cout, ks, stride, pad, circular, 0.0, ptr(dw),
                           ptr(ws), ws.numel(), _st(dy)), "tcx_conv_wgrad")
    return dw


class Conv2dFn(torch.autograd.Function):
    """y = conv(cat[x1, x2]) + b (+ resid).  NHWC activations, weight [Cout][C1+C2][k][k]."""

    @staticmethod
    def forward(ctx, x1, x2, w, b, resid, stride: int, pad: int, circular: int):
        x1, x2, w, b, resid = _c(x1), _c(x2), _c(w), _c(b), _c(resid)
        Cout, Cin, ks, _ = w.shape
        wpk, kpad, cpad = _pack_conv(w)
        # the split forward's h2 records of x are kept for the weight gradient (one activation-sized
        # buffer per split conv until backward; INTEGRATION.md "Training memory note") unless the
        # weight gradients run on fp32 MFMA (TCX_WGRAD_FP32=1), which does not read them
        keep = [] if _WGRAD_SPLIT else None
        y = _conv_fwd(x1, x2, wpk, kpad, cpad, b, None, resid, Cout, ks, stride, pad, circular, keep=keep)
        ctx.save_for_backward(x1, x2, w)
        ctx.xrec = keep[0] if keep else None  # the split path's h2 records of x for the weight gradient
        ctx.cfg = (stride, pad, circular, b is not None, resid is not None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x1, x2, w = ctx.saved_tensors
        stride, pad, circular, has_b, has_r = ctx.cfg
        dy = dy.contiguous()
        Cout, Cin, ks, _ = w.shape
        B, H, W, C1 = x1.shape
        dx1 = dx2 = dw = db = dr = None
        dyrec = []  # dY's h2 records, made once by the first split data-gradient conv and reused
        if ctx.needs_input_grad[0]:
            dx1 = _conv_dgrad(dy, w, 0, C1, stride, pad, circular, H, W, keep=dyrec)
        if x2 is not None and ctx.needs_input_grad[1]:
            dx2 = _conv_dgrad(dy, w, C1, Cin - C1, stride, pad, circular, H, W, keep=dyrec)
        if ctx.needs_input_grad[2]:
            dw = _conv_wgrad(x1, x2, dy, Cout, ks, stride, pad, circular, xrec=ctx.xrec,
                             dyrec=dyrec[0] if dyrec else None)
        ctx.xrec = None
        if has_b and ctx.needs_input_grad[3]:
            db = _colsum_total(dy, dy.numel() // Cout, Cout)
        if has_r and ctx.needs_input_grad[4]:
            dr = dy
        return dx1, dx2, dw, db, dr, None, None, None


def conv2d(x1, x2, conv: torch.nn.Conv2d, resid=None):
    """nn.Conv2d (zeros or circular padding) on NHWC activations, optional channel concat [x1, x2]."""
    pad = conv.padding[0]
    circ = 1 if conv.padding_mode == "circular" else 0
    return Conv2dFn.apply(x1, x2, conv.weight, conv.bias, resid, conv.stride[0], pad, circ)


class ConvTranspose2xFn(torch.autograd.Function):
    """nn.ConvTranspose2d(k=4, s=2, p=1) (zero padding), weight [Cin][Cout][4][4] (vae.py:35-42)."""

    @staticmethod
    def forward(ctx, x, w, b):
        x, w, b = _c(x), _c(w), _c(b)
        L = lib()
        Cin, Cout = w.shape[0], w.shape[1]
        B, H, W, _ = x.shape
        kpad, cpad = _rup(4 * Cin), _rup(Cout)
        wpk = _empty((4, cpad, kpad), x)
        st = _st(x)
        check(L.tcx_pack_convT_weight(ptr(w), ptr(wpk), Cin, Cout, cpad, kpad, st), "pack convT")
        y = _empty((B, 2 * H, 2 * W, Cout), x)
        check(L.tcx_conv_transpose2x(ptr(x), B, H, W, Cin, ptr(wpk), ptr(b), ptr(y), Cout, cpad, kpad, 0, 0, st),
              "tcx_conv_transpose2x")
        ctx.save_for_backward(x, w)
        ctx.has_b = b is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dy = dy.contiguous()
        Cin, Cout = w.shape[0], w.shape[1]
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            # adjoint = Conv2d(4, 2, 1) over dy with w read as a conv weight [out=Cin][in=Cout]
            wpk, kpad, cpad = _pack_conv(w)
            dx = _conv_fwd(dy, None, wpk, kpad, cpad, None, None, None, Cin, 4, 2, 1, 0)
        if ctx.needs_input_grad[1]:
            # dW[ci][co][ky][kx] = wgrad of that conv with input dy and output gradient x
            dw = _conv_wgrad(dy, None, x, Cin, 4, 2, 1, 0)
        if ctx.has_b and ctx.needs_input_grad[2]:
            db = _colsum_total(dy, dy.numel() // Cout, Cout)
        return dx, dw, db


class FirstConvFn(torch.autograd.Function):
    """down1's first conv on cat([x_t, maps broadcast]) with the constant map channels folded
    into a per-(batch, channel) bias (sde_score_model.py:246; circular padding keeps a constant
    map constant).  x_t [B,H,W,1], maps [B,nm], w [C0][1+nm][3][3]."""

    @staticmethod
    def forward(ctx, x, maps, w, b):
        x, maps, w, b = _c(x), _c(maps), _c(w), _c(b)
        L = lib()
        st = _st(x)
        C0, cin, ks, _ = w.shape
        nm = cin - 1
        B = x.shape[0]
        bias_b = _empty((B, C0), x)
        check(L.tcx_first_conv_bias(ptr(maps), ptr(w), ptr(b), B, C0, nm, ks, ptr(bias_b), st), "first conv bias")
        w0 = _empty((C0, 1, ks, ks), x)
        check(L.tcx_copy2d(ptr(w), cin * ks * ks, ptr(w0), ks * ks, C0, ks * ks, 0.0, st), "copy2d")
        wpk, kpad, cpad = _pack_conv(w0)
        y = _conv_fwd(x, None, wpk, kpad, cpad, None, bias_b, None, C0, ks, 1, ks // 2, 1)
        ctx.save_for_backward(x, maps, w)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, maps, w = ctx.saved_tensors
        dy = dy.contiguous()
        L = lib()
        st = _st(dy)
        C0, cin, ks, _ = w.shape
        nm = cin - 1
        B, H, W, _ = dy.shape
        S = _colsum_per_batch(dy, B, H * W, C0)
        dwx = _conv_wgrad(x, None, dy, C0, ks, 1, ks // 2, 1) if ctx.needs_input_grad[2] else None
        dmaps = _empty((B, nm), dy) if ctx.needs_input_grad[1] else None
        dw = _empty(w.shape, dy) if ctx.needs_input_grad[2] else None
        db = _empty((C0,), dy) if ctx.needs_input_grad[3] else None
        check(L.tcx_first_conv_bwd(ptr(S), ptr(maps), ptr(w), ptr(dwx), B, C0, nm, ks, ptr(dmaps), ptr(dw), ptr(db),
                                   st), "first conv bwd")
        return None, dmaps, dw, db


# ---------------------------------------------------------------- GroupNorm (+SiLU)
class GroupNormActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, groups: int, eps: float, silu: int):
        x = x.contiguous()
        L = lib()
        st = _st(x)
        B, H, W, C = x.shape
        HW = H * W
        ns = max(1, HW // 512)
        part = torch.empty((B, ns, C, 2), device=x.device, dtype=torch.float64)
        check(L.tcx_gn_partials(ptr(x), B, HW, C, ns, ptr(part), st), "tcx_gn_partials")
        sc, sh = _empty((B, C), x), _empty((B, C), x)
        mean, rstd = _empty((B, groups), x), _empty((B, groups), x)
        check(L.tcx_gn_stats(ptr(part), B, HW, C, groups, ns, ptr(gamma), ptr(beta), float(eps), ptr(sc), ptr(sh),
                             ptr(mean), ptr(rstd), st), "tcx_gn_stats")
        y = torch.empty_like(x)
        sl = _absmax_slot_for(x, C)
        check(L.tcx_gn_apply_tab_absmax(ptr(x), ptr(y), B, HW, C, ptr(sc), ptr(sh), int(silu), ptr(sl), st),
              "tcx_gn_apply_tab")
        _tag_absmax(y, sl)
        ctx.save_for_backward(x, sc, sh, mean, rstd, gamma)
        ctx.cfg = (groups, int(silu))
        return y

    @staticmethod
    def backward(ctx, dy):
        x, sc, sh, mean, rstd, gamma = ctx.saved_tensors
        groups, silu = ctx.cfg
        dy = dy.contiguous()
        L = lib()
        B, H, W, C = x.shape
        dx = torch.empty_like(x)
        dg = _empty((C,), x) if ctx.needs_input_grad[1] else None
        dbt = _empty((C,), x) if ctx.needs_input_grad[2] else None
        nb = int(L.tcx_gn_bwd_workspace(B, H * W, C))
        ws = _ws(x.device, nb)
        sl = _absmax_slot_for(x, C)
        check(L.tcx_gn_bwd_absmax(ptr(x), ptr(dy), ptr(sc), ptr(sh), ptr(mean), ptr(rstd), ptr(gamma), B, H * W, C,
                                  groups, silu, ptr(dx), ptr(dg), ptr(dbt), ptr(sl), ptr(ws), ws.numel(), _st(x)),
              "tcx_gn_bwd")
        _tag_absmax(dx, sl)
        return dx, dg, dbt, None, None, None


def group_norm_act(x, gn: torch.nn.GroupNorm, silu: bool):
    return GroupNormActFn.apply(x, gn.weight, gn.bias, gn.num_groups, gn.eps, 1 if silu else 0)


# ---------------------------------------------------------------- upsample
class Upsample2xFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        x = x.contiguous()
        B, H, W, C = x.shape
        y = _empty((B, 2 * H, 2 * W, C), x)
        check(lib().tcx_upsample2x(ptr(x), ptr(y), B, H, W, C, None, None, _st(x)), "tcx_upsample2x")
        ctx.shape = (B, H, W, C)
        return y

    @staticmethod
    def backward(ctx, dy):
        B, H, W, C = ctx.shape
        dy = dy.contiguous()
        dx = _empty((B, H, W, C), dy)
        check(lib().tcx_upsample2x_bwd(ptr(dy), ptr(dx), B, H, W, C, _st(dy)), "tcx_upsample2x_bwd")
        return dx


# ---------------------------------------------------------------- attention
class AttentionFn(torch.autograd.Function):
    """SDPA over qkv [B, N, 3C] (q | k | v channel blocks, head h = channels h*d..h*d+d) -> [B, N, C]."""

    @staticmethod
    def forward(ctx, qkv, heads: int):
        qkv = qkv.contiguous()
        L = lib()
        B, N, C3 = qkv.shape
        C = C3 // 3
        d = C // heads
        scale = 1.0 / math.sqrt(d)
        S = _empty((B, heads, N, N), qkv)
        gemm(N, N, d, qkv, C3, 1, qkv, 1, C3, S, N, 1, alpha=scale, batch=B * heads, bdiv=heads,
             a_hl=(N * C3, d), b_hl=(N * C3, d), c_hl=(heads * N * N, N * N), b_off=C)
        P = torch.empty_like(S)
        check(L.tcx_softmax_rows(ptr(S), ptr(P), B * heads * N, N, _st(qkv)), "softmax")
        out = _empty((B, N, C), qkv)
        gemm(N, d, N, P, N, 1, qkv, C3, 1, out, C, 1, batch=B * heads, bdiv=heads,
             a_hl=(heads * N * N, N * N), b_hl=(N * C3, d), c_hl=(N * C, d), b_off=2 * C)
        ctx.save_for_backward(qkv, P)
        ctx.heads = heads
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, P = ctx.saved_tensors
        heads = ctx.heads
        dout = dout.contiguous()
        L = lib()
        B, N, C3 = qkv.shape
        C = C3 // 3
        d = C // heads
        scale = 1.0 / math.sqrt(d)
        z = B * heads
        dP = torch.empty_like(P)
        # dP = dO V^T
        gemm(N, N, d, dout, C, 1, qkv, 1, C3, dP, N, 1, batch=z, bdiv=heads, a_hl=(N * C, d), b_hl=(N * C3, d),
             c_hl=(heads * N * N, N * N), b_off=2 * C)
        dS = torch.empty_like(P)
        check(L.tcx_softmax_bwd_rows(ptr(P), ptr(dP), ptr(dS), z * N, N, _st(P)), "softmax bwd")
        dqkv = _empty((B, N, C3), qkv)
        # dQ = scale dS K
        gemm(N, d, N, dS, N, 1, qkv, C3, 1, dqkv, C3, 1, alpha=scale, batch=z, bdiv=heads,
             a_hl=(heads * N * N, N * N), b_hl=(N * C3, d), c_hl=(N * C3, d), b_off=C)
        # dK = scale dS^T Q
        gemm(N, d, N, dS, 1, N, qkv, C3, 1, dqkv, C3, 1, alpha=scale, batch=z, bdiv=heads,
             a_hl=(heads * N * N, N * N), b_hl=(N * C3, d), c_hl=(N * C3, d), c_off=C)
        # dV = P^T dO
        gemm(N, d, N, P, 1, N, dout, C, 1, dqkv, C3, 1, batch=z, bdiv=heads,
             a_hl=(heads * N * N, N * N), b_hl=(N * C, d), c_hl=(N * C3, d), c_off=2 * C)
        return dqkv, None


# ---------------------------------------------------------------- linear / activations / embedding
class LinearFn(torch.autograd.Function):
    """y = x W^T + b (+ resid), x [M][K] (row stride K), W [N][K], on the fp32-MFMA GEMM (tcx_gemm_ws;
    an f16x3 GEMM for these shapes measured slower per prior step and was removed)."""

    @staticmethod
    def forward(ctx, x, w, b, resid=None):
        x, w, b, resid = _c(x), _c(w), _c(b), _c(resid)
        M, K = x.shape
        N = w.shape[0]
        y = _empty((M, N), x)
        beta = 0.0
        if resid is not None:
            check(lib().tcx_copy2d(ptr(resid), N, ptr(y), N, M, N, 0.0, _st(x)), "copy2d")
            beta = 1.0
        gemm(M, N, K, x, K, 1, w, 1, K, y, N, 1, beta=beta, bias=b)
        ctx.save_for_backward(x, w)
        ctx.has = (b is not None, resid is not None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dy = dy.contiguous()
        M, K = x.shape
        N = w.shape[0]
        dx = dw = db = dr = None
        if ctx.needs_input_grad[0]:
            dx = _empty((M, K), dy)
            gemm(M, K, N, dy, N, 1, w, K, 1, dx, K, 1)
        if ctx.needs_input_grad[1]:
            dw = _empty((N, K), dy)
            gemm(N, K, M, dy, 1, N, x, K, 1, dw, K, 1)
        if ctx.has[0] and ctx.needs_input_grad[2]:
            db = _colsum_total(dy, M, N)
        if ctx.has[1] and ctx.needs_input_grad[3]:
            dr = dy
        return dx, dw, db, dr


def linear(x, m: torch.nn.Linear, resid=None):
    return LinearFn.apply(x, m.weight, m.bias, resid)


class ActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, z, act: int):
        z = z.contiguous()
        y = torch.empty_like(z)
        check(lib().tcx_act_fwd(ptr(z), ptr(y), z.numel(), act, _st(z)), "tcx_act_fwd")
        ctx.save_for_backward(z)
        ctx.act = act
        return y

    @staticmethod
    def backward(ctx, dy):
        (z,) = ctx.saved_tensors
        dy = dy.contiguous()
        dz = torch.empty_like(z)
        check(lib().tcx_act_bwd(ptr(z), ptr(dy), ptr(dz), z.numel(), ctx.act, _st(z)), "tcx_act_bwd")
        return dz, None


def act(z, kind: int):
    return ActFn.apply(z, kind)


class EmbeddingFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, idx, w):
        idx, w = idx.contiguous(), w.contiguous()
        B = idx.shape[0]
        E = w.shape[1]
        out = _empty((B, E), w)
        check(lib().tcx_embedding_fwd(ptr(idx), ptr(w), B, E, ptr(out), _st(w)), "tcx_embedding_fwd")
        ctx.save_for_backward(idx)
        ctx.rows = w.shape[0]
        return out

    @staticmethod
    def backward(ctx, dout):
        (idx,) = ctx.saved_tensors
        dout = dout.contiguous()
        B, E = dout.shape
        dw = _empty((ctx.rows, E), dout)
        check(lib().tcx_embedding_bwd(ptr(idx), ptr(dout), B, ctx.rows, E, ptr(dw), _st(dout)), "tcx_embedding_bwd")
        return None, dw


class CatColsFn(torch.autograd.Function):
    """torch.cat([a, b], dim=1) of 2-D feature rows (tcx_copy2d both ways)."""

    @staticmethod
    def forward(ctx, a, b):
        a, b = a.contiguous(), b.contiguous()
        M, Ka = a.shape
        Kb = b.shape[1]
        out = _empty((M, Ka + Kb), a)
        L = lib()
        st = _st(a)
        check(L.tcx_copy2d(ptr(a), Ka, ptr(out), Ka + Kb, M, Ka, 0.0, st), "copy2d")
        check(L.tcx_copy2d(ptr(b), Kb, ptr(out) + 4 * Ka, Ka + Kb, M, Kb, 0.0, st), "copy2d")
        ctx.k = (Ka, Kb)
        return out

    @staticmethod
    def backward(ctx, d):
        d = d.contiguous()
        Ka, Kb = ctx.k
        M = d.shape[0]
        L = lib()
        st = _st(d)
        da = _empty((M, Ka), d)
        db = _empty((M, Kb), d)
        check(L.tcx_copy2d(ptr(d), Ka + Kb, ptr(da), Ka, M, Ka, 0.0, st), "copy2d")
        check(L.tcx_copy2d(ptr(d) + 4 * Ka, Ka + Kb, ptr(db), Kb, M, Kb, 0.0, st), "copy2d")
        return da, db


def cat_cols(a, b):
    return CatColsFn.apply(a, b)


class TransposeBHCFn(torch.autograd.Function):
    """[B][R][C] -> [B][C][R] (NHWC <-> NCHW flatten order of the VAE FCs)."""

    @staticmethod
    def forward(ctx, x):
        x = x.contiguous()
        B, R, C = x.shape
        y = _empty((B, C, R), x)
        check(lib().tcx_transpose_bhc(ptr(x), ptr(y), B, R, C, _st(x)), "transpose")
        return y

    @staticmethod
    def backward(ctx, dy):
        dy = dy.contiguous()
        B, C, R = dy.shape
        dx = _empty((B, R, C), dy)
        check(lib().tcx_transpose_bhc(ptr(dy), ptr(dx), B, C, R, _st(dy)), "transpose")
        return dx


# ---------------------------------------------------------------- LayerNorm (+FiLM)
class LayerNormFiLMFn(torch.autograd.Function):
    """y = LN(x) (* (1 + gm) + bt with gb = [gm | bt] [M][2W] when given)."""

    @staticmethod
    def forward(ctx, x, w, b, gb, eps: float):
        x, w, b, gb = _c(x), _c(w), _c(b), _c(gb)
        M, Wd = x.shape
        y = torch.empty_like(x)
        mean, rstd = _empty((M,), x), _empty((M,), x)
        check(lib().tcx_ln_fwd(ptr(x), ptr(y), M, Wd, ptr(w), ptr(b), ptr(gb), 2 * Wd, float(eps), ptr(mean),
                               ptr(rstd), _st(x)), "tcx_ln_fwd")
        ctx.save_for_backward(x, w, b, gb, mean, rstd)
        return y

    @staticmethod
    def backward(ctx, dh):
        x, w, b, gb = ctx.saved_tensors[:4]
        mean, rstd = ctx.saved_tensors[4:]
        dh = dh.contiguous()
        M, Wd = x.shape
        dx = torch.empty_like(x)
        dwrow, dbrow = torch.empty_like(x), torch.empty_like(x)
        dgb = _empty((M, 2 * Wd), x) if gb is not None else None
        check(lib().tcx_ln_bwd(ptr(x), ptr(dh), M, Wd, ptr(w), ptr(b), ptr(gb), 2 * Wd, ptr(mean), ptr(rstd), ptr(dx),
                               ptr(dwrow), ptr(dbrow), ptr(dgb), _st(x)), "tcx_ln_bwd")
        dw = _colsum_total(dwrow, M, Wd) if ctx.needs_input_grad[1] else None
        db = _colsum_total(dbrow, M, Wd) if ctx.needs_input_grad[2] else None
        return dx, dw, db, dgb, None


# ---------------------------------------------------------------- losses
class MSELossFn(torch.autograd.Function):
    """F.mse_loss(a, b) (mean); gradient w.r.t. a only (b is data)."""

    @staticmethod
    def forward(ctx, a, b):
        a, b = a.contiguous(), b.contiguous()
        out = _empty((), a)
        ws = _ws(a.device, 8192 + 256)
        check(lib().tcx_mse_loss(ptr(a), ptr(b), a.numel(), ptr(out), ptr(ws), ws.numel(), _st(a)), "tcx_mse_loss")
        ctx.save_for_backward(a, b)
        return out

    @staticmethod
    def backward(ctx, g):
        a, b = ctx.saved_tensors
        g = g.contiguous()
        da = torch.empty_like(a)
        check(lib().tcx_mse_bwd(ptr(a), ptr(b), a.numel(), ptr(g), ptr(da), _st(a)), "tcx_mse_bwd")
        return da, None


def mse_loss(a, b):
    return MSELossFn.apply(a, b)


class ReparamFn(torch.autograd.Function):
    """z = mu + exp(0.5 logvar) * eps (vae.py:57-60); eps is data."""

    @staticmethod
    def forward(ctx, mu, lv, eps):
        mu, lv, eps = mu.contiguous(), lv.contiguous(), eps.contiguous()
        z = torch.empty_like(mu)
        check(lib().tcx_reparam(ptr(mu), ptr(lv), ptr(eps), mu.numel(), ptr(z), _st(mu)), "tcx_reparam")
        ctx.save_for_backward(lv, eps)
        return z

    @staticmethod
    def backward(ctx, dz):
        lv, eps = ctx.saved_tensors
        dz = dz.contiguous()
        dmu, dlv = torch.empty_like(lv), torch.empty_like(lv)
        check(lib().tcx_reparam_bwd(ptr(lv), ptr(eps), ptr(dz), lv.numel(), ptr(dmu), ptr(dlv), 0.0, _st(lv)),
              "tcx_reparam_bwd")
        return dmu, dlv, None


class KLStatsFn(torch.autograd.Function):
    """(kl_used, kl_raw) of scripts/train_vae.py:17-36 (free bits in nats per latent dim)."""

    @staticmethod
    def forward(ctx, mu, lv, free_bits: float):
        mu, lv = mu.contiguous(), lv.contiguous()
        B, Z = mu.shape
        out = _empty((2,), mu)
        check(lib().tcx_vae_kl(ptr(mu), ptr(lv), B, Z, float(free_bits), ptr(out), _st(mu)), "tcx_vae_kl")
        ctx.save_for_backward(mu, lv)
        ctx.fb = float(free_bits)
        return out[0], out[1]

    @staticmethod
    def backward(ctx, g_used, g_raw):
        mu, lv = ctx.saved_tensors
        B, Z = mu.shape
        L = lib()
        st = _st(mu)
        dmu, dlv = torch.zeros_like(mu), torch.zeros_like(lv)
        for g, fb in ((g_used, ctx.fb), (g_raw, 0.0)):
            if g is None:
                continue
            g = g.reshape(1).contiguous().float()
            check(L.tcx_vae_kl_bwd(ptr(mu), ptr(lv), B, Z, fb, ptr(g), ptr(dmu), ptr(dlv), 1.0, st), "kl bwd")
        return dmu, dlv, None


def kl_stats(mu, logvar, free_bits: float = 0.0):
    return KLStatsFn.apply(mu, logvar, float(free_bits))
