"""ctypes binding of libtcx.so (the C ABI in include/tcx.h).

The library is built in-tree (`make -C vae-diffusion-toy-crystals_amd/csrc`, or
`__graft_entry__.build()`).  There is NO fallback: if the library is missing or a call fails,
the caller gets an exception (the product path never routes through a CPU implementation).
torch is imported first so that libtcx binds to the HIP runtime torch already loaded
(same soname, libamdhip64.so.7) and shares its device allocations and streams.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must be loaded before libtcx: shared HIP runtime)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libtcx.so")

c_fp = ctypes.c_void_p
c_int = ctypes.c_int
c_float = ctypes.c_float
c_size = ctypes.c_size_t
c_u64 = ctypes.c_uint64
c_ll = ctypes.c_longlong

TCX_SCAL = 8
TCX_SAMPLE_X0_HAT = 1  # tcx_{sde,ode}_sample_ex flag: return the unclamped x0_hat


class TcxConv(ctypes.Structure):
    _fields_ = [("w", c_fp), ("b", c_fp), ("cin", c_int), ("cout", c_int), ("ks", c_int), ("kpad", c_int),
                ("cout_pad", c_int), ("wh", c_fp), ("wscale", c_fp), ("whf", c_fp)]


_CONV_NAMES = ["down1_0", "down1_1", "ds1", "down2_0", "down2_1", "ds2", "mid_0", "mid_1", "qkv", "proj", "us2",
               "up2_0", "up2_1", "us1", "up1_0", "up1_1"]


class TcxUnet(ctypes.Structure):
    _fields_ = ([(n, c_int) for n in ("base_ch", "emb_dim", "cond_ch", "time_ch", "n_types", "y_cont_dim", "heads")]
                + [(n, c_fp) for n in ("time_w1t", "time_b1", "time_w2t", "time_b2", "ttm_wt", "ttm_b", "tcm_wt",
                                       "tcm_b", "cat_emb", "cmlp_w1t", "cmlp_b1", "cmlp_w2t", "cmlp_b2", "cout_wt",
                                       "cout_b", "map_wsum")]
                + [(n, TcxConv) for n in _CONV_NAMES]
                + [("out_w", c_fp), ("out_b", c_float), ("gn_w", c_fp * 11), ("gn_b", c_fp * 11)]
                + [("precision", c_int), ("h2_ovf", c_fp)])


class TcxLinearW(ctypes.Structure):
    _fields_ = [("w", c_fp), ("b", c_fp), ("n", c_int), ("k", c_int), ("npad", c_int), ("kpad", c_int),
                ("wh", c_fp), ("winv", c_fp)]


class TcxPrior(ctypes.Structure):
    _fields_ = ([(n, c_int) for n in ("z_dim", "n_types", "y_cont_dim", "t_emb_dim", "width", "n_blocks",
                                      "y_cat_emb_dim")]
                + [("ln_eps", c_float), ("temb_freqs", c_fp), ("y_cat_emb", c_fp)]
                + [(n, TcxLinearW) for n in ("t_mlp0", "t_mlp2", "y_cont0", "y_cont2", "y_fuse0", "y_fuse2",
                                             "in_proj", "cond_all", "out_proj")]
                + [("fc1", ctypes.POINTER(TcxLinearW)), ("fc2", ctypes.POINTER(TcxLinearW)),
                   ("norm_w", ctypes.POINTER(c_fp)), ("norm_b", ctypes.POINTER(c_fp)),
                   ("out_norm_w", c_fp), ("out_norm_b", c_fp)])


class TcxAdamTensor(ctypes.Structure):
    _fields_ = [("p", c_fp), ("g", c_fp), ("m", c_fp), ("v", c_fp), ("n", c_ll)]


# name -> (restype, argtypes)
_SIGS = {
    "tcx_last_error": (ctypes.c_char_p, []),
    "tcx_version": (c_int, []),
    "tcx_prof_enable": (c_int, [c_int]),
    "tcx_debug_conv_stamps": (c_int, [c_fp, c_int]),
    "tcx_prof_read": (c_int, [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_longlong),
                              ctypes.POINTER(ctypes.c_double)]),
    "tcx_conv2d": (c_int, [c_fp, c_fp, c_int, c_int, c_int, c_int, c_int, c_int, c_fp, c_fp, c_fp, c_fp, c_fp, c_int,
                           c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_fp, c_fp, c_fp, c_fp, c_fp,
                           c_fp]),
    "tcx_pack_conv_weight": (c_int, [c_fp, c_fp, c_int, c_int, c_int, c_int, c_int, c_fp]),
    "tcx_pack_convT_weight": (c_int, [c_fp, c_fp, c_int, c_int, c_int, c_int, c_fp]),
    "tcx_convT2x": (c_int, [c_fp, c_int, c_int, c_int, c_int, c_fp, c_fp, c_fp, c_int, c_int, c_int, c_int, c_fp]),
    "tcx_gn_partials": (c_int, [c_fp, c_int, c_int, c_int, c_int, c_fp, c_fp]),
    "tcx_gn_apply": (c_int, [c_fp, c_fp, c_int, c_int, c_int, c_int, c_fp, c_int, c_fp, c_fp, c_float, c_int, c_fp]),
    "tcx_gn_apply_tab": (c_int, [c_fp, c_fp, c_int, c_int, c_int, c_fp, c_fp, c_int, c_fp]),
    "tcx_gn_apply_tab_absmax": (c_int, [c_fp, c_fp, c_int, c_int, c_int, c_fp, c_fp, c_int, c_fp, c_fp]),
    "tcx_gn_finalize": (c_int, [c_fp, c_int, c_int, c_int, c_int, c_int, c_fp, c_fp, c_float, c_fp, c_fp, c_fp]),
    "tcx_upsample2x": (c_int, [c_fp, c_fp, c_int, c_int, c_int, c_int, c_fp, c_fp, c_fp]),
    "tcx_attention": (c_int, [c_fp, c_fp, c_int, c_int, c_int, c_int, c_fp]),
    # f16x3 split path (h2 storage)
    "tcx_pack_conv_weight_h2": (c_int, [c_fp, c_fp, c_fp, c_int, c_int, c_fp]),
    "tcx_conv2d_h2": (c_int, [c_fp, c_fp, c_int, c_int, c_int, c_int, c_int, c_int, c_fp, c_fp, c_fp, c_fp, c_fp,
                              c_fp, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_fp, c_fp, c_fp]),
    "tcx_conv2d_h2_pro": (c_int, [c_fp, c_fp, c_int, c_int, c_int, c_int, c_int, c_int, c_fp, c_fp, c_fp, c_fp,
                                  c_fp, c_fp, c_fp, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                                  c_fp, c_fp, c_fp, c_fp, c_fp, c_int, c_fp, c_fp]),
    "tcx_conv_wgrad_h2": (c_int, [c_fp, c_fp, c_int, c_int, c_int, c_int, c_int, c_fp, c_int, c_int, c_int, c_int,
                                  c_int, c_float, c_fp, c_fp, c_fp, c_size, c_fp]),
    "tcx_pack_conv_weight_bf16": (c_int, [c_fp, c_fp, c_fp, c_int, c_int, c_fp]),
    "tcx_gn_apply_tab_bf16": (c_int, [c_fp, c_fp, c_int, c_int, c_int, c_fp, c_fp, c_int, c_fp]),
    "tcx_upsample2x_bf16": (c_int, [c_fp, c_fp, c_int, c_int, c_int, c_int, c_fp, c_fp, c_fp]),
    "tcx_attention_split_bf16": (c_int, [c_fp, c_fp, c_int, c_int, c_int, c_int, c_fp]),
    "tcx_attention_split_b2": (c_int, [c_fp, c_fp, c_int, c_int, c_int, c_int, c_fp]),
    "tcx_gn_apply_tab_b2": (c_int, [c_fp, c_fp, c_int, c_int, c_int, c_fp, c_fp, c_int, c_int, c_fp]),
    "tcx_upsample2x_b2": (c_int, [c_fp, c_fp, c_int, c_int, c_int, c_int, c_fp, c_fp, c_fp]),
    "tcx_conv_weight_h2_frag_bytes": (c_size, [c_int, c_int]),
    "tcx_pack_conv_weight_h2_frag": (c_int, [c_fp, c_fp, c_int, c_int, c_int, c_fp]),
    "tcx_conv_weight_h2_frag4_bytes": (c_size, [c_int, c_int]),
    "tcx_pack_conv_weight_h2_frag4": (c_int, [c_fp, c_fp, c_int, c_int, c_int, c_fp]),
    "tcx_gn_apply_tab_h2": (c_int, [c_fp, c_fp, c_int, c_int, c_int, c_fp, c_fp, c_int, c_fp, c_fp]),
    "tcx_gn_apply_tab_h2_cm": (c_int, [c_fp, c_fp, c_int, c_int, c_int, c_fp, c_fp, c_fp, c_fp]),
    "tcx_gn_apply_tab_b2_cm": (c_int, [c_fp, c_fp, c_int, c_int, c_int, c_fp, c_fp, c_fp]),
    "tcx_upsample2x_h2": (c_int, [c_fp, c_fp, c_int, c_int, c_int, c_int, c_fp, c_fp, c_fp, c_fp]),
    "tcx_attention_h2": (c_int, [c_fp, c_fp, c_int, c_int, c_int, c_int, c_fp, c_fp]),
    "tcx_attention_split": (c_int, [c_fp, c_fp, c_int, c_int, c_int, c_int, c_fp]),
    "tcx_f32_to_h2": (c_int, [c_fp, c_fp, c_size, c_fp, c_fp]),
    "tcx_h2_to_f32": (c_int, [c_fp, c_fp, c_size, c_fp]),
    "tcx_absmax": (c_int, [c_fp, c_size, c_fp, c_fp]),
    "tcx_f32_to_h2_scaled": (c_int, [c_fp, c_fp, c_size, c_fp, c_fp, c_fp, c_fp]),
    "tcx_unet_workspace_size": (c_size, [ctypes.POINTER(TcxUnet), c_int, c_int, c_int]),
    "tcx_set_sample_lanes": (c_int, [c_int]),
    "tcx_debug_conv3mb": (c_int, [c_int]),
    "tcx_debug_wgrad3h": (c_int, [c_int]),
    "tcx_sde_workspace_size": (c_size, [ctypes.POINTER(TcxUnet), c_int, c_int, c_int, c_int, c_float]),
    "tcx_ode_workspace_size": (c_size, [ctypes.POINTER(TcxUnet), c_int, c_int, c_int, c_int, c_float]),
    "tcx_debug_fail_eval": (c_int, [c_int]),
    "tcx_unet_eval": (c_int, [ctypes.POINTER(TcxUnet), c_fp, c_fp, c_fp, c_int, c_fp, c_fp, c_int, c_int, c_int,
                              c_float, c_int, c_fp, c_fp, c_u64, c_u64, c_fp, c_fp, c_fp, c_size, c_fp]),
    "tcx_sde_sample": (c_int, [ctypes.POINTER(TcxUnet), c_fp, c_fp, c_fp, c_int, c_int, c_int, c_int, c_float, c_fp,
                               c_fp, c_u64, c_fp, c_size, c_fp]),
    "tcx_ode_sample": (c_int, [ctypes.POINTER(TcxUnet), c_fp, c_fp, c_fp, c_int, c_int, c_int, c_int, c_float, c_fp,
                               c_fp, c_size, c_fp]),
    "tcx_sde_sample_ex": (c_int, [ctypes.POINTER(TcxUnet), c_fp, c_fp, c_fp, c_int, c_int, c_int, c_int, c_float,
                                  c_fp, c_fp, c_u64, c_int, c_fp, c_size, c_fp]),
    "tcx_ode_sample_ex": (c_int, [ctypes.POINTER(TcxUnet), c_fp, c_fp, c_fp, c_int, c_int, c_int, c_int, c_float,
                                  c_fp, c_int, c_fp, c_size, c_fp]),
    "tcx_sde_sample_shard": (c_int, [ctypes.POINTER(TcxUnet), c_fp, c_fp, c_fp, c_int, c_int, c_int, c_int, c_float,
                                     c_fp, c_fp, c_u64, c_int, c_u64, c_fp, c_size, c_fp]),
    "tcx_randn": (c_int, [c_fp, c_size, c_u64, c_u64, c_fp]),
    "tcx_randn_at": (c_int, [c_fp, c_size, c_u64, c_u64, c_u64, c_fp]),
    "tcx_linear": (c_int, [c_fp, c_int, c_fp, c_int, c_fp, c_fp, c_fp, c_fp, c_int, c_int, c_int, c_int, c_int, c_fp]),
    "tcx_linear_workspace": (c_size, [c_int, c_int, c_int, c_int]),
    "tcx_linear_ws": (c_int, [c_fp, c_int, c_fp, c_int, c_fp, c_fp, c_fp, c_fp, c_int, c_int, c_int, c_int, c_int, c_fp,
                              c_size, c_fp]),
    "tcx_layernorm_film": (c_int, [c_fp, c_fp, c_int, c_int, c_fp, c_fp, c_fp, c_int, c_float, c_fp]),
    "tcx_prior_workspace": (c_size, [ctypes.POINTER(TcxPrior), c_int, c_int]),
    "tcx_prior_forward": (c_int, [ctypes.POINTER(TcxPrior), c_fp, c_fp, c_fp, c_fp, c_int, c_fp, c_fp, c_fp, c_size,
                                  c_fp]),
    "tcx_prior_ddim_sample": (c_int, [ctypes.POINTER(TcxPrior), c_fp, c_fp, c_int, ctypes.POINTER(c_ll),
                                      ctypes.POINTER(c_float), ctypes.POINTER(c_float), c_int, c_fp, c_fp, c_fp,
                                      c_size, c_fp]),
    "tcx_linear_h2_bytes": (c_size, [c_int, c_int]),
    "tcx_pack_linear_h2": (c_int, [c_fp, c_int, c_int, c_fp, c_fp, c_fp]),
    # training path
    "tcx_gemm": (c_int, [c_int, c_int, c_int, c_float, c_fp, c_ll, c_ll, c_fp, c_ll, c_ll, c_float, c_fp, c_ll, c_ll,
                         c_fp, c_int, c_int, c_ll, c_ll, c_ll, c_ll, c_ll, c_ll, c_fp]),
    "tcx_gemm_workspace": (c_size, [c_int, c_int, c_int, c_int]),
    "tcx_gemm_ws": (c_int, [c_int, c_int, c_int, c_float, c_fp, c_ll, c_ll, c_fp, c_ll, c_ll, c_float, c_fp, c_ll,
                            c_ll, c_fp, c_int, c_int, c_ll, c_ll, c_ll, c_ll, c_ll, c_ll, c_fp, c_size, c_fp]),
    "tcx_conv_wgrad_workspace": (c_size, [c_int, c_int, c_int, c_int, c_int, c_int]),
    "tcx_conv_wgrad": (c_int, [c_fp, c_fp, c_int, c_int, c_int, c_int, c_int, c_fp, c_int, c_int, c_int, c_int, c_int,
                               c_float, c_fp, c_fp, c_size, c_fp]),
    "tcx_pack_conv_dgrad_weight": (c_int, [c_fp, c_fp, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_fp]),
    "tcx_conv_transpose2x": (c_int, [c_fp, c_int, c_int, c_int, c_int, c_fp, c_fp, c_fp, c_int, c_int, c_int, c_int,
                                     c_int, c_fp]),
    "tcx_conv_transpose2x_h2": (c_int, [c_fp, c_int, c_int, c_int, c_int, c_fp, c_fp, c_fp, c_fp, c_int, c_int, c_int,
                                        c_int, c_int, c_fp]),
    "tcx_gn_stats": (c_int, [c_fp, c_int, c_int, c_int, c_int, c_int, c_fp, c_fp, c_float, c_fp, c_fp, c_fp, c_fp,
                             c_fp]),
    "tcx_gn_bwd_workspace": (c_size, [c_int, c_int, c_int]),
    "tcx_gn_bwd": (c_int, [c_fp, c_fp, c_fp, c_fp, c_fp, c_fp, c_fp, c_int, c_int, c_int, c_int, c_int, c_fp, c_fp,
                           c_fp, c_fp, c_size, c_fp]),
    "tcx_gn_bwd_absmax": (c_int, [c_fp, c_fp, c_fp, c_fp, c_fp, c_fp, c_fp, c_int, c_int, c_int, c_int, c_int, c_fp,
                                  c_fp, c_fp, c_fp, c_fp, c_size, c_fp]),
    "tcx_upsample2x_bwd": (c_int, [c_fp, c_fp, c_int, c_int, c_int, c_int, c_fp]),
    "tcx_colsum_workspace": (c_size, [c_int, c_int, c_int]),
    "tcx_colsum": (c_int, [c_fp, c_int, c_int, c_int, c_fp, c_fp, c_float, c_fp, c_size, c_fp]),
    "tcx_softmax_rows": (c_int, [c_fp, c_fp, c_ll, c_int, c_fp]),
    "tcx_softmax_bwd_rows": (c_int, [c_fp, c_fp, c_fp, c_ll, c_int, c_fp]),
    "tcx_act_fwd": (c_int, [c_fp, c_fp, c_size, c_int, c_fp]),
    "tcx_act_bwd": (c_int, [c_fp, c_fp, c_fp, c_size, c_int, c_fp]),
    "tcx_mse_loss": (c_int, [c_fp, c_fp, c_size, c_fp, c_fp, c_size, c_fp]),
    "tcx_mse_bwd": (c_int, [c_fp, c_fp, c_size, c_fp, c_fp, c_fp]),
    "tcx_embedding_bwd": (c_int, [c_fp, c_fp, c_int, c_int, c_int, c_fp, c_fp]),
    "tcx_ln_fwd": (c_int, [c_fp, c_fp, c_int, c_int, c_fp, c_fp, c_fp, c_int, c_float, c_fp, c_fp, c_fp]),
    "tcx_ln_bwd": (c_int, [c_fp, c_fp, c_int, c_int, c_fp, c_fp, c_fp, c_int, c_fp, c_fp, c_fp, c_fp, c_fp, c_fp,
                           c_fp]),
    "tcx_adam": (c_int, [c_fp, c_int, c_ll, c_float, c_float, c_float, c_float, c_float, c_ll, c_fp]),
    "tcx_ema": (c_int, [c_fp, c_int, c_ll, c_float, c_fp]),
    "tcx_cond_inputs": (c_int, [c_fp, c_fp, c_fp, c_int, c_int, c_int, c_int, c_fp, c_fp, c_fp, c_fp]),
    "tcx_prior_temb": (c_int, [c_fp, c_fp, c_int, c_int, c_fp, c_fp]),
    "tcx_embedding_fwd": (c_int, [c_fp, c_fp, c_int, c_int, c_fp, c_fp]),
    "tcx_copy2d": (c_int, [c_fp, c_ll, c_fp, c_ll, c_int, c_int, c_float, c_fp]),
    "tcx_transpose_bhc": (c_int, [c_fp, c_fp, c_int, c_int, c_int, c_fp]),
    "tcx_first_conv_bias": (c_int, [c_fp, c_fp, c_fp, c_int, c_int, c_int, c_int, c_fp, c_fp]),
    "tcx_first_conv_bwd": (c_int, [c_fp, c_fp, c_fp, c_fp, c_int, c_int, c_int, c_int, c_fp, c_fp, c_fp, c_fp]),
    "tcx_qsample_vp": (c_int, [c_fp, c_fp, c_fp, c_float, c_float, c_float, c_int, c_int, c_fp, c_fp, c_fp]),
    "tcx_cond_drop": (c_int, [c_fp, c_fp, c_fp, c_float, c_int, c_int, c_int, c_fp, c_fp, c_fp]),
    "tcx_prior_qsample": (c_int, [c_fp, c_fp, c_fp, c_fp, c_fp, c_int, c_int, c_int, c_fp, c_fp, c_fp]),
    "tcx_reparam": (c_int, [c_fp, c_fp, c_fp, c_size, c_fp, c_fp]),
    "tcx_reparam_bwd": (c_int, [c_fp, c_fp, c_fp, c_size, c_fp, c_fp, c_float, c_fp]),
    "tcx_vae_kl": (c_int, [c_fp, c_fp, c_int, c_int, c_float, c_fp, c_fp]),
    "tcx_vae_kl_bwd": (c_int, [c_fp, c_fp, c_int, c_int, c_float, c_fp, c_fp, c_fp, c_float, c_fp]),
    "tcx_vae_yvec": (c_int, [c_fp, c_fp, c_fp, c_float, c_int, c_int, c_int, c_fp, c_fp]),
    "tcx_ddim_step": (c_int, [c_fp, c_fp, c_size, c_float, c_float, c_int, c_fp]),
    "tcx_q_sample": (c_int, [c_fp, c_fp, c_fp, c_fp, c_fp, c_int, c_int, c_fp, c_fp]),
    "tcx_u8_gather": (c_int, [c_fp, c_fp, c_int, c_int, c_fp, c_fp]),
    "tcx_render_crystals": (c_int, [c_fp, c_fp, c_fp, c_int, c_int, c_int, c_fp, c_fp, c_fp]),
}

_lib = None

# Conv arithmetic of the score U-Net evaluator: "f16x3" (split-f16 MFMA over h2 activations,
# fp32-grade: DESIGN.md §3c) or "fp32" (v_mfma_f32_32x32x2_f32).  Env TCX_CONV_PRECISION or
# set_conv_precision(); the U-Net falls back to fp32 per call where the split path does not apply
# (base_ch % 32 != 0) or when an activation leaves the f16 range.
_PRECISIONS = ("f16x3", "fp32", "bf16")  # bf16: the score U-Net evaluator only (config 5)
_conv_precision = os.environ.get("TCX_CONV_PRECISION", "f16x3")
if _conv_precision not in _PRECISIONS:
    raise ValueError(f"TCX_CONV_PRECISION must be one of {_PRECISIONS}, got {_conv_precision!r}")


def set_conv_precision(name: str) -> None:
    global _conv_precision
    if name not in _PRECISIONS:
        raise ValueError(f"conv precision must be one of {_PRECISIONS}, got {name!r}")
    _conv_precision = name


def conv_precision() -> str:
    return _conv_precision


# the precision the score U-Net evaluator actually ran its last call in ("bf16" falls back to f16x3
# where the split attention does not apply, any split run to fp32 after a range overflow); bench.py
# reports this, not the requested one
_used_precision = None


def note_used_precision(name: str) -> None:
    global _used_precision
    _used_precision = name


def used_conv_precision():
    return _used_precision


class TcxError(RuntimeError):
    pass


def lib():
    """Load libtcx.so once (raises if it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise TcxError(f"libtcx.so not found at {LIB_PATH}: build it with "
                           f"`make -C vae-diffusion-toy-crystals_amd/csrc` (no CPU fallback exists)")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def exported_symbols():
    return list(_SIGS)


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        msg = lib().tcx_last_error().decode(errors="replace")
        raise TcxError(f"{what or 'libtcx'} failed (rc={rc}): {msg}")


def ptr(t) -> int | None:
    """Device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    return t.data_ptr()


def stream_ptr(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def require_gpu_tensor(t: torch.Tensor, name: str) -> None:
    if not t.is_cuda:
        raise TcxError(f"{name} must be a GPU tensor (device 'cuda' is the MI355X under ROCm); "
                       f"got {t.device}. This build has no CPU path.")
