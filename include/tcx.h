/*
 * tcx.h — C ABI of libtcx.so, the MI355X (gfx950) kernels behind the toy-crystals hot path.
 *
 * The reference (sahhermans/vae-diffusion-toy-crystals) is pure PyTorch: it has no FFI, so
 * each entry point below replaces the ATen op sequence of one reference call site, cited as
 * /root/reference file:line.  The host binding is ctypes.
 *
 * Conventions (all entry points):
 *   - Activations are NHWC fp32, contiguous.  At the module boundary the images are
 *     [B,1,H,W], for which NCHW == NHWC, so no transpose ever crosses the ABI.
 *   - The caller owns every buffer (PyTorch caching allocator); the library never allocates.
 *     Scratch space is caller-provided; *_workspace_size() queries its size.
 *   - Stream-ordered and asynchronous on `stream` (a hipStream_t); no host sync inside.
 *   - Return 0 on success, a negative TCX_E* code otherwise; tcx_last_error() gives the
 *     message (thread-local).  No C++ exception crosses the ABI.
 */
#ifndef TCX_H_
#define TCX_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TCX_OK 0
#define TCX_EINVAL -1   /* bad shape / argument */
#define TCX_EUNSUP -2   /* unsupported configuration */
#define TCX_EHIP -3     /* HIP runtime error */
#define TCX_EWS -4      /* workspace too small */

const char* tcx_last_error(void);
int tcx_version(void);

/* Live timing of the implicit-GEMM conv launches (the path's dominant kernel) for the roofline
 * in bench.py: tcx_prof_enable(1) resets the counters and brackets every conv launch with HIP
 * events on its stream; tcx_prof_read syncs the outstanding events and returns the summed kernel
 * time, the launch count and the summed algorithmic FLOPs (2*M*Cout*ks^2*Cin per launch). */
int tcx_prof_enable(int on);
int tcx_prof_read(double* total_ms, long long* launches, double* flops);
/* Diagnostic timeline of the 16x16x32 3x3 conv (k_conv3m): with buf non-null, each of the first n
 * workgroups of every later launch writes 8 u64 at buf[8 * workgroup]: s_memrealtime (100 MHz) at
 * entry, prologue done, tap loop done, epilogue stores issued and exit, s_memtime at entry and at
 * loop end, and HW_ID | XCC_ID << 16.  buf = NULL (the default) turns it off.  Test / profiling only. */
int tcx_debug_conv_stamps(void* buf, int n);

/* ------------------------------------------------------------------ primitive ops */

/* 2-D convolution as an implicit GEMM on fp32 MFMA (v_mfma_f32_32x32x2_f32).
 * Replaces nn.Conv2d(..., padding_mode="circular") (sde_score_model.py:102,105,133-134,
 * 208,210,218,222,225) and the zero-padded encoder convs (vae.py:19-26).
 *   x1 [Bsrc,H,W,C1], x2 [Bsrc,H,W,C2] or NULL: channel concat [x1, x2] read in place
 *     (torch.cat at sde_score_model.py:246,258,263 is never materialised).
 *   bmod: if > 0, output batch b reads input batch b % bmod (CFG halves share x_t).
 *   wpk [cout_pad][kpad]: weight packed with k = (dy*ks + dx)*Cin + ci, zero padded
 *     (tcx_pack_conv_weight).  bias [Cout] or NULL; bias_b [Bt][Cout] per-batch or NULL;
 *     resid [Bt,Ho,Wo,Cout] added in the epilogue or NULL.
 *   circular: 1 = wrap-around halo, 0 = zero padding.
 *   upsample: 1 = the input is read through a bilinear x2 upsample (align_corners=False,
 *     edge clamped; nn.Upsample at sde_score_model.py:217,221), H,W are the PRE-upsample
 *     dims; only x1 may be set.
 *   act: epilogue activation 0 none, 1 ReLU, 2 sigmoid, 3 SiLU (vae.py:20-26).
 *   gn_stats: if non-NULL, per-(batch, m-tile, channel) partial sums {sum, sumsq} of the
 *     output (fp64) are written for the following GroupNorm: [Bt][nsplit][Cout][2],
 *     nsplit = ceil(Ho*Wo/128).
 *   pro_scale/shift{1,2}: optional fused GroupNorm+SiLU prologue per source:
 *     x -> silu(x * scale[b][c] + shift[b][c]) (tables [Bt][C] from tcx_gn_finalize), applied
 *     once per element as the staged tile is written to LDS — the normalised tensor never
 *     exists in HBM (sde_score_model.py:103-107 feeding the next conv).  Needs Cin, C1 % 32 == 0,
 *     circular padding, Ho*Wo % 128 == 0.  */
int tcx_conv2d(const float* x1, const float* x2, int Bt, int bmod, int H, int W, int C1, int C2,
               const float* wpk, const float* bias, const float* bias_b, const float* resid,
               float* y, int Cout, int cout_pad, int kpad, int ks, int stride, int pad,
               int circular, int upsample, int act, double* gn_stats, const float* pro_scale1,
               const float* pro_shift1, const float* pro_scale2, const float* pro_shift2,
               void* stream);

/* Pack an nn.Conv2d weight [Cout][Cin][ks][ks] into the implicit-GEMM layout above. */
int tcx_pack_conv_weight(const float* w, float* wpk, int Cout, int Cin, int ks, int cout_pad,
                         int kpad, void* stream);
/* Pack an nn.ConvTranspose2d weight [Cin][Cout][4][4] (stride 2, pad 1) into 4 phase
 * weights, each a 2x2 conv in the layout above: wpk [4][cout_pad][kpad]. */
int tcx_pack_convT_weight(const float* w, float* wpk, int Cin, int Cout, int cout_pad, int kpad,
                          void* stream);

/* Transposed conv 4x4 / s2 / p1 (nn.ConvTranspose2d, vae.py:35-42) as 4 sub-pixel phase
 * implicit GEMMs.  x [Bt,H,W,Cin] -> y [Bt,2H,2W,Cout]; act: 0 none, 1 ReLU, 2 sigmoid. */
int tcx_convT2x(const float* x, int Bt, int H, int W, int Cin, const float* wpk4, const float* bias,
                float* y, int Cout, int cout_pad, int kpad, int act, void* stream);

/* GroupNorm statistics (nn.GroupNorm, sde_score_model.py:103,106,130), phase 1:
 * partial {sum, sumsq} per (batch, split, channel) in fp64: part [Bt][nsplit][C][2]. */
int tcx_gn_partials(const float* x, int Bt, int HW, int C, int nsplit, double* part, void* stream);

/* GroupNorm apply (+ optional SiLU, sde_score_model.py:104,107), reading the partials:
 * y = act((x - mean_g) * rstd_g * gamma_c + beta_c).  In-place allowed (y == x). */
int tcx_gn_apply(const float* x, float* y, int Bt, int HW, int C, int groups, const double* part,
                 int nsplit, const float* gamma, const float* beta, float eps, int silu,
                 void* stream);

/* GroupNorm finalize: partials -> per-(batch, channel) scale = rstd*gamma, shift = beta - mean*scale
 * ([Bt][C] each), consumed by the fused prologues of tcx_conv2d / tcx_upsample2x. */
int tcx_gn_finalize(const double* part, int Bt, int HW, int C, int groups, int nsplit,
                    const float* gamma, const float* beta, float eps, float* scale, float* shift,
                    void* stream);

/* GroupNorm apply from finalize tables: y = x*scale[b][c] + shift[b][c] (+ SiLU); in place OK. */
int tcx_gn_apply_tab(const float* x, float* y, int Bt, int HW, int C, const float* scale,
                     const float* shift, int silu, void* stream);
/* The same, also raising *amax (the bit pattern of max |y| as a non-negative float; the caller zeroes
 * it) so that the split training conv consuming y skips its tcx_absmax pass (functional.py). */
int tcx_gn_apply_tab_absmax(const float* x, float* y, int Bt, int HW, int C, const float* scale,
                            const float* shift, int silu, unsigned* amax, void* stream);

/* Bilinear x2 upsample, align_corners=False (nn.Upsample, sde_score_model.py:217,221); optional
 * fused GN+SiLU of the source (scale/shift tables as above, or NULL). */
int tcx_upsample2x(const float* x, float* y, int Bt, int H, int W, int C, const float* scale,
                   const float* shift, void* stream);

/* ------------------------------------------------------------------ procedural dataset
 * Toy-crystal renderer (ToyCrystalsDataset, /root/reference/src/toycrystals/data.py:132-153 +
 * :204-206, and the uint8 quantisation of scripts/build_dataset.py:34): for each image b, atoms
 * pts[offsets[b] .. offsets[b+1]) ([*][2] fp32 (x, y) pixel coordinates, from the host point
 * generator), s2[b] = fp32(2 sigma^2):  v(y, x) = sum_atoms exp(-((x-ax)^2 + (y-ay)^2) / s2[b]),
 * x = clamp(v / (max v + 1e-8), 0, 1) -> x_out [n_img][H][W] fp32 and/or
 * u8_out [n_img][H][W] = (uint8)(x * 255).  H*W <= 16384. */
int tcx_render_crystals(const float* pts, const int* offsets, const float* s2, int n_img, int H, int W,
                        float* x_out, unsigned char* u8_out, void* stream);

/* ------------------------------------------------------------------ f16x3 split path
 * "h2" storage (csrc/h2.hpp): an fp32 tensor [..][C] (C % 8 == 0) kept as [..][C/8][2][8] f16
 * = per 8-channel group 8 hi halves then 8 lo halves (hi = f16(v), lo = f16(v - hi)), four bytes
 * per element like fp32.  A conv over h2 operands forms every product as three f16 MFMAs
 * (hi*hi + hi*lo + lo*hi, f32 accumulation): fp32-grade results at the f16 MFMA
 * rate.  Values must stay below 65504 in magnitude: every h2 writer takes `ovf`, a device word
 * that is OR-ed with 1 when a value does not fit (NULL = no check); the caller then recomputes
 * in fp32.  Same nn.Conv2d sites as tcx_conv2d (sde_score_model.py:102,105,133-134,208,210,218,
 * 222). */

/* Split a packed fp32 conv weight (tcx_pack_conv_weight output, [cout_pad][kpad]) into h2 with a
 * power-of-two scale chosen from max|w|; *wscale (device float) receives the inverse scale. */
int tcx_pack_conv_weight_h2(const float* wpk, void* wh, float* wscale, int cout_pad, int kpad,
                            void* stream);

/* tcx_conv2d over h2 sources x1/x2 and h2 weights (MODE-3 geometry: C1 % 32 == 0, C2 in {0, C1},
 * ks*ks <= 16, kpad == ks*ks*Cin, no upsample/prologue).  Output fp32 (out_h2 = 0) or h2 (1);
 * the fused GroupNorm statistics are taken on the fp32 output value either way. */
int tcx_conv2d_h2(const void* x1, const void* x2, int Bt, int bmod, int H, int W, int C1, int C2,
                  const void* wh, const float* wscale, const float* bias, const float* bias_b,
                  const float* resid, void* y, int out_h2, int Cout, int cout_pad, int kpad, int ks,
                  int stride, int pad, int circular, int act, double* gn_stats, unsigned* ovf,
                  void* stream);

/* Fragment-ordered copy of a 3x3 h2 conv weight ([cout_pad][9 Cin], cout_pad % 96 == 0, Cin % 32 ==
 * 0) for the 3x3 kernel k_conv3g, which loads its B fragments straight from it (one coalesced 1 KB
 * load per wave and fragment, no LDS staging): wf[cout_pad/96][9 Cin/16][3][hi, lo][64][16 B].
 * Same byte size as wh (tcx_conv_weight_h2_frag_bytes). */
size_t tcx_conv_weight_h2_frag_bytes(int cout_pad, int Cin);
int tcx_pack_conv_weight_h2_frag(const void* wh, void* wf, int cout_pad, int kpad, int Cin, void* stream);
/* The same for a 4x4 stride-2 h2 weight ([cout_pad][16 Cin], cout_pad % 96 == 0, Cin % 8 == 0), read by
 * the LDS-DMA downsample kernel k_conv4s2g (ds1 / ds2, sde_score_model.py:208,210) in 16-deep k-steps
 * of two taps x 8 channels: wf[cout_pad/96][2 Cin][3][hi, lo][64][16 B] (k-step 8 j + 2 dy + p holds
 * taps (dy, 2p + lane/32) of channels 8j..8j+7).  Same byte size as wh. */
size_t tcx_conv_weight_h2_frag4_bytes(int cout_pad, int Cin);
int tcx_pack_conv_weight_h2_frag4(const void* wh, void* wf, int cout_pad, int kpad, int Cin, void* stream);

/* ------------------------------------------------------------------ bf16 single-product path
 * Config 5 (256x256, "bf16 MFMA conv-as-GEMM", BASELINE.json configs[4]): the same record layout as
 * h2 with bf16 halves (hi = bf16(v), lo = bf16(v - hi)); every product is ONE
 * v_mfma_f32_32x32x16_bf16 of the hi halves (fp32 accumulation), weights unscaled (*wscale = 1).
 * The evaluator selects it with tcx_unet.precision = 2; tcx_conv2d_h2_pro with bf16 = 1. */
int tcx_pack_conv_weight_bf16(const float* wpk, void* wh, float* wscale, int cout_pad, int kpad, void* stream);
int tcx_gn_apply_tab_bf16(const float* x, void* y, int Bt, int HW, int C, const float* scale, const float* shift,
                          int silu, void* stream);
int tcx_upsample2x_bf16(const float* x, void* y, int Bt, int H, int W, int C, const float* scale,
                        const float* shift, void* stream);
int tcx_attention_split_bf16(const void* qkv, void* out, int Bt, int N, int C, int heads, void* stream);
/* 2-byte bf16 ("b2", csrc/h2.hpp): config 5's tensors at 256^2 are plain NHWC bf16 (round to nearest
 * even) — the hi halves of the bf16 records, which are all a bf16 product reads.  tcx_conv2d_h2_pro with
 * bf16 = 2 reads b2 sources and writes a b2 output for out_h2 = 1 (k_conv3lb, k_conv4s2g, k_lin1x1 shapes
 * only, no prologue); tcx_gn_apply_tab_b2 normalises an fp32 source into b2 (in_b2 = 0) or a b2 tensor in
 * place (in_b2 = 1, x == y); tcx_upsample2x_b2 / tcx_attention_split_b2 write b2 (the attention reads b2
 * qkv).  The U-Net evaluator uses them at precision 2 and 256^2 (sde_score_model.py:170-266). */
int tcx_gn_apply_tab_b2(const void* x, void* y, int Bt, int HW, int C, const float* scale, const float* shift,
                        int silu, int in_b2, void* stream);
int tcx_upsample2x_b2(const float* x, void* y, int Bt, int H, int W, int C, const float* scale, const float* shift,
                      void* stream);
int tcx_attention_split_b2(const void* qkv, void* out, int Bt, int N, int C, int heads, void* stream);

/* tcx_conv2d_h2 with the fragment-ordered weights (wfrag, or NULL) and a GroupNorm+SiLU prologue per
 * source: a source whose pro_scale/pro_shift
 * ([Bt][C] tables from tcx_gn_finalize) are given is read as FP32 and staged as
 * h2(silu(x * scale[b][c] + shift[b][c])) — GroupNorm(+affine)+SiLU of the _ConvBlock
 * (sde_score_model.py:103-107) feeding this conv, never written to memory; a source without
 * tables is h2.  Only k_conv3g takes prologues (wfrag given; 3x3 stride 1 pad 1, W in {32, 64,
 * 128}, Cin % 32 == 0, Cin <= 384, cout_pad % 96 == 0): otherwise a table is TCX_EINVAL.  Without
 * wfrag the call is tcx_conv2d_h2.  bf16: 0 f16x3 records, 1 bf16 records, 2 two-byte bf16; + 16: source 1
 * is chunk-major ([C1/8][bsrc*H*W][32 B] record planes, tcx_gn_apply_tab_h2_cm; 4x4/s2 shapes of k_conv4s2g),
 * + 32: source 2 is chunk-major (3x3 shapes of k_conv3m); f16x3 records without prologue only, else
 * TCX_EINVAL.  With bf16 = 2 (config 5, round 6) the chunk-major planes are 2-byte bf16
 * ([C/8][bsrc*H*W][16 B], tcx_gn_apply_tab_b2_cm): + 16 on k_conv4s2g's slim 4x4/s2 shapes, + 32 on
 * k_conv3lb's 3x3 shapes (rows of 64 / 128 / 256 px). */
int tcx_conv2d_h2_pro(const void* x1, const void* x2, int Bt, int bmod, int H, int W, int C1, int C2,
                      const void* wh, const void* wfrag, const float* wscale, const float* bias,
                      const float* bias_b,
                      const float* resid, void* y, int out_h2, int Cout, int cout_pad, int kpad, int ks,
                      int stride, int pad, int circular, int act, double* gn_stats,
                      const float* pro_scale1, const float* pro_shift1, const float* pro_scale2,
                      const float* pro_shift2, int bf16, unsigned* ovf, void* stream);

/* tcx_gn_apply_tab with the output written as h2 (x == y allowed: in place). */
int tcx_gn_apply_tab_h2(const float* x, void* y, int Bt, int HW, int C, const float* scale,
                        const float* shift, int silu, unsigned* ovf, void* stream);
/* GroupNorm + SiLU apply from tables into CHUNK-MAJOR f16x3 records: y = [C/8][Bt*HW][32 B] (x != y;
 * C % 8 == 0 and HW a multiple of 1536 / (C / 8) pixels) — the U-Net's skip tensors h1 / h2
 * (sde_score_model.py:248-263: h1, h2 and their concats), read by tcx_conv2d_h2_pro with the chunk-major bits. */
int tcx_gn_apply_tab_h2_cm(const float* x, void* y, int Bt, int HW, int C, const float* scale,
                           const float* shift, unsigned* ovf, void* stream);
/* Config 5 (round 6): GroupNorm + SiLU of a 2-byte bf16 tensor x [Bt][HW][C] (a conv's pre-norm b2 output)
 * into CHUNK-MAJOR 2-byte bf16 planes y = [C/8][Bt*HW][16 B] (x != y; the tcx_gn_apply_tab_h2_cm shape
 * conditions) — the 256^2 net's skip tensors h1 / h2 (sde_score_model.py:248-263), the same values as the
 * in-place tcx_gn_apply_tab_b2 bit for bit, read by tcx_conv2d_h2_pro with bf16 = 2 + 16 / 32. */
int tcx_gn_apply_tab_b2_cm(const void* x, void* y, int Bt, int HW, int C, const float* scale,
                           const float* shift, void* stream);
/* tcx_upsample2x with the output written as h2. */
int tcx_upsample2x_h2(const float* x, void* y, int Bt, int H, int W, int C, const float* scale,
                      const float* shift, unsigned* ovf, void* stream);
/* tcx_attention (MFMA kernel, N % 32 == 0) with the output written as h2. */
int tcx_attention_h2(const float* qkv, void* out, int Bt, int N, int C, int heads, unsigned* ovf,
                     void* stream);
/* The same attention with qkv AND out in h2 storage, both products on f16x3 MFMA
 * (attention_split.hip): N % 256 == 0, head dim 16, 32, 48 or 64.  Replaces the SDPA of
 * SelfAttention2d (sde_score_model.py:150-160) in the split-precision evaluator. */
int tcx_attention_split(const void* qkv, void* out, int Bt, int N, int C, int heads, void* stream);
/* Conversions of n elements (n % 8 == 0, channel-fastest tensors with C % 8 == 0). */
int tcx_f32_to_h2(const float* x, void* y, size_t n, unsigned* ovf, void* stream);
int tcx_h2_to_f32(const void* x, float* y, size_t n, void* stream);
/* Power-of-two operand scaling for the split convs of the training path (activations and
 * gradients, which may sit below the f16 normal range or above its maximum):
 * tcx_absmax atomically maxes max|x| (as float bits, exact) into *bits (zero it first; several
 * tensors may share one word); tcx_f32_to_h2_scaled writes h2(x * s) with s = 2^k chosen so that
 * max|x|*s lies in [2^13, 2^14), and, if comb is non-NULL, *comb = *wscale / s (the factor the
 * conv epilogue applies: tcx_conv2d_h2's wscale argument). */
int tcx_absmax(const float* x, size_t n, unsigned* bits, void* stream);
int tcx_f32_to_h2_scaled(const float* x, void* y, size_t n, const unsigned* absmax_bits,
                         const float* wscale, float* comb, void* stream);

/* Multi-head self-attention core of SelfAttention2d (sde_score_model.py:150-160):
 * qkv [Bt,N,3C] (1x1-conv output, channel order [q,k,v], head-major inside each),
 * out [Bt,N,C] = softmax(q k^T / sqrt(C/heads)) v. */
int tcx_attention(const float* qkv, float* out, int Bt, int N, int C, int heads, void* stream);

/* ------------------------------------------------------------------ score U-Net */

typedef struct tcx_conv {
    const float* w;  /* packed [cout_pad][kpad] */
    const float* b;  /* [cout] */
    int cin, cout, ks, kpad, cout_pad;
    const void* wh;       /* h2 split of w (tcx_pack_conv_weight_h2), or NULL */
    const float* wscale;  /* device float: inverse power-of-two scale of wh */
    const void* whf;      /* fragment-ordered copy of wh (tcx_pack_conv_weight_h2_frag), or NULL */
} tcx_conv;

/* Every pointer refers to device memory prepared by the host mirror of CondUNetTiny
 * (sde_score_model.py:170-266): linears are stored transposed ([in][out]).  */
typedef struct tcx_unet {
    int base_ch, emb_dim, cond_ch, time_ch, n_types, y_cont_dim, heads;
    /* conditioning (sde_score_model.py:17-82,195-202,227-241) */
    const float *time_w1t, *time_b1, *time_w2t, *time_b2;        /* time_mlp.0 / .2 */
    const float *ttm_wt, *ttm_b, *tcm_wt, *tcm_b;                /* to_time_map / to_cond_map */
    const float *cat_emb;                                        /* [n_types+1][emb] */
    const float *cmlp_w1t, *cmlp_b1, *cmlp_w2t, *cmlp_b2;        /* cond_emb.cont_mlp.0 / .2 */
    const float *cout_wt, *cout_b;                               /* cond_emb.out.1 [2emb][emb] */
    const float *map_wsum;  /* [base_ch][time_ch+cond_ch]: down1.net.0 weight summed over taps */
    tcx_conv down1_0, down1_1, ds1, down2_0, down2_1, ds2, mid_0, mid_1, qkv, proj, us2, up2_0,
        up2_1, us1, up1_0, up1_1;
    const float *out_w;  /* out conv repacked [base_ch][9] */
    float out_b;
    /* GroupNorm affine, in forward order: down1 x2, down2 x2, mid x2, attn, up2 x2, up1 x2 */
    const float* gn_w[11];
    const float* gn_b[11];
    /* 0: fp32 MFMA convs; 1: f16x3 split convs over h2 activations (needs base_ch % 32 == 0 and
     * every conv's wh/wscale); h2_ovf: device word raised when an activation leaves the f16 range
     * (the host re-runs the evaluation in fp32); 2: bf16 single-product convs and attention over bf16
     * records (wh/whf/wscale then hold the tcx_pack_conv_weight_bf16 packs; (H/4)*(W/4) % 256 == 0) */
    int precision;
    unsigned* h2_ovf;
} tcx_unet;

size_t tcx_unet_workspace_size(const tcx_unet* net, int Bt, int H, int W);

/* Concurrent sampling lanes of tcx_sde_sample: the batch is split into `lanes` (1-4) groups of
 * images advanced step by step on their own HIP streams (joined to the caller's stream at the
 * end); results are identical to one lane.  0 restores the TCX_LANES environment default (1).
 * Returns the previous setting.  Workspace queries made after the call size for the lanes.
 * The setting is per host thread (query the workspace and sample on the thread that set it); the
 * lane streams are created per device on first use, so two devices in one process never share them. */
int tcx_set_sample_lanes(int lanes);

/* Per-step scalar table used by the fused step kernels: row i = {t_i, t_{i+1}, dt, beta(t_i),
 * sigma(t_i), sqrt(beta), sqrt|dt|, alpha(t_i)}, computed on the host with the reference's
 * fp32 formulas (sde_score_model.py:273-298,540-550). */
#define TCX_SCAL 8

/* One U-Net evaluation of a (possibly CFG-doubled) batch, ending in the fused head.
 *   x [B,H,W] (C=1), t_tab: per-sample t is t_tab[0] (a scalar on device) if t_per_sample==0,
 *   else t [B] (t_tab points at it).  y_cat [B] int64, y_cont [B][y_cont_dim].
 *   cfg: if guidance > 0 the batch is evaluated as Bt = 2B ([uncond(null token, y_cont=0);
 *   cond], predict_eps_cfg, sde_score_model.py:402-423) and combined in the head.
 *   mode: 0 eps_out = eps_hat [B,H,W];
 *         1 reverse-SDE Euler-Maruyama update of x in place with noise z (sde_score_model.py:545-559);
 *         2 final projection x0 = clamp(((x - s*eps)/max(a,1e-6) + 1)/2) into eps_out (:562-569);
 *         3 Heun stage 1: drift d (-> eps_out) and x_e = x + d*dt (-> x2)   (:490-492, :426-449);
 *         4 Heun stage 2: x += 0.5*(d + d(x_e))*dt, d read from eps_out, x_e = x2 (:493);
 *         5 as 2 but stops at x0_hat = (x - s*eps)/max(a,1e-6) (:566): no (x0+1)/2 map, no clamp.
 *   scal: device pointer to the current row of the per-step table.
 *   z: noise [B,H,W] for mode 1 (host-injected, parity mode) or NULL to draw it in-kernel from
 *   Philox4x32-10 keyed by (seed, step) (fast mode).  */
int tcx_unet_eval(const tcx_unet* net, const float* x, float* x2, const float* t,
                  int t_per_sample, const int64_t* y_cat, const float* y_cont, int B, int H, int W,
                  float guidance, int mode, const float* scal, const float* z, uint64_t seed,
                  uint64_t step, float* x_inout, float* eps_out, void* ws, size_t ws_bytes,
                  void* stream);

/* Whole reverse-SDE Euler-Maruyama sampler (sample_reverse_sde_euler_maruyama,
 * sde_score_model.py:507-569) natively: n_steps fused evaluations + the final projection.
 *   x [B,H,W]: in = x_T, out = clamped x0 image in [0,1] (C=1).
 *   scal_table [n_steps+1][TCX_SCAL] on device.
 *   noise: [n_steps][B,H,W] host-generated draws (parity mode), or NULL for in-kernel Philox. */
int tcx_sde_sample(const tcx_unet* net, float* x, const int64_t* y_cat, const float* y_cont, int B,
                   int H, int W, int n_steps, float guidance, const float* scal_table,
                   const float* noise, uint64_t seed, void* ws, size_t ws_bytes, void* stream);

/* Probability-flow ODE Heun sampler (sample_probability_flow_ode, :452-504). */
int tcx_ode_sample(const tcx_unet* net, float* x, const int64_t* y_cat, const float* y_cont, int B,
                   int H, int W, int n_steps, float guidance, const float* scal_table, void* ws,
                   size_t ws_bytes, void* stream);

/* The two samplers with output flags.  TCX_SAMPLE_X0_HAT: x receives the unclamped projection
 * x0_hat = (x - sigma*eps)/max(alpha,1e-6) (sde_score_model.py:500,566) instead of the clamped
 * [0,1] image — the reference's last two lines (:503-504, :568-569) are then
 * clamp((x0_hat + 1)/2, 0, 1).  flags = 0 is tcx_sde_sample / tcx_ode_sample. */
#define TCX_SAMPLE_X0_HAT 1
int tcx_sde_sample_ex(const tcx_unet* net, float* x, const int64_t* y_cat, const float* y_cont,
                      int B, int H, int W, int n_steps, float guidance, const float* scal_table,
                      const float* noise, uint64_t seed, int flags, void* ws, size_t ws_bytes,
                      void* stream);
int tcx_ode_sample_ex(const tcx_unet* net, float* x, const int64_t* y_cat, const float* y_cont,
                      int B, int H, int W, int n_steps, float guidance, const float* scal_table,
                      int flags, void* ws, size_t ws_bytes, void* stream);

/* Workspace of one sampler call (the library never allocates: every buffer is the caller's): the
 * U-Net workspace of the (CFG-doubled) rows under the current lane setting, the conditioning tables
 * of the call's n_steps + 1 step-table rows (time / condition maps and the per-(step, image)
 * first-conv bias rows that replace the reference's per-call _make_maps, sde_score_model.py:227-241)
 * and, for the PF-ODE, its drift / Euler-point images.  A smaller ws_bytes is TCX_EWS, whose error
 * message (tcx_last_error) carries the required size.  Query after tcx_set_sample_lanes.
 * BREAKING CHANGE (round 5): the sampler entry points (tcx_sde_sample, tcx_sde_sample_ex,
 * tcx_sde_sample_shard, tcx_ode_sample, tcx_ode_sample_ex) need these sizes; a workspace sized by
 * tcx_unet_workspace_size alone (the round-1..4 contract) is now TCX_EWS, since the conditioning
 * tables grow with n_steps and the library no longer allocates them itself. */
size_t tcx_sde_workspace_size(const tcx_unet* net, int B, int H, int W, int n_steps, float guidance);
size_t tcx_ode_workspace_size(const tcx_unet* net, int B, int H, int W, int n_steps, float guidance);

/* Test hook for the samplers' error paths: the k-th U-Net evaluation after the call (k > 0) fails
 * with TCX_EINVAL before launching anything (one shot; 0 disarms).  Per host thread: arming it never
 * fails another thread's evaluations.  Every sampler exit joins its lane streams back into the
 * caller's stream, so a failed call leaves nothing running unordered. */
int tcx_debug_fail_eval(int k);

/* Test hook (round 6): which 3x3 kernel runs config 5's 2-byte bf16 convs on this host thread — 0 k_conv3lb
 * only (the default: measured 1.1 % faster end to end), 1 k_conv3mb at Cin >= 192 with a 2-byte output, 2
 * k_conv3mb on every shape it covers, -1 back to the TCX_CONV3MB environment default.  Returns the previous
 * override.  Both kernels sum the same bf16 products in the same k order: the outputs are bit-identical (the
 * GroupNorm partials to the fp32 rounding of their per-lane sums). */
int tcx_debug_conv3mb(int mode);

/* Test hook (round 6): the calling thread's choice for the halo-staged 3x3 weight gradient of
 * tcx_conv_wgrad_h2 (wgrad3h.hip: all nine taps of a 32-channel group per workgroup): -1 default
 * (on; TCX_WGRAD3H=0 turns it off), 0 = k_wgrad_h2, 1 = the halo kernel.  Returns the previous mode. */
int tcx_debug_wgrad3h(int mode);

/* (Workspace: tcx_sde_workspace_size(net, B, H, W, n_steps, guidance) bytes — see the breaking-change
 * note above; tcx_ode_sample_ex likewise needs tcx_ode_workspace_size.)
 * tcx_sde_sample_ex on one shard of a larger sampling batch (batch-DP sampling):
 * the Philox counter of element i of x is e_base + i, so images [s, e) of a B-image batch sampled
 * with e_base = s*H*W are bit-identical to those rows of the whole batch sampled in one call with the
 * same seed (the reference draws ONE stream for the whole batch, sde_score_model.py:537,557).
 * e_base = 0 is tcx_sde_sample_ex.  Host-injected `noise` is this shard's slice. */
int tcx_sde_sample_shard(const tcx_unet* net, float* x, const int64_t* y_cat, const float* y_cont,
                         int B, int H, int W, int n_steps, float guidance, const float* scal_table,
                         const float* noise, uint64_t seed, int flags, uint64_t e_base, void* ws,
                         size_t ws_bytes, void* stream);

/* Standard normal draws from Philox4x32-10 (+ Box-Muller), keyed (seed, stream id). */
int tcx_randn(float* out, size_t n, uint64_t seed, uint64_t stream_id, void* stream);
/* The same draws for elements [e_off, e_off + n) of the (seed, stream id) sequence: a shard of x_T. */
int tcx_randn_at(float* out, size_t n, uint64_t seed, uint64_t stream_id, uint64_t e_off, void* stream);

/* ------------------------------------------------------------------ latent prior / MLP */

/* y[M][N] = act([x1 | x2][M][K1+K2] W^T + b) (+ resid) on fp32 MFMA, row-major contiguous.
 * x2 (K2 columns) is an optional second source read as a column concat (torch.cat never
 * materialised, e.g. FiLM cond = [t_feat, y_feat], diffusion_prior.py:121).
 * wpk: nn.Linear weight [N][K1+K2] packed by tcx_pack_conv_weight(ks=1) to [npad][kpad].
 * act: 0 none, 1 ReLU, 2 sigmoid, 3 SiLU.  Replaces the prior's nn.Linear stack
 * (diffusion_prior.py:39-54, 103-110) and the VAE FCs (vae.py:28-33). */
int tcx_linear(const float* x1, int K1, const float* x2, int K2, const float* wpk, const float* b,
               const float* resid, float* y, int M, int N, int npad, int kpad, int act, void* stream);
/* tcx_linear with caller scratch: for skinny batches whose output tiles cannot fill the chip
 * (DDIM sampling of the prior over 36 samples, diffusion_prior.py:203-252) each source is a
 * split-K GEMM (raw partials in ws) and one fixed-order reduce applies bias, residual and the
 * activation (deterministic).  tcx_linear_workspace returns the bytes needed (0: plain
 * tcx_linear, which tcx_linear_ws then runs). */
size_t tcx_linear_workspace(int M, int N, int K1, int K2);
int tcx_linear_ws(const float* x1, int K1, const float* x2, int K2, const float* wpk, const float* b,
                  const float* resid, float* y, int M, int N, int npad, int kpad, int act, void* ws,
                  size_t ws_bytes, void* stream);

/* LayerNorm over the last dim with optional FiLM: y = LN(x)*(1+gamma)+beta where
 * gamma = gb[:, :W], beta = gb[:, W:2W] (FiLMResBlock, diffusion_prior.py:49-52). */
int tcx_layernorm_film(const float* x, float* y, int M, int Wd, const float* ln_w,
                       const float* ln_b, const float* gb, int ld_gb, float eps, void* stream);

/* A packed nn.Linear: w = weight [n][k] packed by tcx_pack_conv_weight(ks=1) to [npad][kpad]
 * (npad >= 16*ceil(n/16), kpad % 4 == 0), b = bias [n]. */
typedef struct tcx_linear_w {
    const float* w;
    const float* b;
    int n, k, npad, kpad;
    /* optional f16x3 pack (tcx_pack_linear_h2) or NULL: rows scaled by 1/winv[n], h2 storage */
    const void* wh;
    const float* winv;
} tcx_linear_w;

/* f16x3 pack of an nn.Linear weight [n][k]: each row scaled by an exact power of two (its max |w|
 * into [2^14, 2^15)), split into h2 storage [ceil16(n)][ceil32(k)/8][2][8] f16 (hi, lo; see the f16x3
 * section); winv [ceil16(n)] receives the inverse scales.  tcx_linear_h2_bytes gives wh's size. */
size_t tcx_linear_h2_bytes(int n, int k);
int tcx_pack_linear_h2(const float* w, int n, int k, void* wh, float* winv, void* stream);

/* DiffusionPriorFiLM (diffusion_prior.py:57-127) as packed device weights.  fc1 / fc2 / norm_w /
 * norm_b are HOST arrays of n_blocks entries (device pointers inside); cond_all is the n_blocks
 * FiLM `cond` linears stacked along N ([n_blocks*2W][2W], input [t_feat | y_feat]). */
typedef struct tcx_prior {
    int z_dim, n_types, y_cont_dim, t_emb_dim, width, n_blocks, y_cat_emb_dim;
    float ln_eps;
    const float* temb_freqs; /* [t_emb_dim/2]: exp(-linspace(0, ln 1e4, half)) (:11-25) */
    const float* y_cat_emb;  /* [n_types][y_cat_emb_dim] */
    tcx_linear_w t_mlp0, t_mlp2, y_cont0, y_cont2, y_fuse0, y_fuse2, in_proj, cond_all, out_proj;
    const tcx_linear_w* fc1;
    const tcx_linear_w* fc2;
    const float* const* norm_w;
    const float* const* norm_b;
    const float* out_norm_w;
    const float* out_norm_b;
} tcx_prior;

/* Scratch bytes for tcx_prior_forward (n_steps = 0) or tcx_prior_ddim_sample (n_steps > 0). */
size_t tcx_prior_workspace(const tcx_prior* net, int B, int n_steps);
/* eps_pred = DiffusionPriorFiLM.forward(z_t, t, y_cat, y_cont) (diffusion_prior.py:108-127), eval mode.
 * B <= 64 runs the skinny path (each weight streamed once, LayerNorm+FiLM fused into the residual
 * reduce); larger B the tiled GEMMs.  ovf: NULL = fp32 products throughout; a device word (zeroed by
 * the caller) = fc1 / fc2 / out_proj on f16x3 MFMA when their h2 packs are present and B <= 64,
 * *ovf != 0 afterwards if an activation left the f16 range (re-run with ovf = NULL). */
int tcx_prior_forward(const tcx_prior* net, const float* z_t, const int64_t* t, const int64_t* y_cat,
                      const float* y_cont, int B, float* eps_out, unsigned* ovf, void* ws, size_t ws_bytes,
                      void* stream);
/* DiffusionSchedule.ddim_sample, eta = 0 (diffusion_prior.py:203-252): z [B][z_dim] holds x_T on entry
 * and z0_pred on return.  ts / abar_t / abar_prev are HOST arrays of n_steps entries (the rounded,
 * de-duplicated timestep grid and alpha_bar at t_i and t_{i+1}).  Loop invariants are hoisted: the
 * y branch and the y half of every FiLM projection once per call, the t branch and the t half for
 * all n_steps timesteps in one batched GEMM (the same sums, split over K at the [t_feat | y_feat]
 * boundary); the DDIM update is fused into the output projection's reduce. */
int tcx_prior_ddim_sample(const tcx_prior* net, const int64_t* y_cat, const float* y_cont, int B,
                          const int64_t* ts, const float* abar_t, const float* abar_prev, int n_steps, float* z,
                          unsigned* ovf, void* ws, size_t ws_bytes, void* stream);

/* ------------------------------------------------------------------ training path (backward)
 * The reference trains with torch autograd (loss.backward(), scripts/train_*.py); these are the
 * native kernels behind the package's autograd Functions.  Activations NHWC fp32 contiguous. */

/* Batched strided fp32-MFMA GEMM: for z in [0,batch): C_z = alpha * A_z B_z + beta * C_z (+ bias[n]).
 * Element A_z(m,k) = A[off_a(z) + m*sa_m + k*sa_k], B_z(k,n) = B[off_b(z) + k*sb_k + n*sb_n],
 * C_z(m,n) = C[off_c(z) + m*sc_m + n*sc_n], off_x(z) = (z / bdiv)*sx_hi + (z % bdiv)*sx_lo.
 * Replaces nn.Linear forward/backward (every model) and the SDPA products Q K^T, P V and their
 * backward (sde_score_model.py:150-157). */
int tcx_gemm(int M, int N, int K, float alpha, const float* A, long long sa_m, long long sa_k,
             const float* B, long long sb_k, long long sb_n, float beta, float* C, long long sc_m,
             long long sc_n, const float* bias, int batch, int bdiv, long long sa_hi, long long sa_lo,
             long long sb_hi, long long sb_lo, long long sc_hi, long long sc_lo, void* stream);
/* tcx_gemm with caller scratch for split-K: when the output tiles cannot fill the chip (e.g. the
 * batch-256 linears of DiffusionPriorFiLM, diffusion_prior.py:39-54) the reduction is split into
 * up to 16 ranges written to ws as raw partials and summed in a fixed order by a second kernel
 * (deterministic).  tcx_gemm_workspace returns the bytes needed (0: no split for this shape);
 * with less scratch than that the call runs unsplit. */
size_t tcx_gemm_workspace(int M, int N, int K, int batch);
int tcx_gemm_ws(int M, int N, int K, float alpha, const float* A, long long sa_m, long long sa_k,
                const float* B, long long sb_k, long long sb_n, float beta, float* C, long long sc_m,
                long long sc_n, const float* bias, int batch, int bdiv, long long sa_hi, long long sa_lo,
                long long sb_hi, long long sb_lo, long long sc_hi, long long sc_lo, void* ws,
                size_t ws_bytes, void* stream);

/* Conv2d weight gradient dw[Cout][C1+C2][ks][ks] (= beta*dw + ...) from the NHWC input
 * [x1 | x2] [Bt][H][W][C1+C2] and the output gradient dy [Bt][Ho][Wo][Cout] (circular or zero
 * padding).  Also the ConvTranspose2d weight gradient (input/output roles swapped).  Backward of
 * nn.Conv2d (sde_score_model.py:102-105,133-134,208-225; vae.py:19-26) / ConvTranspose2d (vae.py:35-42). */
size_t tcx_conv_wgrad_workspace(int Bt, int Ho, int Wo, int Cin, int Cout, int ks);
/* tcx_conv_wgrad on the f16x3 split path: x1/x2 (the conv's input) and dy in h2 records, each scaled
 * by an exact power of two (tcx_absmax + tcx_f32_to_h2_scaled); comb -> 1 / (s_x s_dy).  Products on
 * v_mfma_f32_32x32x16_f16 (three per fp32 product), same split plan, workspace and fixed-order
 * reduce as tcx_conv_wgrad.  C1, C2, Cout % 8 == 0. */
int tcx_conv_wgrad_h2(const void* x1, const void* x2, int Bt, int H, int W, int C1, int C2, const void* dy, int Cout,
                      int ks, int stride, int pad, int circular, float beta, const float* comb, float* dw, void* ws,
                      size_t ws_bytes, void* stream);
int tcx_conv_wgrad(const float* x1, const float* x2, int Bt, int H, int W, int C1, int C2, const float* dy,
                   int Cout, int ks, int stride, int pad, int circular, float beta, float* dw, void* ws,
                   size_t ws_bytes, void* stream);

/* Stride-1 Conv2d data gradient as a forward conv: packs the flipped, transposed weight rows
 * ci in [ci_lo, ci_lo + n_ci) of w [Cout][Cin][ks][ks] to wpk[cout_pad][kpad] with
 * k = (dy*ks + dx)*Cout + co, value w[co][ci][ks-1-dy][ks-1-dx]; run tcx_conv2d(dy_out, ...,
 * pad = ks-1-pad) with it.  Two-source (concat) inputs get one pack per source. */
int tcx_pack_conv_dgrad_weight(const float* w, float* wpk, int Cout, int Cin, int ks, int ci_lo, int n_ci,
                               int cout_pad, int kpad, void* stream);

/* ConvTranspose2d(4, 2, 1) with circular (1) or zero (0) padding of the input grid: the data
 * gradient of the stride-2 circular downsample convs (ds1/ds2, sde_score_model.py:208,210; the
 * weight [Cout][Cin][4][4] packed by tcx_pack_convT_weight(w, wpk, Cout, Cin, ...)) and of the
 * VAE encoder convs (zero padding). */
int tcx_conv_transpose2x(const float* x, int Bt, int H, int W, int Cin, const float* wpk4, const float* bias,
                         float* y, int Cout, int cout_pad, int kpad, int act, int circular, void* stream);

/* The same on the f16x3 split path (round 6): xh = h2 records of x (tcx_f32_to_h2_scaled, scale s_x),
 * wh4 = h2 records of tcx_pack_convT_weight's [4][cout_pad][kpad] (scale s_w), *wscale = 1 / (s_w s_x);
 * Cin % 32 == 0, kpad == 4 Cin.  fp32 output.  The training step's ds1 / ds2 data gradients. */
int tcx_conv_transpose2x_h2(const void* xh, int Bt, int H, int W, int Cin, const void* wh4, const float* wscale,
                            const float* bias, float* y, int Cout, int cout_pad, int kpad, int act, int circular,
                            void* stream);

/* GroupNorm forward statistics from fp64 partials: scale/shift tables [Bt][C] and per-(batch,
 * group) mean / rstd [Bt][groups] saved for the backward (nn.GroupNorm, sde_score_model.py:103). */
int tcx_gn_stats(const double* part, int Bt, int HW, int C, int groups, int nsplit, const float* gamma,
                 const float* beta, float eps, float* scale, float* shift, float* mean, float* rstd,
                 void* stream);

/* Backward of y = silu?(GroupNorm(x)) (silu = 1: the _ConvBlock GN+SiLU pair, :103-105; 0: the
 * attention norm, :150).  dgamma/dbeta optional. */
size_t tcx_gn_bwd_workspace(int Bt, int HW, int C);
int tcx_gn_bwd(const float* x, const float* dy, const float* scale, const float* shift, const float* mean,
               const float* rstd, const float* gamma, int Bt, int HW, int C, int groups, int silu, float* dx,
               float* dgamma, float* dbeta, void* ws, size_t ws_bytes, void* stream);
/* The same, also raising *amax with max |dx| (as tcx_gn_apply_tab_absmax): dx is the dY operand of the
 * split data-gradient conv that follows in backward. */
int tcx_gn_bwd_absmax(const float* x, const float* dy, const float* scale, const float* shift,
                      const float* mean, const float* rstd, const float* gamma, int Bt, int HW, int C,
                      int groups, int silu, float* dx, float* dgamma, float* dbeta, unsigned* amax, void* ws,
                      size_t ws_bytes, void* stream);

/* Adjoint of tcx_upsample2x (nn.Upsample(2, bilinear, align_corners=False), :217-222). */
int tcx_upsample2x_bwd(const float* dy, float* dx, int Bt, int H, int W, int C, void* stream);

/* Column sums of x [Bt][HW][C]: per_batch[Bt][C] and/or total[C] (= beta*total + sum): conv/linear
 * bias gradients and the folded constant-map channels of the first conv. */
size_t tcx_colsum_workspace(int Bt, int HW, int C);
int tcx_colsum(const float* x, int Bt, int HW, int C, float* per_batch, float* total, float beta, void* ws,
               size_t ws_bytes, void* stream);

/* Row softmax and its backward (SDPA, :150-157): P = softmax(S); dS = P * (dP - rowsum(dP * P)). */
int tcx_softmax_rows(const float* S, float* P, long long rows, int n, void* stream);
int tcx_softmax_bwd_rows(const float* P, const float* dP, float* dS, long long rows, int n, void* stream);

/* Elementwise activation (1 ReLU, 2 Sigmoid, 3 SiLU) and its backward from the pre-activation. */
int tcx_act_fwd(const float* z, float* y, size_t n, int act, void* stream);
int tcx_act_bwd(const float* z, const float* dy, float* dz, size_t n, int act, void* stream);

/* mean((a - b)^2) into out[0] (fp64 fixed-order reduction) and its gradient w.r.t. a:
 * da = grad_out[0] * 2 (a - b) / n (sde_score_model.py:399, train_vae.py:309,
 * train_diffusion_prior.py:265).  tcx_mse_loss needs >= 8 KiB + 256 B of workspace. */
int tcx_mse_loss(const float* a, const float* b, size_t n, float* out, void* ws, size_t ws_bytes, void* stream);
int tcx_mse_bwd(const float* a, const float* b, size_t n, const float* grad_out, float* da, void* stream);

/* nn.Embedding backward: dW[rows][E] = sum over b with idx[b] == row of dout[b] (deterministic). */
int tcx_embedding_bwd(const int64_t* idx, const float* dout, int B, int rows, int E, float* dW, void* stream);

/* LayerNorm(+FiLM) forward saving mean/rstd, and its backward (FiLMResBlock / out_norm,
 * diffusion_prior.py:39-54,113).  Backward writes dx, per-row dwrow = dl*xhat and dbrow = dl (sum them
 * over rows with tcx_colsum for the LN weight/bias grads) and, with FiLM, dgb [M][2Wd] = [dh*l | dh]. */
int tcx_ln_fwd(const float* x, float* y, int M, int Wd, const float* w, const float* b, const float* gb,
               int ld_gb, float eps, float* mean, float* rstd, void* stream);
int tcx_ln_bwd(const float* x, const float* dh, int M, int Wd, const float* w, const float* b, const float* gb,
               int ld_gb, const float* mean, const float* rstd, float* dx, float* dwrow, float* dbrow, float* dgb,
               void* stream);

/* Multi-tensor optimiser steps over a HOST array of tensor descriptors (copied into the kernel
 * arguments, 48 tensors per launch: no device table, no host synchronisation).
 * tcx_adam: torch.optim.Adam (amsgrad off) step `step` (1-based) on every {p, g, m, v, n}.
 * tcx_ema:  p = p*decay + (1-decay)*g for every entry ({p_ema, p_model}; m/v unused)
 * (train_sde_score_model.py:233-240). */
typedef struct tcx_adam_tensor {
    float* p;
    const float* g;
    float* m;
    float* v;
    long long n;
} tcx_adam_tensor;
int tcx_adam(const tcx_adam_tensor* table, int ntensors, long long max_n, float lr, float beta1, float beta2,
             float eps, float weight_decay, long long step, void* stream);
int tcx_ema(const tcx_adam_tensor* table, int ntensors, long long max_n, float decay, void* stream);

/* ---- small training-path kernels (conditioning inputs, layout, losses) */
/* score-net conditioning inputs (sde_score_model.py:17-32,66-79): te = timestep_embedding(t, E),
 * yv = theta-sincos rewrite of y_cont, yc = clamp(y_cat, 0, n_types). */
int tcx_cond_inputs(const float* t, const int64_t* y_cat, const float* y_cont, int B, int E, int n_types, int ycd,
                    float* te, float* yv, int64_t* yc, void* stream);
/* prior timestep embedding [sin, cos](t * freqs) (diffusion_prior.py:11-25; freqs from the host). */
int tcx_prior_temb(const int64_t* t, const float* freqs, int B, int E, float* te, void* stream);
/* nn.Embedding forward (row gather). */
int tcx_embedding_fwd(const int64_t* idx, const float* W, int B, int E, float* out, void* stream);
/* dst[r][c] = beta*dst + src with row strides: torch.cat / chunk of feature columns. */
int tcx_copy2d(const float* src, long long ld_src, float* dst, long long ld_dst, int rows, int cols, float beta,
               void* stream);
/* dst[b][c][r] = src[b][r][c]: NHWC <-> NCHW at the VAE flatten (vae.py:51,72). */
int tcx_transpose_bhc(const float* src, float* dst, int B, int R, int C, void* stream);
/* First conv with the 16 constant map channels folded (sde_score_model.py:246): forward bias and backward. */
int tcx_first_conv_bias(const float* maps, const float* w, const float* bias, int B, int C0, int nm, int ks,
                        float* bias_b, void* stream);
int tcx_first_conv_bwd(const float* S, const float* maps, const float* w, const float* dwx, int B, int C0, int nm,
                       int ks, float* dmaps, float* dw, float* db, void* stream);
/* diffusion_loss_eps data path (sde_score_model.py:380-389): t = u^p, x_t = alpha(t)(2x0-1) + sigma(t) eps;
 * half_dbeta = 0.5*(beta_max - beta_min). */
int tcx_qsample_vp(const float* x0, const float* eps, const float* u, float t_power, float beta_min,
                   float half_dbeta, int B, int HW, float* t_out, float* x_t, void* stream);
/* CFG condition dropout (:392-397); r = the rand(B) draws (NULL: no drop). */
int tcx_cond_drop(const int64_t* y_cat, const float* y_cont, const float* r, float p, int B, int ycd, int n_types,
                  int64_t* out_cat, float* out_cont, void* stream);
/* prior training q_sample with t = clamp(long(u^2 T), 0, T-1) (train_diffusion_prior.py:256-260). */
int tcx_prior_qsample(const float* z0, const float* eps, const float* u, const float* sqrt_ab, const float* sqrt_1mab,
                      int T, int B, int Z, int64_t* t_out, float* z_t, void* stream);
/* VAE reparameterise (vae.py:57-60) and kl_stats (train_vae.py:17-36) with their backward. */
int tcx_reparam(const float* mu, const float* lv, const float* eps, size_t n, float* z, void* stream);
int tcx_reparam_bwd(const float* lv, const float* eps, const float* dz, size_t n, float* dmu, float* dlv, float beta,
                    void* stream);
int tcx_vae_kl(const float* mu, const float* lv, int B, int Z, float free_bits, float* out, void* stream);
int tcx_vae_kl_bwd(const float* mu, const float* lv, int B, int Z, float free_bits, const float* grad_out, float* dmu,
                   float* dlv, float beta, void* stream);

/* CondVAE._y_vec [one_hot | y_cont] with the optional training keep mask (vae.py:45-48,65-67). */
int tcx_vae_yvec(const int64_t* y_cat, const float* y_cont, const float* keep_u, float cond_drop, int B, int n_types,
                 int ycd, float* out, void* stream);
/* DDIM eta=0 update in place (diffusion_prior.py:226-250); last != 0 returns z0_pred. */
int tcx_ddim_step(float* z, const float* eps, size_t n, float abar_t, float abar_prev, int last, void* stream);
/* DiffusionSchedule.q_sample with given integer t (diffusion_prior.py:194-201). */
int tcx_q_sample(const float* z0, const int64_t* t, const float* eps, const float* sqrt_ab, const float* sqrt_1mab,
                 int B, int Z, float* out, void* stream);

/* Device-side batch of the disk dataset: out[b] = x_u8[idx[b]] / 255 (disk_data.py:27-31). */
int tcx_u8_gather(const uint8_t* x_u8, const int64_t* idx, int B, int npix, float* out, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* TCX_H_ */
