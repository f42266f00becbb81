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

/* Bilinear x2 upsample, align_corners=False (nn.Upsample, sde_score_model.py:217,221); optional
 * fused GN+SiLU of the source (scale/shift tables as above, or NULL). */
int tcx_upsample2x(const float* x, float* y, int Bt, int H, int W, int C, const float* scale,
                   const float* shift, void* stream);

/* Multi-head self-attention core of SelfAttention2d (sde_score_model.py:150-160):
 * qkv [Bt,N,3C] (1x1-conv output, channel order [q,k,v], head-major inside each),
 * out [Bt,N,C] = softmax(q k^T / sqrt(C/heads)) v. */
int tcx_attention(const float* qkv, float* out, int Bt, int N, int C, int heads, void* stream);

/* ------------------------------------------------------------------ score U-Net */

typedef struct tcx_conv {
    const float* w;  /* packed [cout_pad][kpad] */
    const float* b;  /* [cout] */
    int cin, cout, ks, kpad, cout_pad;
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
} tcx_unet;

size_t tcx_unet_workspace_size(const tcx_unet* net, int Bt, int H, int W);

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
 *         4 Heun stage 2: x += 0.5*(d + d(x_e))*dt, d read from eps_out, x_e = x2 (:493).
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

/* Standard normal draws from Philox4x32-10 (+ Box-Muller), keyed (seed, stream id). */
int tcx_randn(float* out, size_t n, uint64_t seed, uint64_t stream_id, void* stream);

/* ------------------------------------------------------------------ latent prior / MLP */

/* y[M][N] = act([x1 | x2][M][K1+K2] W^T + b) (+ resid) on fp32 MFMA, row-major contiguous.
 * x2 (K2 columns) is an optional second source read as a column concat (torch.cat never
 * materialised, e.g. FiLM cond = [t_feat, y_feat], diffusion_prior.py:121).
 * wpk: nn.Linear weight [N][K1+K2] packed by tcx_pack_conv_weight(ks=1) to [npad][kpad].
 * act: 0 none, 1 ReLU, 2 sigmoid, 3 SiLU.  Replaces the prior's nn.Linear stack
 * (diffusion_prior.py:39-54, 103-110) and the VAE FCs (vae.py:28-33). */
int tcx_linear(const float* x1, int K1, const float* x2, int K2, const float* wpk, const float* b,
               const float* resid, float* y, int M, int N, int npad, int kpad, int act, void* stream);

/* LayerNorm over the last dim with optional FiLM: y = LN(x)*(1+gamma)+beta where
 * gamma = gb[:, :W], beta = gb[:, W:2W] (FiLMResBlock, diffusion_prior.py:49-52). */
int tcx_layernorm_film(const float* x, float* y, int M, int Wd, const float* ln_w,
                       const float* ln_b, const float* gb, int ld_gb, float eps, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* TCX_H_ */
