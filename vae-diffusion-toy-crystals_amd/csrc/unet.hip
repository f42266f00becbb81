// CondUNetTiny forward + sampler step, natively (/root/reference/src/toycrystals/models/
// sde_score_model.py:170-266 forward, :402-423 CFG, :507-569 reverse SDE, :452-504 PF-ODE).
//
// Per U-Net evaluation the host issues ONE call (tcx_unet_eval); the whole reverse-SDE loop is
// one call too (tcx_sde_sample), so no Python runs between kernels.  Kernels here:
//   k_cond   — conditioning MLPs (timestep_embedding :17-32, ConditionEmbedding :35-82,
//              time_mlp/to_*_map :195-202) and the fold of the 16 spatially-constant map
//              channels of the first conv into a per-(batch, channel) bias (circular padding
//              keeps a constant map constant, so its 3x3 contribution is sum_taps(w) * value).
//   k_head   — GroupNorm+SiLU of up1's last conv fused with the out conv's channel reduction:
//              r[b][tap][p] = sum_ci silu(gn(h))[b,p,ci] * w_out[ci][tap] (a 9-wide GEMV per pixel).
//   k_step   — out conv's 9-tap circular gather of r + bias, CFG combine eps_u + s(eps_c - eps_u),
//              and the sampler update (EM / Heun stage / final x0 projection) in one pass;
//              noise either host-injected or Philox4x32-10 in-kernel.
#include <map>
#include <mutex>
#include "common.hpp"
#include "h2.hpp"

namespace tcx {
bool conv3g_covers(int H, int W, int Cin, int cout_pad, bool bf);  // conv3g.hip
// h2 / bf16 record writers (norm.hip, attention_split.hip): bf != 0 writes bf16 halves
bool upsample_fused_ok(int H, int W, int C);  // norm.hip: band / segmented band
bool attn_prep_ok(int HW, int C, int groups, int bf);  // norm.hip: the attention input pass
int attn_prep_h2(float* a, void* y, int Bt, int HW, int C, const float* sc, const float* sh, const float* gamma,
                 const float* beta, int groups, unsigned* ovf, int bf, hipStream_t st);
int upsample2x_h2(const float* x, void* y, int Bt, int H, int W, int C, const float* scale, const float* shift,
                  unsigned* ovf, int bf, hipStream_t st);
int gn_apply_tab_h2(const float* x, void* y, int Bt, int HW, int C, const float* scale, const float* shift, int silu,
                    unsigned* ovf, int bf, hipStream_t st);
int gn_apply_b2_inplace(void* x, int Bt, int HW, int C, const float* scale, const float* shift, int silu,
                        hipStream_t st);
bool gn_apply_cm_ok(int HW, int C);  // norm.hip: chunk-major skip-tensor records
int gn_apply_b2cm(const void* x, void* y, int Bt, int HW, int C, const float* scale, const float* shift,
                  hipStream_t st);  // norm.hip: config 5's chunk-major b2 skip planes
int gn_apply_cm(const float* x, void* y, int Bt, int HW, int C, const float* scale, const float* shift,
                unsigned* ovf, hipStream_t st);
int attention_split(const void* qkv, void* out, int Bt, int N, int C, int heads, int bf, hipStream_t st);
}

#include <cmath>

namespace tcx {
namespace {

constexpr float kLn1e4 = 9.210340371976184f;  // math.log(10000.0)
constexpr float kTwoPi = 6.283185307179586f;

struct CondArgs {
    const float *time_w1t, *time_b1, *time_w2t, *time_b2, *ttm_wt, *ttm_b, *tcm_wt, *tcm_b, *cat_emb, *cmlp_w1t,
        *cmlp_b1, *cmlp_w2t, *cmlp_b2, *cout_wt, *cout_b, *map_wsum, *conv_b;
    int E, n_types, ycd, time_ch, cond_ch, C0;
};

// One block of CT threads per (CFG-doubled) batch row.  Every linear layer is a split-K matvec
// (kgroups of threads each reduce K/kgroups products, then one fixed-order fold over the groups):
// the serial dependency per layer is ~K/8 loads instead of K (one thread per output), which made
// this latency-bound kernel ~58 us per evaluation.
constexpr int CT = 1024;

// out[n] = act(bias[n] + sum_k wt[k*N + n] * in[k]) for n < N (wt: [K][N]); all CT threads call it.
__device__ void cond_mv(const float* __restrict__ wt, const float* __restrict__ bias, const float* in, int K, int N,
                        float* out, float* red, bool silu) {
    const int j = threadIdx.x;
    const int G = max(1, min(CT / N, 16));
    const int n = j % N, g = j / N;
    if (g < G) {
        float s = 0.f;
        for (int k = g; k < K; k += G) s = fmaf(wt[k * N + n], in[k], s);
        red[g * N + n] = s;
    }
    __syncthreads();
    if (j < N) {
        float s = bias[n];
        for (int gg = 0; gg < G; ++gg) s += red[gg * N + n];
        out[n] = silu ? silu_f(s) : s;
    }
    __syncthreads();
}

__global__ __launch_bounds__(CT) void k_cond(CondArgs a, const float* __restrict__ t, int t_per_sample,
                                             const int64_t* __restrict__ y_cat, const float* __restrict__ y_cont,
                                             int B, int cfg, float* __restrict__ bias_b) {
    __shared__ float te[256], h1[256], te2[256], yv[16], g1[256], c2[256], u[512], ce[256], maps[64];
    __shared__ float red[16 * 256];
    const int bb = blockIdx.x;
    const int bs = bb % B;
    const bool null_c = cfg && bb < B;  // first half of a CFG batch = unconditional
    const int E = a.E, half = E / 2;
    const int j = threadIdx.x;
    const float tv = t_per_sample ? t[bs] : t[0];
    if (j < E) {
        // timestep_embedding: freqs = exp(-ln(1e4) * k / max(half-1,1)); args = (2*pi*t) * freqs
        const int k = j < half ? j : j - half;
        const float fr = expf((-kLn1e4 * (float)k) / (float)(half > 1 ? half - 1 : 1));
        const float arg = (kTwoPi * tv) * fr;
        te[j] = j < half ? cosf(arg) : sinf(arg);
    }
    if (j < a.ycd) {
        // y = y_cont; y[1] = sin(theta); y[2] = cos(y[1]).  NB: the reference takes
        // theta = y[:, 1] as a VIEW, so its cos reads the already-replaced sin(theta)
        // (sde_score_model.py:75-78): y[2] = cos(sin(theta)).
        float v = null_c ? 0.f : y_cont[(size_t)bs * a.ycd + j];
        const float th = null_c ? 0.f : y_cont[(size_t)bs * a.ycd + 1];
        if (j == 1) v = sinf(th);
        if (j == 2) v = cosf(sinf(th));
        yv[j] = v;
    }
    __syncthreads();
    cond_mv(a.time_w1t, a.time_b1, te, E, E, h1, red, true);
    cond_mv(a.cmlp_w1t, a.cmlp_b1, yv, a.ycd, E, g1, red, true);
    cond_mv(a.time_w2t, a.time_b2, h1, E, E, te2, red, false);
    cond_mv(a.cmlp_w2t, a.cmlp_b2, g1, E, E, c2, red, false);
    if (j < E) {
        long long yc = null_c ? a.n_types : y_cat[bs];
        yc = yc < 0 ? 0 : (yc > a.n_types ? a.n_types : yc);
        u[j] = silu_f(a.cat_emb[(size_t)yc * E + j]);
        u[E + j] = silu_f(c2[j]);
    }
    __syncthreads();
    cond_mv(a.cout_wt, a.cout_b, u, 2 * E, E, ce, red, false);
    const int nm = a.time_ch + a.cond_ch;
    cond_mv(a.ttm_wt, a.ttm_b, te2, E, a.time_ch, maps, red, false);
    cond_mv(a.tcm_wt, a.tcm_b, ce, E, a.cond_ch, maps + a.time_ch, red, false);
    for (int co = j; co < a.C0; co += CT) {
        float s = a.conv_b[co];
        for (int c = 0; c < nm; ++c) s = fmaf(maps[c], a.map_wsum[co * nm + c], s);
        bias_b[(size_t)bb * a.C0 + co] = s;
    }
}

// Sampler form of the conditioning (round 3): the reference recomputes timestep_embedding + time_mlp
// and ConditionEmbedding for every U-Net call (sde_score_model.py:243-252), but over one sampling
// call t takes only the n_t values of the step table and the condition rows never change.  One
// launch per call computes them all: block i < n_t the time map of t = tvals[i * tstride] (time_ch
// values), block n_t + r the condition map of image r (r == B: the null token with y_cont = 0, the
// unconditional half of every CFG batch).  Same per-value arithmetic as k_cond (cond_mv), so the
// first conv's folded bias (k_conv_first FOLD form) is bit-identical to the per-evaluation path.
__global__ __launch_bounds__(CT) void k_cond_maps(CondArgs a, const float* __restrict__ tvals, int tstride, int n_t,
                                                  const int64_t* __restrict__ y_cat, const float* __restrict__ y_cont,
                                                  int B, float* __restrict__ tmaps, float* __restrict__ cmaps) {
    __shared__ float te[256], h1[256], te2[256], yv[16], g1[256], c2[256], u[512], ce[256];
    __shared__ float red[16 * 256];
    const int E = a.E, half = E / 2;
    const int j = threadIdx.x;
    if ((int)blockIdx.x < n_t) {  // uniform per block
        const float tv = tvals[(size_t)blockIdx.x * tstride];
        if (j < E) {
            const int k = j < half ? j : j - half;
            const float fr = expf((-kLn1e4 * (float)k) / (float)(half > 1 ? half - 1 : 1));
            const float arg = (kTwoPi * tv) * fr;
            te[j] = j < half ? cosf(arg) : sinf(arg);
        }
        __syncthreads();
        cond_mv(a.time_w1t, a.time_b1, te, E, E, h1, red, true);
        cond_mv(a.time_w2t, a.time_b2, h1, E, E, te2, red, false);
        cond_mv(a.ttm_wt, a.ttm_b, te2, E, a.time_ch, tmaps + (size_t)blockIdx.x * a.time_ch, red, false);
        return;
    }
    const int r = blockIdx.x - n_t;
    const bool null_c = r >= B;
    if (j < a.ycd) {  // as k_cond: y[1] = sin(theta), y[2] = cos(sin(theta)) (the reference's view quirk)
        float v = null_c ? 0.f : y_cont[(size_t)r * a.ycd + j];
        const float th = null_c ? 0.f : y_cont[(size_t)r * a.ycd + 1];
        if (j == 1) v = sinf(th);
        if (j == 2) v = cosf(sinf(th));
        yv[j] = v;
    }
    __syncthreads();
    cond_mv(a.cmlp_w1t, a.cmlp_b1, yv, a.ycd, E, g1, red, true);
    cond_mv(a.cmlp_w2t, a.cmlp_b2, g1, E, E, c2, red, false);
    if (j < E) {
        long long yc = null_c ? a.n_types : y_cat[r];
        yc = yc < 0 ? 0 : (yc > a.n_types ? a.n_types : yc);
        u[j] = silu_f(a.cat_emb[(size_t)yc * E + j]);
        u[E + j] = silu_f(c2[j]);
    }
    __syncthreads();
    cond_mv(a.cout_wt, a.cout_b, u, 2 * E, E, ce, red, false);
    cond_mv(a.tcm_wt, a.tcm_b, ce, E, a.cond_ch, cmaps + (size_t)r * a.cond_ch, red, false);
}

// The first-conv bias of every (step, image) of a sampling call: the fold of k_cond (conv_b +
// sum_c maps[c] * map_wsum[co][c], time channels first, the same fmaf order), written once per call
// as bias_tab[n_t][B + 1][C0] (row B: the null token) so an evaluation only reads its rows.
__global__ __launch_bounds__(256) void k_bias_table(const float* __restrict__ tmaps, const float* __restrict__ cmaps,
                                                    const float* __restrict__ map_wsum, const float* __restrict__ conv_b,
                                                    int time_ch, int cond_ch, int C0, int B, int n_t,
                                                    float* __restrict__ bias_tab) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (size_t)n_t * (B + 1) * C0) return;
    const int co = (int)(i % C0);
    const int r = (int)((i / C0) % (B + 1));
    const int step = (int)(i / ((size_t)C0 * (B + 1)));
    const int nm = time_ch + cond_ch;
    const float* tm = tmaps + (size_t)step * time_ch;
    const float* cm = cmaps + (size_t)r * cond_ch;
    float s = conv_b[co];
    for (int c = 0; c < time_ch; ++c) s = fmaf(tm[c], map_wsum[co * nm + c], s);
    for (int c = 0; c < cond_ch; ++c) s = fmaf(cm[c], map_wsum[co * nm + time_ch + c], s);
    bias_tab[i] = s;
}

// One evaluation's view of the table: its images' bias rows and the null-token row.
struct CondTab {
    const float* bias_img;   // [B][C0] of this evaluation's images (null: per-evaluation k_cond)
    const float* bias_null;  // [C0] the null-token row (CFG's unconditional half)
};

__device__ __forceinline__ const float* cond_bias_row(const CondTab& ct, int row, int B, int cfg, int C0) {
    return (cfg && row < B) ? ct.bias_null : ct.bias_img + (size_t)(row % B) * C0;
}

// generic first-conv path: gather the rows into the per-evaluation bias buffer
__global__ __launch_bounds__(256) void k_fold_bias(CondTab ct, int C0, int B, int cfg, int Bt, float* __restrict__ bias_b) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= Bt * C0) return;
    const int row = i / C0, co = i - row * C0;
    bias_b[i] = cond_bias_row(ct, row, B, cfg, C0)[co];
}

// First conv of down1 (17 -> C0, 3x3 circular) with the 16 constant map channels already folded
// into bias_b: y[b,p,co] = bias_b[b][co] + sum_tap w0[co][tap] * x[b % bmod][wrap(p + tap)].
// Output-write bound (C0 floats per input float): a 64-pixel x C0 tile is built in LDS (small, so
// several blocks per CU overlap their load/compute/store phases) and written as one contiguous
// block; per-channel {sum, sumsq} (fp64) of the tile feed the following GroupNorm.
// grid (HW/64, Bt); block 256 = 64 pixels x 4 channel quarters; needs HW % 128 == 0, C0 % 16 == 0.
// MODE 0: fp32 output + GroupNorm partials per 64-pixel tile (the fp32 path / the f16x3 prologue form).
// MODE 2 (split path, round 3): silu(GroupNorm_0(conv)) written as the h2 / bf16 record of
//   down1.net.3's input (scale/shift tables of tcx_gn_finalize over the statistics of k_first_acf /
//   k_first_gnsum below; SiLU as the conv prologues: y rcp(1 + exp2(-y log2 e))), so that conv runs
//   without a prologue and the fp32 tensor is never written or re-read.
constexpr int FIRST_PX = 64;
template <int MODE>
__global__ __launch_bounds__(256) void k_conv_first(const float* __restrict__ x, int bmod, int H, int W, int C0,
                                                    const float* __restrict__ w0, int kpad,
                                                    const float* __restrict__ bias_b, float* __restrict__ y,
                                                    double* __restrict__ gn, CondTab ct, int Bimg, int cfg,
                                                    const float* __restrict__ tsc, const float* __restrict__ tsh,
                                                    unsigned* ovf, int bf) {
    extern __shared__ __attribute__((aligned(16))) float fs[];  // tile[64][C0+4] | w[9][C0] | red[4][C0][2] (dbl)
    const int LD = C0 + 4;
    float* tile = fs;
    float* w = fs + FIRST_PX * LD;
    double* red = reinterpret_cast<double*>(w + 9 * C0);
    const int HW = H * W;
    const int b = blockIdx.y;
    const int tid = threadIdx.x;
    for (int i = tid; i < 9 * C0; i += 256) {
        const int co = i / 9, k = i - (i / 9) * 9;  // w0 packed [co][kpad] with k = tap (Cin = 1)
        w[k * C0 + co] = w0[(size_t)co * kpad + k];
    }
    float* const tab = reinterpret_cast<float*>(red);  // MODE 2: this image's scale | shift (LDS)
    if constexpr (MODE == 2) {
        for (int c = tid; c < C0; c += 256) {
            tab[c] = tsc[(size_t)b * C0 + c];
            tab[C0 + c] = tsh[(size_t)b * C0 + c];
        }
    }
    const int px = tid & (FIRST_PX - 1), qtr = tid >> 6;
    const float* xb = x + (size_t)(b % bmod) * HW;
    const int cq = C0 / 4;
    const float* bb = ct.bias_img ? cond_bias_row(ct, b, Bimg, cfg, C0) : bias_b + (size_t)b * C0;
    constexpr int NT = 1;
    double as[2] = {0.0, 0.0}, aq[2] = {0.0, 0.0};  // this thread's (quarter, c) sums
    for (int tt = 0; tt < NT; ++tt) {
        const int p0 = (blockIdx.x * NT + tt) * FIRST_PX;
        __syncthreads();  // w staged / the previous tile consumed
        const int p = p0 + px;
        const int yy = p / W, xx = p - (p / W) * W;
        float xv[9];
#pragma unroll
        for (int dy = 0; dy < 3; ++dy)
#pragma unroll
            for (int dx = 0; dx < 3; ++dx) xv[dy * 3 + dx] = xb[wrap_idx(yy + dy - 1, H) * W + wrap_idx(xx + dx - 1, W)];
        for (int c = qtr * cq; c < (qtr + 1) * cq; c += 4) {
            float4 a = *reinterpret_cast<const float4*>(bb + c);
#pragma unroll
            for (int k = 0; k < 9; ++k) {
                const float4 wk = *reinterpret_cast<const float4*>(&w[k * C0 + c]);  // broadcast read
                a.x = fmaf(wk.x, xv[k], a.x);
                a.y = fmaf(wk.y, xv[k], a.y);
                a.z = fmaf(wk.z, xv[k], a.z);
                a.w = fmaf(wk.w, xv[k], a.w);
            }
            *reinterpret_cast<float4*>(&tile[px * LD + c]) = a;
        }
        __syncthreads();
        if constexpr (MODE == 0) {
            float* dst = y + ((size_t)b * HW + p0) * C0;
            const int C4 = C0 / 4;
            for (int i = tid; i < FIRST_PX * C4; i += 256) {
                const int r = i / C4, c = (i - (i / C4) * C4) * 4;
                *reinterpret_cast<float4*>(dst + (size_t)i * 4) = *reinterpret_cast<const float4*>(&tile[r * LD + c]);
            }
        } else if constexpr (MODE == 2) {
            // 8-channel groups, channel fastest: consecutive threads write consecutive 32-B records
            char* dst = reinterpret_cast<char*>(y) + ((size_t)b * HW + p0) * C0 * 4;
            const int C8 = C0 / 8;
            const float* s8 = tab;
            const float* h8p = tab + C0;
            bool bad = false;
            for (int i = tid; i < FIRST_PX * C8; i += 256) {
                const int r = i / C8, g = i - (i / C8) * C8;
                const float4 v0 = *reinterpret_cast<const float4*>(&tile[r * LD + 8 * g]);
                const float4 v1 = *reinterpret_cast<const float4*>(&tile[r * LD + 8 * g + 4]);
                const float4 s0 = *reinterpret_cast<const float4*>(s8 + 8 * g);
                const float4 s1 = *reinterpret_cast<const float4*>(s8 + 8 * g + 4);
                const float4 t0 = *reinterpret_cast<const float4*>(h8p + 8 * g);
                const float4 t1 = *reinterpret_cast<const float4*>(h8p + 8 * g + 4);
                auto sl = [](float v, float sc, float sh) {
                    const float q = fmaf(v, sc, sh);
                    return q * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-1.4426950408889634f * q));
                };
                const float4 a0 = make_float4(sl(v0.x, s0.x, t0.x), sl(v0.y, s0.y, t0.y), sl(v0.z, s0.z, t0.z),
                                              sl(v0.w, s0.w, t0.w));
                const float4 a1 = make_float4(sl(v1.x, s1.x, t1.x), sl(v1.y, s1.y, t1.y), sl(v1.z, s1.z, t1.z),
                                              sl(v1.w, s1.w, t1.w));
                uint2 hi0, lo0, hi1, lo1;
                split4x(a0, hi0, lo0, bf != 0);
                split4x(a1, hi1, lo1, bf != 0);
                if (!bf)
                    bad = bad || h2_bad(a0.x) || h2_bad(a0.y) || h2_bad(a0.z) || h2_bad(a0.w) || h2_bad(a1.x) ||
                          h2_bad(a1.y) || h2_bad(a1.z) || h2_bad(a1.w);
                char* gp = dst + (size_t)r * C0 * 4 + 32 * g;
                *reinterpret_cast<uint4*>(gp) = make_uint4(hi0.x, hi0.y, hi1.x, hi1.y);
                *reinterpret_cast<uint4*>(gp + 16) = make_uint4(lo0.x, lo0.y, lo1.x, lo1.y);
            }
            h2_flag(ovf, bad);
        }
        if constexpr (MODE != 2) {
            if (gn) {
#pragma unroll
                for (int e = 0; e < 2; ++e) {
                    const int i = tid + 256 * e;
                    if (i < 4 * C0) {
                        const int c = i % C0, part = i / C0;  // 4 row quarters of 16 pixels
                        double s = 0.0, q = 0.0;
                        for (int r = part * 16; r < part * 16 + 16; ++r) {
                            const double v = tile[r * LD + c];
                            s += v;
                            q += v * v;
                        }
                        as[e] += s;
                        aq[e] += q;
                    }
                }
            }
        }
    }
    if constexpr (MODE != 2) {
        if (gn) {  // 128-pixel GN split = 2 tiles (each half-split in its own slot, summed by the
                   // consumer's fold)
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const int i = tid + 256 * e;
                if (i < 4 * C0) {
                    red[i * 2] = as[e];
                    red[i * 2 + 1] = aq[e];
                }
            }
            __syncthreads();
            const int nsplit = HW / (FIRST_PX * NT);
            for (int c = tid; c < C0; c += 256) {
                double s = 0.0, q = 0.0;
#pragma unroll
                for (int part = 0; part < 4; ++part) {
                    s += red[(part * C0 + c) * 2];
                    q += red[(part * C0 + c) * 2 + 1];
                }
                double* g = gn + (((size_t)b * nsplit + blockIdx.x) * C0 + c) * 2;
                g[0] = s;
                g[1] = q;
            }
        }
    }
}

// GroupNorm statistics of the first conv without evaluating it (split path, round 3).  The conv is
// out[p][c] = bias[c] + sum_k w[c][k] x[p + o_k] over the 9 circular taps o_k of ONE input channel, so
//   sum_p out   = HW bias + (sum_k w_k) S,                         S = sum_q x[q]
//   sum_p out^2 = HW bias^2 + 2 bias (sum_k w_k) S + sum_{k,l} w_k w_l R(o_l - o_k),  R(d) = sum_q x[q] x[q + d]
// (circular shifts preserve both sums): per image, S and the 25 circular autocorrelations R(d),
// d in [-2, 2]^2, then 96 channel sums from them.  Everything in fp64 from the fp32 inputs.
// k_first_acf: grid (HW / chunk, Bt) -> part[b][chunk][26] (chunk = 1024 pixels: at 64^2 a 4096-pixel
// chunk is one workgroup per image, one wave per SIMD with nothing to hide its fp64 chains and loads
// behind: 44 vs 31 us per launch, r03_af vs r03_z; equal at 256^2); k_first_gnsum: grid Bt -> the [Bt][1][C0][2]
// GroupNorm partials tcx_gn_finalize reads (one split).
constexpr int FIRST_ACF_PX = 1024;  // smallest chunk (HW % 1024 == 0)
__global__ __launch_bounds__(256) void k_first_acf(const float* __restrict__ x, int bmod, int H, int W, int chunk,
                                                   double* __restrict__ part) {
    __shared__ double wred[4][26];
    const int b = blockIdx.y, HW = H * W;
    const float* xb = x + (size_t)(b % bmod) * HW;
    double acc[26];
#pragma unroll
    for (int k = 0; k < 26; ++k) acc[k] = 0.0;
    for (int p = blockIdx.x * chunk + threadIdx.x; p < (blockIdx.x + 1) * chunk; p += 256) {
        const int yy = p / W, xx = p - (p / W) * W;
        const double v = xb[p];
        acc[25] += v;
#pragma unroll
        for (int dy = -2; dy <= 2; ++dy) {
            const float* row = xb + wrap_idx(yy + dy, H) * W;
#pragma unroll
            for (int dx = -2; dx <= 2; ++dx) acc[(dy + 2) * 5 + dx + 2] = fma(v, (double)row[wrap_idx(xx + dx, W)], acc[(dy + 2) * 5 + dx + 2]);
        }
    }
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < 26; ++k) {
        double t = acc[k];
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) t += __shfl_xor(t, o);
        if (lane == 0) wred[wv][k] = t;
    }
    __syncthreads();
    if (threadIdx.x < 26) {
        const int k = threadIdx.x;
        part[((size_t)b * gridDim.x + blockIdx.x) * 26 + k] = ((wred[0][k] + wred[1][k]) + wred[2][k]) + wred[3][k];
    }
}

__global__ __launch_bounds__(256) void k_first_gnsum(const double* __restrict__ part, int nchunk, int HW, int C0,
                                                     const float* __restrict__ w0, int kpad,
                                                     const float* __restrict__ bias_b, CondTab ct, int Bimg, int cfg,
                                                     double* __restrict__ gn) {
    __shared__ double a[26];
    const int b = blockIdx.x;
    if (threadIdx.x < 26) {
        double t = 0.0;
        // the CFG halves share x_t: k_first_acf ran over the Bimg distinct images only
        for (int j = 0; j < nchunk; ++j) t += part[((size_t)(b % Bimg) * nchunk + j) * 26 + threadIdx.x];
        a[threadIdx.x] = t;
    }
    __syncthreads();
    const float* bb = ct.bias_img ? cond_bias_row(ct, b, Bimg, cfg, C0) : bias_b + (size_t)b * C0;
    for (int c = threadIdx.x; c < C0; c += 256) {
        double w[9], ws = 0.0;
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            w[k] = w0[(size_t)c * kpad + k];
            ws += w[k];
        }
        const double bi = bb[c], S = a[25];
        double q = 0.0;
#pragma unroll
        for (int k = 0; k < 9; ++k)
#pragma unroll
            for (int l = 0; l < 9; ++l) {
                const int dy = l / 3 - k / 3, dx = l % 3 - k % 3;
                q = fma(w[k] * w[l], a[(dy + 2) * 5 + dx + 2], q);
            }
        double* g = gn + ((size_t)b * C0 + c) * 2;
        g[0] = (double)HW * bi + ws * S;
        g[1] = (double)HW * bi * bi + 2.0 * bi * ws * S + q;
    }
}

// Head: out conv (C -> 1, 3x3 circular) split into a per-pixel channel reduction here and a
// 9-tap circular gather in k_step.  grid (HW/128, Bt); block 256.  The 128-pixel x C tile is read
// coalesced (contiguous 128*C floats), GroupNorm+SiLU applied from the per-image table, staged in
// LDS; then thread (pixel, tap set) computes r[b][tap][p] = sum_c h[p][c] * w_out[c][tap].
constexpr int HEAD_PX = 64;
__global__ __launch_bounds__(256) void k_head(const float* __restrict__ h, int HW, int C, const float* __restrict__ tsc,
                                              const float* __restrict__ tsh, const float* __restrict__ w_out,
                                              float* __restrict__ r) {
    extern __shared__ __attribute__((aligned(16))) float hs[];  // tile[128][C+4] | w[9][C] | sc[C] sh[C]
    const int LD = C + 4;
    float* tile = hs;
    float* w = hs + HEAD_PX * LD;
    float* sc = w + 9 * C;
    float* sh = sc + C;
    const int b = blockIdx.y;
    const int p0 = blockIdx.x * HEAD_PX;
    const int tid = threadIdx.x;
    const int C4 = C / 4;
    const int npx = min(HEAD_PX, HW - p0);
    const float* src = h + ((size_t)b * HW + p0) * C;
    // the tile's loads are all issued before anything waits on them (HK float4 per thread in
    // flight: the block's whole 64 x C tile for C <= 128); a load-transform-store loop keeps one
    // load per thread in flight and ran at 2.8 TB/s
    constexpr int HK = 8;
    const int nq = npx * C4;
    const bool hoist = nq <= HK * 256;
    float4 v[HK];
    if (hoist) {
#pragma unroll
        for (int k = 0; k < HK; ++k) {
            const int i = tid + 256 * k;
            if (i < nq) v[k] = *reinterpret_cast<const float4*>(src + (size_t)i * 4);
        }
    }
    for (int i = tid; i < 9 * C; i += 256) {
        const int c = i / 9, k = i - (i / 9) * 9;  // w_out is [C][9]; stored tap-major
        w[k * C + c] = w_out[i];
    }
    for (int c = tid; c < C; c += 256) {
        sc[c] = tsc[(size_t)b * C + c];
        sh[c] = tsh[(size_t)b * C + c];
    }
    __syncthreads();
    auto put = [&](int i, float4 u) {
        const int px = i / C4, c = (i - (i / C4) * C4) * 4;
        u.x = silu_f(fmaf(u.x, sc[c], sh[c]));
        u.y = silu_f(fmaf(u.y, sc[c + 1], sh[c + 1]));
        u.z = silu_f(fmaf(u.z, sc[c + 2], sh[c + 2]));
        u.w = silu_f(fmaf(u.w, sc[c + 3], sh[c + 3]));
        *reinterpret_cast<float4*>(&tile[px * LD + c]) = u;
    };
    if (hoist) {
#pragma unroll
        for (int k = 0; k < HK; ++k) {
            const int i = tid + 256 * k;
            if (i < nq) put(i, v[k]);
        }
    } else {
        for (int i = tid; i < nq; i += 256) put(i, *reinterpret_cast<const float4*>(src + (size_t)i * 4));
    }
    __syncthreads();
    const int px = tid & (HEAD_PX - 1);
    const int tg = tid >> 6;  // tap group: taps tg, tg + 4, (tg + 8 for group 0)
    if (px >= npx) return;
    const int nk = tg == 0 ? 3 : 2;
    float acc[3] = {0.f, 0.f, 0.f};
    const float* row = &tile[px * LD];
    for (int c = 0; c < C; c += 4) {
        const float4 v = *reinterpret_cast<const float4*>(row + c);
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            if (j < nk) {
                const float4 ww = *reinterpret_cast<const float4*>(&w[(tg + 4 * j) * C + c]);  // broadcast
                float a = acc[j];
                a = fmaf(v.x, ww.x, a);
                a = fmaf(v.y, ww.y, a);
                a = fmaf(v.z, ww.z, a);
                a = fmaf(v.w, ww.w, a);
                acc[j] = a;
            }
        }
    }
    float* dst = r + (size_t)b * 9 * HW + p0 + px;
#pragma unroll
    for (int j = 0; j < 3; ++j)
        if (j < nk) dst[(size_t)(tg + 4 * j) * HW] = acc[j];
}

// Head, register form (round 3): as k_head8, but each lane's CL channels of w_out (9 taps) and of the
// image's scale / shift live in VGPRs for the whole block instead of being re-read from LDS for every
// element (5 LDS reads per element, ~22 LDS clocks per wave-element: the LDS, not HBM, bounded
// k_head8).  A block takes HR_PASS passes of 32 pixels of one image; the loads of the next two passes
// are in flight during the current pass's math (~185 VGPRs: 2 waves per SIMD).  Same arithmetic in the
// same order as k_head8 (bit-identical).
constexpr int HR_PASS = 8;
constexpr int HPR = 32 * HR_PASS;
// B2: the source is 2-byte bf16 (config 5: up1_1's pre-norm output, h2.hpp "b2"): 8 B per 4 channels
template <bool B2>
__device__ __forceinline__ float4 head_ld4(const float* h, size_t e) {
    if constexpr (B2) {
        const uint2 u = *reinterpret_cast<const uint2*>(reinterpret_cast<const char*>(h) + e * 2);
        return make_float4(bf_lo(u.x), bf_hi(u.x), bf_lo(u.y), bf_hi(u.y));
    } else {
        return *reinterpret_cast<const float4*>(h + e);
    }
}
// LA: passes whose loads are in flight ahead of the one being computed (round 5: 2 -> 4, the whole pass
// loop unrolled so the ring is static; 2 passes ahead left the 403 MB read at 3.8 TB/s)
constexpr int HR_LA = 4;
template <int Q, bool B2 = false>
__global__ __launch_bounds__(256) void k_head8r(const float* __restrict__ h, int HW, const float* __restrict__ tsc,
                                                const float* __restrict__ tsh, const float* __restrict__ w_out,
                                                float* __restrict__ r) {
    constexpr int C = 32 * Q;
    constexpr int CL = 4 * Q;
    const int p0 = blockIdx.x * HPR;
    const int b = p0 / HW;
    const int tid = threadIdx.x;
    const int sub = tid & 7, pl = tid >> 3;
    const int c0 = sub * CL;
    float4 v[HR_PASS][Q];  // pass k's channels; only HR_LA + 1 passes are live at a time
    const size_t src0 = (size_t)(p0 + pl) * C + c0;
    // config 5's b2 head (B2, C = 96, round 6): lane sub takes channels [8 sub, 8 sub + 8) — one 16-B load, the 8
    // lanes of a pixel its first 128 contiguous bytes — and [64 + 4 sub, 64 + 4 sub + 4) — one 8-B load, the
    // last 64 B — instead of 12 contiguous channels as three 8-B loads at a 24-B lane stride (the 1.06 GB read
    // ran at 2.3 TB/s, r06_b layers).  The lane's channel j is 8 sub + j (j < 8) or 64 + 4 sub + j - 8.
    constexpr bool CM = B2 && Q == 3;
    auto ld_pass = [&](int k) __attribute__((always_inline)) {
        if constexpr (CM) {
            const char* hp = reinterpret_cast<const char*>(h) + ((size_t)(p0 + pl + k * 32) * C) * 2;
            const uint4 a = *reinterpret_cast<const uint4*>(hp + 16 * sub);
            const uint2 c = *reinterpret_cast<const uint2*>(hp + 128 + 8 * sub);
            v[k][0] = make_float4(bf_lo(a.x), bf_hi(a.x), bf_lo(a.y), bf_hi(a.y));
            v[k][1] = make_float4(bf_lo(a.z), bf_hi(a.z), bf_lo(a.w), bf_hi(a.w));
            v[k][2 % Q] = make_float4(bf_lo(c.x), bf_hi(c.x), bf_lo(c.y), bf_hi(c.y));
        } else {
#pragma unroll
            for (int q = 0; q < Q; ++q) v[k][q] = head_ld4<B2>(h, src0 + (size_t)k * 32 * C + 4 * q);
        }
    };
#pragma unroll
    for (int k = 0; k < HR_LA && k < HR_PASS; ++k) ld_pass(k);
    // the lane's constants as 16-B loads (its 9 CL weights are contiguous in w_out[c][tap], its CL scale /
    // shift entries in the image's table rows): 9 Q + 2 Q vector loads instead of 11 CL scalar ones, which
    // were 5x the data loads' instruction count per block
    float wr[CL][9], scl[CL], shf[CL];
    {
        float4 wq[9 * Q], sq[Q], hq[Q];
        if constexpr (CM) {  // channels 8 sub .. + 7 (18 float4 of w_out), then 64 + 4 sub .. + 3 (9 float4)
            const float4* wa = reinterpret_cast<const float4*>(w_out + (size_t)(8 * sub) * 9);
            const float4* wb = reinterpret_cast<const float4*>(w_out + (size_t)(64 + 4 * sub) * 9);
#pragma unroll
            for (int i = 0; i < 18; ++i) wq[i] = wa[i];
#pragma unroll
            for (int i = 0; i < 9; ++i) wq[18 + i] = wb[i];
            const float* ts = tsc + (size_t)b * C;
            const float* th = tsh + (size_t)b * C;
            sq[0] = reinterpret_cast<const float4*>(ts + 8 * sub)[0];
            sq[1] = reinterpret_cast<const float4*>(ts + 8 * sub)[1];
            sq[2 % Q] = reinterpret_cast<const float4*>(ts + 64 + 4 * sub)[0];
            hq[0] = reinterpret_cast<const float4*>(th + 8 * sub)[0];
            hq[1] = reinterpret_cast<const float4*>(th + 8 * sub)[1];
            hq[2 % Q] = reinterpret_cast<const float4*>(th + 64 + 4 * sub)[0];
        } else {
            const float4* wp = reinterpret_cast<const float4*>(w_out + (size_t)c0 * 9);
#pragma unroll
            for (int i = 0; i < 9 * Q; ++i) wq[i] = wp[i];
#pragma unroll
            for (int i = 0; i < Q; ++i) {
                sq[i] = reinterpret_cast<const float4*>(tsc + (size_t)b * C + c0)[i];
                hq[i] = reinterpret_cast<const float4*>(tsh + (size_t)b * C + c0)[i];
            }
        }
#pragma unroll
        for (int f = 0; f < 36 * Q; ++f) {
            const float4 v = wq[f >> 2];
            wr[f / 9][f % 9] = (f & 3) == 0 ? v.x : (f & 3) == 1 ? v.y : (f & 3) == 2 ? v.z : v.w;
        }
#pragma unroll
        for (int j = 0; j < CL; ++j) {
            const float4 a = sq[j >> 2], c = hq[j >> 2];
            scl[j] = (j & 3) == 0 ? a.x : (j & 3) == 1 ? a.y : (j & 3) == 2 ? a.z : a.w;
            shf[j] = (j & 3) == 0 ? c.x : (j & 3) == 1 ? c.y : (j & 3) == 2 ? c.z : c.w;
        }
    }
#pragma unroll
    for (int pass = 0; pass < HR_PASS; ++pass) {
        const int pg = p0 + pass * 32 + pl;
        if (pass + HR_LA < HR_PASS) ld_pass(pass + HR_LA);
        float acc[9];
#pragma unroll
        for (int t = 0; t < 9; ++t) acc[t] = 0.f;
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const float xs[4] = {v[pass][q].x, v[pass][q].y, v[pass][q].z, v[pass][q].w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int j = 4 * q + e;
                const float yv = fmaf(xs[e], scl[j], shf[j]);
                const float x = yv * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-1.4426950408889634f * yv));
#pragma unroll
                for (int t = 0; t < 9; ++t) acc[t] = fmaf(x, wr[j][t], acc[t]);
            }
        }
#pragma unroll
        for (int t = 0; t < 9; ++t) {
            acc[t] += __shfl_xor(acc[t], 1);
            acc[t] += __shfl_xor(acc[t], 2);
            acc[t] += __shfl_xor(acc[t], 4);
        }
        const int p = pg - b * HW;
        float* dst = r + (size_t)b * 9 * HW + p;
        float mine = acc[0];
#pragma unroll
        for (int t = 1; t < 8; ++t)
            if (sub == t) mine = acc[t];
        dst[(size_t)sub * HW] = mine;  // lane sub writes tap sub; lane 0 also tap 8
        if (sub == 0) dst[(size_t)8 * HW] = acc[8];
    }
}

// First conv + GroupNorm_0 + SiLU written straight as down1.net.3's h2 / bf16 records (round 3, the
// tile-free form of k_conv_first<2>): a workgroup takes FR_PX pixels of one image (one or more whole
// rows, or part of one); the x_t rows it touches (plus the wrapped row above / below) are staged in LDS
// once, with the 3x3 weights [tap][C0] and the image's bias / scale / shift rows; then each thread
// computes whole 8-channel records (item = pixel * C0/8 + group: consecutive lanes write consecutive
// 32-B records, as the tile form's store phase) from 9 broadcast x reads and 18 b128 weight reads.
// No fp32 tile, one barrier, ~5-8 KB of LDS (the tile form held 35 KB: 4 workgroups per CU).
// Needs HW % FR_PX == 0, and FR_PX % W == 0 or W % FR_PX == 0; C0 % 8 == 0.
// fpx (round 6): pixels per workgroup, FR_PX at 64^2; at config 5's 256^2 rows FR_PX_WIDE: the 128-pixel blocks
// (43,008 workgroups per 84-image pass) spent their time on the per-block prologue — three staged x rows,
// the 9 x C0 weight transpose, the bias / table rows — and wrote 1.06 GB at 2.0 TB/s (r06_b layers).
constexpr int FR_PX = 128;
constexpr int FR_PX_WIDE = 1024;
__global__ __launch_bounds__(256) void k_conv_first_rec(const float* __restrict__ x, int bmod, int H, int W, int C0,
                                                        const float* __restrict__ w0, int kpad,
                                                        const float* __restrict__ bias_b, char* __restrict__ y,
                                                        CondTab ct, int Bimg, int cfg, const float* __restrict__ tsc,
                                                        const float* __restrict__ tsh, unsigned* ovf, int bf, int fpx) {
    extern __shared__ __attribute__((aligned(16))) float fr[];  // w[9][C0] | bias[C0] | sc[C0] | sh[C0] | xr[nr][W]
    float* w = fr;
    float* bs = w + 9 * C0;
    float* sc = bs + C0;
    float* sh = sc + C0;
    float* xr = sh + C0;
    const int HW = H * W;
    const int b = blockIdx.y;
    const int tid = threadIdx.x;
    const int p0 = blockIdx.x * fpx;
    const int y0 = p0 / W;                                  // first row of the block's pixels
    const int nrow = (fpx >= W ? fpx / W : 1) + 2;         // staged rows y0-1 .. y0+rows
    const float* xb = x + (size_t)(b % bmod) * HW;
    for (int i = tid; i < nrow * W; i += 256) {
        const int r = i / W, c = i - (i / W) * W;
        xr[i] = xb[(size_t)wrap_idx(y0 - 1 + r, H) * W + c];
    }
    for (int i = tid; i < 9 * C0; i += 256) {
        const int co = i / 9, k = i - (i / 9) * 9;  // w0 packed [co][kpad], k = tap (Cin = 1)
        w[k * C0 + co] = w0[(size_t)co * kpad + k];
    }
    const float* bb = ct.bias_img ? cond_bias_row(ct, b, Bimg, cfg, C0) : bias_b + (size_t)b * C0;
    for (int c = tid; c < C0; c += 256) {
        bs[c] = bb[c];
        sc[c] = tsc[(size_t)b * C0 + c];
        sh[c] = tsh[(size_t)b * C0 + c];
    }
    __syncthreads();
    const int G8 = C0 / 8;
    char* dst = y + ((size_t)b * HW + p0) * C0 * 4;
    bool bad = false;
    for (int item = tid; item < fpx * G8; item += 256) {
        const int pl = item / G8, g = item - (item / G8) * G8;
        const int p = p0 + pl;
        const int yy = p / W, xx = p - (p / W) * W;
        const int ry = yy - y0;  // staged row of (yy - 1) is ry
        float xv[9];
#pragma unroll
        for (int dy = 0; dy < 3; ++dy)
#pragma unroll
            for (int dx = 0; dx < 3; ++dx) xv[dy * 3 + dx] = xr[(ry + dy) * W + wrap_idx(xx + dx - 1, W)];
        float4 a0 = *reinterpret_cast<const float4*>(bs + 8 * g);
        float4 a1 = *reinterpret_cast<const float4*>(bs + 8 * g + 4);
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            const float4 u = *reinterpret_cast<const float4*>(w + k * C0 + 8 * g);
            const float4 v = *reinterpret_cast<const float4*>(w + k * C0 + 8 * g + 4);
            a0.x = fmaf(u.x, xv[k], a0.x); a0.y = fmaf(u.y, xv[k], a0.y);
            a0.z = fmaf(u.z, xv[k], a0.z); a0.w = fmaf(u.w, xv[k], a0.w);
            a1.x = fmaf(v.x, xv[k], a1.x); a1.y = fmaf(v.y, xv[k], a1.y);
            a1.z = fmaf(v.z, xv[k], a1.z); a1.w = fmaf(v.w, xv[k], a1.w);
        }
        const float4 s0 = *reinterpret_cast<const float4*>(sc + 8 * g);
        const float4 s1 = *reinterpret_cast<const float4*>(sc + 8 * g + 4);
        const float4 t0 = *reinterpret_cast<const float4*>(sh + 8 * g);
        const float4 t1 = *reinterpret_cast<const float4*>(sh + 8 * g + 4);
        auto sl = [](float v, float scl, float shf) {
            const float q = fmaf(v, scl, shf);
            return q * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-1.4426950408889634f * q));
        };
        const float4 o0 = make_float4(sl(a0.x, s0.x, t0.x), sl(a0.y, s0.y, t0.y), sl(a0.z, s0.z, t0.z),
                                      sl(a0.w, s0.w, t0.w));
        const float4 o1 = make_float4(sl(a1.x, s1.x, t1.x), sl(a1.y, s1.y, t1.y), sl(a1.z, s1.z, t1.z),
                                      sl(a1.w, s1.w, t1.w));
        uint2 hi0, lo0, hi1, lo1;
        split4x(o0, hi0, lo0, bf != 0);
        split4x(o1, hi1, lo1, bf != 0);
        if (!bf)
            bad = bad || h2_bad(o0.x) || h2_bad(o0.y) || h2_bad(o0.z) || h2_bad(o0.w) || h2_bad(o1.x) ||
                  h2_bad(o1.y) || h2_bad(o1.z) || h2_bad(o1.w);
        if (bf == 2) {  // 2-byte bf16 (h2.hpp "b2"): the hi halves only
            *reinterpret_cast<uint4*>(y + (((size_t)b * HW + p) * C0 + 8 * g) * 2) = make_uint4(hi0.x, hi0.y, hi1.x, hi1.y);
        } else {
            char* gp = dst + (size_t)pl * C0 * 4 + 32 * g;
            *reinterpret_cast<uint4*>(gp) = make_uint4(hi0.x, hi0.y, hi1.x, hi1.y);
            *reinterpret_cast<uint4*>(gp + 16) = make_uint4(lo0.x, lo0.y, lo1.x, lo1.y);
        }
    }
    h2_flag(ovf, bad);
}

// ---------------------------------------------------------------- 8-lanes-per-pixel forms
// For C = 32*Q (every split-path net): a pixel's C channels are 8 contiguous runs of 4Q channels,
// one per lane of an 8-lane group, so a wave reads/writes 8 whole pixels (8*C*4 contiguous bytes)
// per instruction group and nothing goes through an LDS tile; per-pixel reductions are three
// xor-shuffles inside the group (fixed order).

// (A first-conv of this form measured slower than k_conv_first: its per-lane 48-B output runs
// leave every store instruction one-third coalesced, where the LDS tile writes 1 KB contiguous.)
// Head, 8-lane form: r[b][tap][p] = sum_c silu(gn(h))[b,p,c] * w_out[c][tap].  Block 256 threads =
// 32 pixels per pass, HP8 pixels per block (all in one image: HW % HP8 == 0).  w_out and the
// image's scale/shift rows are staged in LDS once per block.
constexpr int HP8 = 128;
template <int Q>
__global__ __launch_bounds__(256) void k_head8(const float* __restrict__ h, int HW, const float* __restrict__ tsc,
                                               const float* __restrict__ tsh, const float* __restrict__ w_out,
                                               float* __restrict__ r) {
    constexpr int C = 32 * Q;
    constexpr int CL = 4 * Q;  // channels per lane
    __shared__ __attribute__((aligned(16))) float ws[C * 12];  // [c][12]: taps 0-8 + pad: 3 ds_read_b128 per channel
    __shared__ __attribute__((aligned(16))) float ssc[C], ssh[C];
    const int p0 = blockIdx.x * HP8;  // first pixel (flat over b, p)
    const int b = p0 / HW;
    const int tid = threadIdx.x;
    const int sub = tid & 7, pl = tid >> 3;  // lane in the pixel group, pixel of the pass
    const int c0 = sub * CL;
    // the first pass's loads go out before the tables are staged
    float4 v[Q];
    {
        const float* src = h + (size_t)(p0 + pl) * C + c0;
#pragma unroll
        for (int q = 0; q < Q; ++q) v[q] = *reinterpret_cast<const float4*>(src + 4 * q);
    }
    for (int i = tid; i < C * 12; i += 256) {
        const int c = i / 12, t = i - (i / 12) * 12;
        ws[i] = t < 9 ? w_out[c * 9 + t] : 0.f;
    }
    for (int i = tid; i < C; i += 256) {
        ssc[i] = tsc[(size_t)b * C + i];
        ssh[i] = tsh[(size_t)b * C + i];
    }
    __syncthreads();
    for (int pass = 0; pass < HP8 / 32; ++pass) {
        const int pg = p0 + pass * 32 + pl;
        float4 vn[Q];
        if (pass + 1 < HP8 / 32) {  // next pass's loads in flight during this pass's math
            const float* src = h + (size_t)(pg + 32) * C + c0;
#pragma unroll
            for (int q = 0; q < Q; ++q) vn[q] = *reinterpret_cast<const float4*>(src + 4 * q);
        }
        float acc[9];
#pragma unroll
        for (int t = 0; t < 9; ++t) acc[t] = 0.f;
#pragma unroll 1
        for (int q = 0; q < Q; ++q) {
            float4 vq = v[0];  // register select (a runtime-indexed v[q] would go to scratch)
#pragma unroll
            for (int j = 1; j < Q; ++j)
                if (q == j) vq = v[j];
            const float xs[4] = {vq.x, vq.y, vq.z, vq.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int c = c0 + 4 * q + e;
                // SiLU as y rcp(1 + exp2(-y log2 e)) (hardware exp2 / rcp, as the conv prologues): the
                // IEEE expf + division form made this kernel VALU-bound (~25 instructions per element)
                const float yv = fmaf(xs[e], ssc[c], ssh[c]);
                const float x = yv * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-1.4426950408889634f * yv));
                const float4 w0 = *reinterpret_cast<const float4*>(&ws[c * 12]);
                const float4 w1 = *reinterpret_cast<const float4*>(&ws[c * 12 + 4]);
                const float w8 = ws[c * 12 + 8];
                acc[0] = fmaf(x, w0.x, acc[0]); acc[1] = fmaf(x, w0.y, acc[1]);
                acc[2] = fmaf(x, w0.z, acc[2]); acc[3] = fmaf(x, w0.w, acc[3]);
                acc[4] = fmaf(x, w1.x, acc[4]); acc[5] = fmaf(x, w1.y, acc[5]);
                acc[6] = fmaf(x, w1.z, acc[6]); acc[7] = fmaf(x, w1.w, acc[7]);
                acc[8] = fmaf(x, w8, acc[8]);
            }
        }
#pragma unroll
        for (int t = 0; t < 9; ++t) {
            acc[t] += __shfl_xor(acc[t], 1);
            acc[t] += __shfl_xor(acc[t], 2);
            acc[t] += __shfl_xor(acc[t], 4);
        }
        const int p = pg - b * HW;
        float* dst = r + (size_t)b * 9 * HW + p;
        dst[(size_t)sub * HW] = acc[sub];  // lane sub writes tap sub; lane 0 also tap 8
        if (sub == 0) dst[(size_t)8 * HW] = acc[8];
        if (pass + 1 < HP8 / 32) {
#pragma unroll
            for (int q = 0; q < Q; ++q) v[q] = vn[q];
        }
    }
}

// ---------------------------------------------------------------- Philox4x32-10
__device__ __forceinline__ void philox(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
        const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0;
        const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
        c[1] = (uint32_t)p1;
        c[3] = (uint32_t)p0;
        c[0] = n0;
        c[2] = n2;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
}

// N(0,1) for element `idx` of draw stream `sid` (Box-Muller on the first two Philox words).
__device__ __forceinline__ float philox_normal(uint64_t seed, uint64_t sid, uint64_t idx) {
    uint32_t c[4] = {(uint32_t)idx, (uint32_t)(idx >> 32), (uint32_t)sid, (uint32_t)(sid >> 32)};
    philox(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    const float u1 = ((float)c[0] + 1.0f) * 2.3283064365386963e-10f;  // (0, 1]
    const float u2 = (float)c[1] * 2.3283064365386963e-10f;
    return sqrtf(-2.0f * logf(u1)) * cosf(kTwoPi * u2);
}

__global__ void k_randn(float* out, size_t n, uint64_t seed, uint64_t sid, uint64_t e_off) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        out[i] = philox_normal(seed, sid, e_off + i);
}

// ---------------------------------------------------------------- fused out-conv gather + update
struct StepArgs {
    const float* r;       // [Bt][9][HW]
    float out_b;
    int B, H, W, cfg;
    float guidance;
    int mode;
    const float* scal;    // current row of the step table
    const float* x;       // U-Net input image [B][HW] (x_t, or x_e in Heun stage 2)
    float* x_inout;       // sampler state
    float* x2;            // Heun x_e
    float* eps_out;
    const float* z;
    uint64_t seed, step;
    size_t e0;  // element offset of this batch chunk (Philox counter = e0 + i: chunking-invariant noise)
};

__device__ __forceinline__ float gather_eps(const float* __restrict__ rb, int HW, int W, int H, int y, int x,
                                            float ob) {
    // out[p] = b + sum_{dy,dx} r[tap=(dy*3+dx)][wrap(y+dy-1), wrap(x+dx-1)]
    float s = ob;
#pragma unroll
    for (int dy = 0; dy < 3; ++dy) {
        const int yy = wrap_idx(y + dy - 1, H);
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) {
            const int xx = wrap_idx(x + dx - 1, W);
            s += rb[(size_t)(dy * 3 + dx) * HW + yy * W + xx];
        }
    }
    return s;
}

__global__ __launch_bounds__(256) void k_step(StepArgs a) {
    const int HW = a.H * a.W;
    const size_t n = (size_t)a.B * HW;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const int b = (int)(i / HW);
        const int p = (int)(i - (size_t)b * HW);
        const int y = p / a.W, x = p - (p / a.W) * a.W;
        float eps;
        if (a.cfg) {
            const float eu = gather_eps(a.r + (size_t)b * 9 * HW, HW, a.W, a.H, y, x, a.out_b);
            const float ec = gather_eps(a.r + (size_t)(a.B + b) * 9 * HW, HW, a.W, a.H, y, x, a.out_b);
            eps = eu + a.guidance * (ec - eu);
        } else {
            eps = gather_eps(a.r + (size_t)b * 9 * HW, HW, a.W, a.H, y, x, a.out_b);
        }
        if (a.mode == 0) {
            a.eps_out[i] = eps;
        } else if (a.mode == 1) {
            // reverse-SDE EM (sde_score_model.py:548-559)
            const float dt = a.scal[2], beta = a.scal[3], sigma = a.scal[4], g = a.scal[5], sq = a.scal[6];
            const float xv = a.x_inout[i];
            const float score = -eps / sigma;
            const float drift = ((-0.5f * beta) * xv) - (beta * score);
            const float z = a.z ? a.z[i] : philox_normal(a.seed, a.step + 1, a.e0 + i);
            a.x_inout[i] = (xv + drift * dt) + (g * sq) * z;
        } else if (a.mode == 2 || a.mode == 5) {
            // final projection (sde_score_model.py:562-569); mode 5 stops at x0_hat (:566), before
            // the (x0 + 1) / 2 map and the clamp (parity reads of the unsaturated trajectory)
            const float sigma = a.scal[4], alpha = a.scal[7];
            const float x0 = (a.x[i] - sigma * eps) / fmaxf(alpha, 1e-6f);
            const float v = (x0 + 1.0f) * 0.5f;
            a.eps_out[i] = a.mode == 5 ? x0 : fminf(fmaxf(v, 0.f), 1.f);
        } else if (a.mode == 3) {
            // Heun stage 1: d = -0.5 b x - 0.5 b score; x_e = x + d dt (sde_score_model.py:444-449,490-491)
            const float dt = a.scal[2], beta = a.scal[3], sigma = a.scal[4];
            const float xv = a.x_inout[i];
            const float score = -eps / sigma;
            const float d = ((-0.5f * beta) * xv) - ((0.5f * beta) * score);
            a.eps_out[i] = d;
            a.x2[i] = xv + d * dt;
        } else {
            // Heun stage 2 at t_next on x_e: x += 0.5 (d + d_next) dt  (sde_score_model.py:492-493)
            const float dt = a.scal[2];
            const float beta = a.scal[TCX_SCAL + 3], sigma = a.scal[TCX_SCAL + 4];
            const float xe = a.x[i];
            const float score = -eps / sigma;
            const float dn = ((-0.5f * beta) * xe) - ((0.5f * beta) * score);
            a.x_inout[i] = a.x_inout[i] + (0.5f * (a.eps_out[i] + dn)) * dt;
        }
    }
}

// ---------------------------------------------------------------- workspace plan
struct Plan {
    int Bt, H, W, C, C2, P0, P1, P2;
    float *bias0, *a64, *b64, *h1, *a32, *b32, *h2, *a16, *b16, *qkv, *r;
    double* gn;
    float* tab;  // GroupNorm scale/shift tables: [11 norms][2][Bt][C2]
    size_t bytes;
    float* sc(int i) const { return tab + (size_t)(2 * i) * Bt * C2; }
    float* sh(int i) const { return tab + (size_t)(2 * i + 1) * Bt * C2; }
};

Plan make_plan(const tcx_unet* net, int Bt, int H, int W, char* base) {
    Plan p{};
    p.Bt = Bt; p.H = H; p.W = W;
    p.C = net->base_ch; p.C2 = 2 * net->base_ch;
    p.P0 = H * W; p.P1 = (H / 2) * (W / 2); p.P2 = (H / 4) * (W / 4);
    size_t off = 0;
    auto take = [&](size_t bytes) -> char* {
        char* ptr = base ? base + off : nullptr;
        off += align_up(bytes, 256);
        return ptr;
    };
    const size_t f = sizeof(float);
    p.bias0 = (float*)take((size_t)Bt * p.C * f);
    p.a64 = (float*)take((size_t)Bt * p.P0 * p.C * f);
    p.b64 = (float*)take((size_t)Bt * p.P0 * p.C * f);
    p.h1 = (float*)take((size_t)Bt * p.P0 * p.C * f);
    p.a32 = (float*)take((size_t)Bt * p.P1 * p.C2 * f);
    p.b32 = (float*)take((size_t)Bt * p.P1 * p.C2 * f);
    p.h2 = (float*)take((size_t)Bt * p.P1 * p.C2 * f);
    p.a16 = (float*)take((size_t)Bt * p.P2 * p.C2 * f);
    p.b16 = (float*)take((size_t)Bt * p.P2 * p.C2 * f);
    p.qkv = (float*)take((size_t)Bt * p.P2 * 3 * p.C2 * f);
    p.r = (float*)take((size_t)Bt * 9 * p.P0 * f);
    const int maxsplit = std::max(1, p.P0 / 128);
    p.gn = (double*)take((size_t)Bt * maxsplit * std::max(p.C2, 2 * p.C2) * 2 * sizeof(double));
    p.tab = (float*)take((size_t)22 * Bt * p.C2 * f);
    p.bytes = off;
    return p;
}

struct GnRef {
    int nsplit;
};

// conv helper: writes GN partials in the epilogue when the tile geometry allows it, else runs
// the partials kernel afterwards; sc/sh{1,2}: fused GN+SiLU prologue tables of the sources.
// H2: split-path context of one evaluation (on: sources are h2 and the f16x3 conv runs)
struct H2Ctx {
    bool on;
    unsigned* ovf;
    bool bf;  // precision 2: bf16 records, one bf16 MFMA per product (no range limit, no flag)
    int fmt;  // conv / writer format flag: 0 h2, 1 bf16 records, 2 two-byte bf16 ("b2", h2.hpp: config 5)
};

int conv_gn(const tcx_conv& cv, const float* x1, const float* x2, int C1, int C2, int Bt, int bmod, int H, int W,
            int stride, int pad, const float* bias_b, const float* resid, float* y, double* gn, int* nsplit,
            hipStream_t st, const float* sc1 = nullptr, const float* sh1 = nullptr, const float* sc2 = nullptr,
            const float* sh2 = nullptr, H2Ctx h2 = {false, nullptr, false, 0}, int out_h2 = 0) {
    const int Ho = (H + 2 * pad - cv.ks) / stride + 1, Wo = (W + 2 * pad - cv.ks) / stride + 1;
    const int HoWo = Ho * Wo;
    const bool fused = gn && HoWo % 128 == 0;
    if (h2.on) {
        // split path: sc/sh tables here are the GroupNorm+SiLU prologue of k_conv3g (fp32 source)
        TCX_REQUIRE(cv.wh && cv.wscale, "tcx_unet: split path needs packed h2 weights");
        TCX_TRY(tcx_conv2d_h2_pro(x1, x2, Bt, bmod, H, W, C1, C2, cv.wh, cv.whf, cv.wscale, cv.b, bias_b, resid, y, out_h2,
                                  cv.cout, cv.cout_pad, cv.kpad, cv.ks, stride, pad, 1, 0, fused ? gn : nullptr, sc1,
                                  sh1, sc2, sh2, h2.fmt, h2.ovf, st));
    } else {
        TCX_TRY(tcx_conv2d(x1, x2, Bt, bmod, H, W, C1, C2, cv.w, cv.b, bias_b, resid, y, cv.cout, cv.cout_pad,
                           cv.kpad, cv.ks, stride, pad, 1, 0, 0, fused ? gn : nullptr, sc1, sh1, sc2, sh2, st));
    }
    if (gn && !fused) {
        const int ns = std::max(1, HoWo / 512);
        TCX_TRY(tcx_gn_partials(y, Bt, HoWo, cv.cout, ns, gn, st));
        *nsplit = ns;
    } else if (gn) {
        *nsplit = HoWo / 128;
    }
    return TCX_OK;
}

// TCX_ATTN_PREP=0: the attention input as four passes (apply, partials, finalize, apply) instead of
// k_attn_prep (its statistics are summed in another fp64 order: not bit-identical; A/B and parity test)
bool attn_prep_enabled() {
    static const bool on = [] {
        const char* e = getenv("TCX_ATTN_PREP");
        return !(e && e[0] == '0');
    }();
    return on;
}

// TCX_SKIP_CM=0: the skip tensors h1 / h2 as pixel-major records (the in-place apply pass), A/B;
// 1 / 2: h1 / h2 only chunk-major (default 3: both)
int skip_cm_mask() {
    static const int m = [] {
        const char* e = getenv("TCX_SKIP_CM");
        return (e && e[0] >= '0' && e[0] <= '3') ? e[0] - '0' : 3;
    }();
    return m;
}

// a skip tensor (H x W x C) can be chunk-major when both readers take it: the downsample on k_conv4s2g
// (fragment-ordered 4x4 weights, Wo in {16, 32, 64}) and the concat conv on k_conv3m (fragment-ordered 3x3
// weights, rows of 16 / 32 / 64 px, Cin = 2 C <= 384, Cout a multiple of 96), neither with a prologue
bool skip_cm_ok(const tcx_conv& ds, const tcx_conv& cat, int H, int W, int C, bool pro) {
    return !pro && gn_apply_cm_ok(H * W, C) && ds.whf && cat.whf && ds.ks == 4 && cat.ks == 3 && H % 2 == 0 &&
           (W == 32 || W == 64) && (H * W / 4) % 128 == 0 && ds.cout_pad % 96 == 0 && 2 * C <= 384 &&
           C % 16 == 0 && cat.cout_pad % 96 == 0 && cat.cout % 96 == 0 && (H * W) % 256 == 0;
}

// config 5 (b2, round 6): a skip tensor can be chunk-major b2 planes when its downsample runs on k_conv4s2g's
// slim form and its concat conv on k_conv3lb (rows of 128 / 256 px), the apply pass tiles the image
bool skip_cm_b2_ok(const tcx_conv& ds, const tcx_conv& cat, int H, int W, int C) {
    return gn_apply_cm_ok(H * W, C) && ds.whf && cat.whf && ds.ks == 4 && cat.ks == 3 && H % 2 == 0 &&
           (W == 128 || W == 256) && (H * W / 4) % 128 == 0 && ds.cout_pad % 96 == 0 && C % 16 == 0 &&
           cat.cout_pad % 96 == 0 && (H * W) % 256 == 0;
}

// TCX_ATTN_SPLIT=0 keeps the split evaluator's attention on fp32 MFMA (A/B measurements)
bool attn_split_enabled() {
    static const bool on = [] {
        const char* e = getenv("TCX_ATTN_SPLIT");
        return !(e && e[0] == '0');
    }();
    return on;
}

int groups_of(int ch) {
    for (int g : {8, 4, 2})
        if (ch % g == 0) return g;
    return 1;
}

int gn_tab(const tcx_unet* net, const Plan& P, int idx, int HW, int C, const double* gn, int ns, hipStream_t st) {
    return tcx_gn_finalize(gn, P.Bt, HW, C, groups_of(C), ns, net->gn_w[idx], net->gn_b[idx], 1e-5f, P.sc(idx),
                           P.sh(idx), st);
}

// The U-Net body (everything up to and including the head partials r).  Input x [B][H][W] (C=1).
// GroupNorm+SiLU outputs are never materialised except where a consumer needs the normalised
// tensor itself (the attention input / residual): every other one is applied by the consuming
// conv's staging prologue from [Bt][C] scale/shift tables (tcx_gn_finalize), with the statistics
// coming from the producing conv's epilogue.
int unet_body(const tcx_unet* net, const Plan& P, const float* x, int B, const float* t, int t_per_sample,
              const int64_t* y_cat, const float* y_cont, int cfg, hipStream_t st, CondTab ct = {}) {
    const int Bt = P.Bt, H = P.H, W = P.W, C = P.C, C2 = P.C2;
    const int H1 = H / 2, W1 = W / 2, H2 = H / 4, W2 = W / 4;
    // conditioning -> per-batch first-conv bias (sampler calls: maps precomputed once per call,
    // k_cond_maps, and folded into the bias by the first conv itself)
    if (!ct.bias_img) {
        CondArgs a{};
        a.time_w1t = net->time_w1t; a.time_b1 = net->time_b1; a.time_w2t = net->time_w2t; a.time_b2 = net->time_b2;
        a.ttm_wt = net->ttm_wt; a.ttm_b = net->ttm_b; a.tcm_wt = net->tcm_wt; a.tcm_b = net->tcm_b;
        a.cat_emb = net->cat_emb; a.cmlp_w1t = net->cmlp_w1t; a.cmlp_b1 = net->cmlp_b1;
        a.cmlp_w2t = net->cmlp_w2t; a.cmlp_b2 = net->cmlp_b2; a.cout_wt = net->cout_wt; a.cout_b = net->cout_b;
        a.map_wsum = net->map_wsum; a.conv_b = net->down1_0.b;
        a.E = net->emb_dim; a.n_types = net->n_types; a.ycd = net->y_cont_dim;
        a.time_ch = net->time_ch; a.cond_ch = net->cond_ch; a.C0 = C;
        hipLaunchKernelGGL(k_cond, dim3(Bt), dim3(CT), 0, st, a, t, t_per_sample, y_cat, y_cont, B, cfg, P.bias0);
        TCX_TRY(check_launch("k_cond"));
    }
    int ns = 1;
    double* gn = P.gn;
    // Where a consumer cannot take the fused prologue (channels not a multiple of 32, or a tile
    // spanning two images at tiny resolutions), the GroupNorm is applied in place instead.
    auto can = [](int Csrc, int Coth, int HoWo) {
        return Csrc % 32 == 0 && Coth % 32 == 0 && HoWo % 128 == 0 && Csrc <= 384 && Coth <= 384;
    };
    // Measured (profiles/r01_*): on gfx950 fp32 MFMA shares the fp32 VALU rate, so a SiLU
    // recomputed for every im2col tap (9x per element) costs the conv ~25 %, more than the
    // separate HBM-bound GroupNorm pass it removes.  The prologue path stays in the ABI
    // (tcx_conv2d pro_*) but the U-Net materialises each GroupNorm once (fused_gn_prologue=false).
    constexpr bool fused_gn_prologue = false;
    bool pro[11] = {};
    if (fused_gn_prologue) {
        pro[0] = can(C, 0, P.P0);
        pro[1] = can(C, 0, P.P1) && can(C, C, P.P0);
        pro[2] = can(C2, 0, P.P1);
        pro[3] = can(C2, 0, P.P2) && can(C2, C2, P.P1);
        pro[4] = can(C2, 0, P.P2);
        pro[7] = can(C, 0, P.P1);
        pro[9] = can(C, 0, P.P0);
    }
    // Split path: a GroupNorm+SiLU whose only consumer is a 3x3 conv on k_conv3g (rows of 16/32/64/128
    // pixels) is applied by that conv's halo staging from the fp32 tensor (tcx_conv2d_h2_pro), so the
    // normalised tensor is never written: norms 0, 2, 4, 7, 9 (down1.net.1, down2.net.1, mid.net.1,
    // up2.net.1, up1.net.1 feeding the .net.3 conv of their block).  The skip tensors h1/h2 (norms 1,
    // 3: read by a 4x4/s2 conv AND an up-path concat) keep the in-place h2 apply pass.
    // (round 2-3 A/B: every GroupNorm as an h2 apply pass instead measured 2-3 % slower; knob removed r04)
    constexpr bool gn_pro = true;
    // bf16 at rows of 64/128/256 pixels: the h2-source conv there is the LDS-DMA k_conv3lb, which has no
    // prologue form; an apply pass + k_conv3lb beats k_conv3g's register-staged prologue form, whose
    // transform (7 halo units per thread at 256-px rows, 3x redundant over the tiles of a row) is not
    // hidden behind a bf16 tap's 6 MFMAs (the prologue form measured equal, r03_y; knob removed r04)
    constexpr bool bf_pro = false;
    auto pro_ok = [&](const tcx_conv& cv, int h, int w, int cin) {
        const bool bf = net->precision == 2;
        if (!cv.whf || !conv3g_covers(h, w, cin, cv.cout_pad, bf)) return false;
        return !(bf && !bf_pro && (w == 64 || w == 128 || w == 256));
    };
    if (net->precision >= 1 && gn_pro) {
        pro[0] = pro_ok(net->down1_1, H, W, C);
        pro[2] = pro_ok(net->down2_1, H1, W1, C2);
        pro[7] = pro_ok(net->up2_1, H1, W1, C);
        pro[9] = pro_ok(net->up1_1, H, W, C);
        pro[4] = pro_ok(net->mid_1, H2, W2, C2);  // mid.net.1 -> mid.net.3
    }
    auto SC = [&](int i) -> const float* { return pro[i] ? P.sc(i) : nullptr; };
    auto SH = [&](int i) -> const float* { return pro[i] ? P.sh(i) : nullptr; };
    // finalize the table of norm i, or normalise `y` in place when no prologue can consume it
    // split path: every conv source is h2 (h2.hpp) — GroupNorm applies feeding a conv write h2
    // in place, convs feeding only convs (ds1, ds2, us2, us1) write h2, the rest stay fp32
    // Config 5 (bf16 at 256^2): every conv there runs on an LDS-DMA kernel that reads 2-byte bf16 (k_conv3lb
    // at 256 / 128 / 64-px rows, k_conv4s2g's slim slots at Wo 128 / 64, k_lin1x1, the split attention), so
    // the tensors are 2-byte bf16 ("b2", h2.hpp) instead of 4-byte records whose lo halves a bf16 product never
    // reads, and the pre-GroupNorm conv outputs are bf16 too (the GroupNorm statistics are taken on the fp32
    // values in the conv epilogue; the apply pass normalises the stored bf16 in place, 2 B read + 2 B written
    // per element).  fp32 stays where a consumer needs it: the attention input / residual (mid_1) and up2_1's
    // output (the upsample applies its GroupNorm from fp32).  TCX_BF_B2=0 keeps the 4-byte records (A/B).
    static const bool b2_on = [] {
        const char* e = getenv("TCX_BF_B2");
        return !(e && e[0] == '0');
    }();
    const int fmt = net->precision == 2 ? ((b2_on && W == 256 && H % 4 == 0 && C == 96) ? 2 : 1) : 0;
    const H2Ctx h2{net->precision >= 1, net->h2_ovf, net->precision == 2, fmt};
    const int pre_b2 = fmt == 2 ? 1 : 0;  // out_h2 of a conv whose output only a GroupNorm apply reads
    auto norm = [&](int i, float* y, int HW, int Cn, bool to_h2 = true) -> int {
        TCX_TRY(gn_tab(net, P, i, HW, Cn, gn, ns, st));
        if (pro[i]) return TCX_OK;
        if (h2.on && to_h2 && fmt == 2) return gn_apply_b2_inplace(y, Bt, HW, Cn, P.sc(i), P.sh(i), 1, st);
        if (h2.on && to_h2) return gn_apply_tab_h2(y, y, Bt, HW, Cn, P.sc(i), P.sh(i), 1, h2.ovf, h2.bf, st);
        return tcx_gn_apply_tab(y, y, Bt, HW, Cn, P.sc(i), P.sh(i), 1, st);
    };
    // down1 (first conv: x_t channel only, maps folded into bias0; the conv bias is inside bias0)
    // Split path (round 3): statistics pass + a second pass that recomputes the conv and writes
    // silu(GroupNorm_0(.)) as down1.net.3's h2 / bf16 record (k_first_acf + k_first_gnsum, k_conv_first MODE 2), so norm 0 needs
    // neither a prologue nor an apply pass and the fp32 tensor is never written (faster than the fp32
    // tensor + prologue form, r03_y; knob removed r04)
    constexpr bool first_fuse = true;
    bool first_fused = false;
    {
        const tcx_conv& c0 = net->down1_0;
        if ((H * W) % FIRST_PX == 0 && C % 16 == 0 && C <= 128 && c0.kpad == 32) {
            const size_t shm = ((size_t)FIRST_PX * (C + 4) + 9 * (size_t)C) * sizeof(float) +
                               8 * (size_t)C * sizeof(double);
            // b2 (fmt 2) tensors are written only by the tile-free record kernel: a shape that would reach
            // k_conv_first<2> (4-byte records) or the fp32 first conv with fmt 2 fails here, loudly
            TCX_REQUIRE(fmt != 2 || (h2.on && first_fuse && (H * W) % FIRST_ACF_PX == 0 && C % 8 == 0 &&
                                     (H * W) % FR_PX == 0 && (FR_PX % W == 0 || W % FR_PX == 0)),
                        "tcx_unet: the 2-byte bf16 format needs the record first conv (H*W %% %d, W vs %d)", FR_PX, FR_PX);
            if (h2.on && first_fuse && (H * W) % FIRST_ACF_PX == 0 && C % 8 == 0) {
                const int chunk = FIRST_ACF_PX;
                const int nchunk = H * W / chunk;
                double* acf = gn + (size_t)Bt * C * 2;  // the autocorrelation partials, past the [Bt][1][C][2] sums
                hipLaunchKernelGGL(k_first_acf, dim3(nchunk, std::min(Bt, B)), dim3(256), 0, st, x, B, H, W, chunk, acf);
                TCX_TRY(check_launch("k_first_acf"));
                hipLaunchKernelGGL(k_first_gnsum, dim3(Bt), dim3(256), 0, st, acf, nchunk, H * W, C, c0.w, c0.kpad,
                                   P.bias0, ct, B, cfg, gn);
                TCX_TRY(check_launch("k_first_gnsum"));
                ns = 1;
                TCX_TRY(gn_tab(net, P, 0, P.P0, C, gn, ns, st));
                // tile-free record kernel (r03_af: 143 -> 114 us at 64^2); the LDS-tile form for other shapes
                if ((H * W) % FR_PX == 0 && (FR_PX % W == 0 || W % FR_PX == 0)) {
                    static const int fr_wide = [] {  // TCX_FR_PX: pixels per block at W >= 256 (A/B)
                        const char* e = getenv("TCX_FR_PX");
                        const int v = e ? atoi(e) : FR_PX_WIDE;
                        return (v >= FR_PX && v <= 4096 && (v & (v - 1)) == 0) ? v : FR_PX_WIDE;
                    }();
                    const int fpx = (W >= 256 && (H * W) % fr_wide == 0 && fr_wide % W == 0) ? fr_wide : FR_PX;
                    const int nrow = (fpx >= W ? fpx / W : 1) + 2;
                    const size_t shr = ((size_t)12 * C + (size_t)nrow * W) * sizeof(float);
                    hipLaunchKernelGGL(k_conv_first_rec, dim3(H * W / fpx, Bt), dim3(256), shr, st, x, B, H, W, C,
                                       c0.w, c0.kpad, P.bias0, (char*)P.a64, ct, B, cfg, P.sc(0), P.sh(0), h2.ovf,
                                       fmt, fpx);
                } else {
                    hipLaunchKernelGGL(k_conv_first<2>, dim3(H * W / FIRST_PX, Bt), dim3(256), shm, st, x, B, H, W,
                                       C, c0.w, c0.kpad, P.bias0, P.a64, nullptr, ct, B, cfg, P.sc(0), P.sh(0),
                                       h2.ovf, h2.bf ? 1 : 0);
                }
                TCX_TRY(check_launch("k_conv_first (GroupNorm+SiLU records)"));
                first_fused = true;
                pro[0] = false;
            } else {
                hipLaunchKernelGGL(k_conv_first<0>, dim3(H * W / FIRST_PX, Bt), dim3(256), shm, st, x, B, H, W, C,
                                   c0.w, c0.kpad, P.bias0, P.a64, gn, ct, B, cfg, nullptr, nullptr, nullptr, 0);
                TCX_TRY(check_launch("k_conv_first"));
                ns = H * W / FIRST_PX;
            }
        } else {
            TCX_REQUIRE(fmt != 2, "tcx_unet: the 2-byte bf16 format needs the record first conv");
            if (ct.bias_img) {
                hipLaunchKernelGGL(k_fold_bias, dim3(cdiv(Bt * C, 256)), dim3(256), 0, st, ct, C, B, cfg, Bt, P.bias0);
                TCX_TRY(check_launch("k_fold_bias"));
            }
            TCX_TRY(tcx_conv2d(x, nullptr, Bt, B, H, W, 1, 0, c0.w, nullptr, P.bias0, nullptr, P.a64, c0.cout,
                               c0.cout_pad, c0.kpad, 3, 1, 1, 1, 0, 0, nullptr, nullptr, nullptr, nullptr, nullptr, st));
            ns = std::max(1, H * W / 512);
            TCX_TRY(tcx_gn_partials(P.a64, Bt, H * W, C, ns, gn, st));
        }
    }
    if (!first_fused) TCX_TRY(norm(0, P.a64, P.P0, C));
    // Chunk-major skip tensors (round 5, TCX_SKIP_CM=0 off): silu(gn(h1)) / silu(gn(h2)) are written as
    // [C/8][Bt*HW][32 B] record planes (gn_apply_cm) for their two readers, the 4x4/s2 downsample (source 1,
    // whose halo DMA re-fetched pixel-major lines) and the up-path concat conv on k_conv3m (source 2).  The
    // raw conv output goes to a buffer that is free at that point (b64 / a32) and the apply writes h1 / h2.
    // (config 5, round 6: the b2 skip tensors as chunk-major b2 planes, gn_apply_b2cm, same readers' roles)
    const bool cm1 = h2.on && (skip_cm_mask() & 1) &&
                     ((fmt == 0 && skip_cm_ok(net->ds1, net->up1_0, H, W, C, pro[1])) ||
                      (fmt == 2 && !pro[1] && skip_cm_b2_ok(net->ds1, net->up1_0, H, W, C)));
    const bool cm2 = h2.on && (skip_cm_mask() & 2) &&
                     ((fmt == 0 && skip_cm_ok(net->ds2, net->up2_0, H1, W1, C2, pro[3])) ||
                      (fmt == 2 && !pro[3] && skip_cm_b2_ok(net->ds2, net->up2_0, H1, W1, C2)));
    auto apply_cm = [&](const float* raw, float* dst, int HWn, int Cn, int i) -> int {
        TCX_TRY(gn_tab(net, P, i, HWn, Cn, gn, ns, st));
        if (fmt == 2) return gn_apply_b2cm(raw, dst, Bt, HWn, Cn, P.sc(i), P.sh(i), st);
        return gn_apply_cm(raw, dst, Bt, HWn, Cn, P.sc(i), P.sh(i), h2.ovf, st);
    };
    H2Ctx h2cs = h2, h2cc = h2;  // h2 with the chunk-major bits: source 1 (downsample), source 2 (concat)
    h2cs.fmt |= 16;
    h2cc.fmt |= 32;
    TCX_TRY(conv_gn(net->down1_1, P.a64, nullptr, C, 0, Bt, 0, H, W, 1, 1, nullptr, nullptr, cm1 ? P.b64 : P.h1, gn,
                    &ns, st, SC(0), SH(0), nullptr, nullptr, h2, pre_b2));
    if (cm1) {
        TCX_TRY(apply_cm(P.b64, P.h1, P.P0, C, 1));
    } else {
        TCX_TRY(norm(1, P.h1, P.P0, C));  // h1 stays raw; its two consumers apply table 1
    }
    // ds1: 4x4/s2 circular on silu(gn(h1))
    TCX_TRY(conv_gn(net->ds1, P.h1, nullptr, C, 0, Bt, 0, H, W, 2, 1, nullptr, nullptr, P.a32, nullptr, &ns, st,
                    SC(1), SH(1), nullptr, nullptr, cm1 ? h2cs : h2, 1));
    // down2
    TCX_TRY(conv_gn(net->down2_0, P.a32, nullptr, C, 0, Bt, 0, H1, W1, 1, 1, nullptr, nullptr, P.b32, gn, &ns, st,
                    nullptr, nullptr, nullptr, nullptr, h2, pre_b2));
    TCX_TRY(norm(2, P.b32, P.P1, C2));
    TCX_TRY(conv_gn(net->down2_1, P.b32, nullptr, C2, 0, Bt, 0, H1, W1, 1, 1, nullptr, nullptr, cm2 ? P.a32 : P.h2, gn,
                    &ns, st, SC(2), SH(2), nullptr, nullptr, h2, pre_b2));
    if (cm2) {
        TCX_TRY(apply_cm(P.a32, P.h2, P.P1, C2, 3));
    } else {
        TCX_TRY(norm(3, P.h2, P.P1, C2));  // h2 raw; consumers apply table 3
    }
    // ds2
    TCX_TRY(conv_gn(net->ds2, P.h2, nullptr, C2, 0, Bt, 0, H1, W1, 2, 1, nullptr, nullptr, P.a16, nullptr, &ns, st,
                    SC(3), SH(3), nullptr, nullptr, cm2 ? h2cs : h2, 1));
    // mid
    TCX_TRY(conv_gn(net->mid_0, P.a16, nullptr, C2, 0, Bt, 0, H2, W2, 1, 1, nullptr, nullptr, P.b16, gn, &ns, st,
                    nullptr, nullptr, nullptr, nullptr, h2, pre_b2));
    TCX_TRY(norm(4, P.b16, P.P2, C2));
    TCX_TRY(conv_gn(net->mid_1, P.b16, nullptr, C2, 0, Bt, 0, H2, W2, 1, 1, nullptr, nullptr, P.a16, gn, &ns, st,
                    SC(4), SH(4), nullptr, nullptr, h2));
    // the attention block needs the normalised tensor itself (input of attn.norm and residual): fp32
    TCX_TRY(gn_tab(net, P, 5, P.P2, C2, gn, ns, st));
    // attention: x_in = a16; b16 = GN(x_in); qkv = 1x1; b16 = attn; a16 = x_in + proj(b16)
    {
        if (h2.on && attn_prep_enabled() && attn_prep_ok(P.P2, C2, groups_of(C2), fmt)) {
            // one pass per image: GN5+SiLU in place, attn.norm statistics, tables and h2 records (round 5)
            TCX_TRY(attn_prep_h2(P.a16, P.b16, Bt, P.P2, C2, P.sc(5), P.sh(5), net->gn_w[6], net->gn_b[6],
                                 groups_of(C2), h2.ovf, fmt, st));
        } else {
            TCX_TRY(tcx_gn_apply_tab(P.a16, P.a16, Bt, P.P2, C2, P.sc(5), P.sh(5), 1, st));
            const int ns_a = std::max(1, P.P2 / 256);
            TCX_TRY(tcx_gn_partials(P.a16, Bt, P.P2, C2, ns_a, gn, st));
            TCX_TRY(gn_tab(net, P, 6, P.P2, C2, gn, ns_a, st));
            if (h2.on) TCX_TRY(gn_apply_tab_h2(P.a16, P.b16, Bt, P.P2, C2, P.sc(6), P.sh(6), 0, h2.ovf, fmt, st));
            else TCX_TRY(tcx_gn_apply_tab(P.a16, P.b16, Bt, P.P2, C2, P.sc(6), P.sh(6), 0, st));
        }
        const tcx_conv& q = net->qkv;
        int dummy = 0;
        // split path with N % 256 == 0 and a supported head dim: the qkv conv writes h2 and the
        // attention runs on f16x3 MFMA (attention_split.hip); else fp32 qkv + fp32-MFMA attention
        const int D = C2 / net->heads;
        const bool split_attn = h2.on && attn_split_enabled() && P.P2 % 256 == 0 && C2 % net->heads == 0 &&
                                (D == 16 || D == 32 || D == 48 || D == 64);
        TCX_TRY(conv_gn(q, P.b16, nullptr, C2, 0, Bt, 0, H2, W2, 1, 0, nullptr, nullptr, P.qkv, nullptr, &dummy, st,
                        nullptr, nullptr, nullptr, nullptr, h2, split_attn ? 1 : 0));
        TCX_REQUIRE(split_attn || !h2.bf, "tcx_unet: bf16 precision needs the split attention (N %% 256 == 0)");
        if (split_attn) TCX_TRY(attention_split(P.qkv, P.b16, Bt, P.P2, C2, net->heads, fmt, st));
        else if (h2.on) TCX_TRY(tcx_attention_h2(P.qkv, P.b16, Bt, P.P2, C2, net->heads, h2.ovf, st));
        else TCX_TRY(tcx_attention(P.qkv, P.b16, Bt, P.P2, C2, net->heads, st));
        const tcx_conv& pr = net->proj;
        TCX_TRY(conv_gn(pr, P.b16, nullptr, C2, 0, Bt, 0, H2, W2, 1, 0, nullptr, P.a16, P.a16, nullptr, &dummy, st,
                        nullptr, nullptr, nullptr, nullptr, h2));
    }
    // us2: bilinear x2 (edge-clamped) into the free b32 buffer, then the circular 3x3 conv -> a32.
    // (The upsample-on-load conv variant re-reads 4 source taps per im2col element and measured
    // slower than this separate 250 MB pass.)
    if (h2.on) TCX_TRY(upsample2x_h2(P.a16, P.b32, Bt, H2, W2, C2, nullptr, nullptr, h2.ovf, fmt, st));
    else TCX_TRY(tcx_upsample2x(P.a16, P.b32, Bt, H2, W2, C2, nullptr, nullptr, st));
    TCX_TRY(conv_gn(net->us2, P.b32, nullptr, C2, 0, Bt, 0, H1, W1, 1, 1, nullptr, nullptr, P.a32, nullptr, &ns, st,
                    nullptr, nullptr, nullptr, nullptr, h2, 1));
    // up2 on cat[a32, silu(gn(h2))]
    TCX_TRY(conv_gn(net->up2_0, P.a32, P.h2, C2, C2, Bt, 0, H1, W1, 1, 1, nullptr, nullptr, P.b32, gn, &ns, st,
                    nullptr, nullptr, SC(3), SH(3), cm2 ? h2cc : h2, pre_b2));
    TCX_TRY(norm(7, P.b32, P.P1, C));
    TCX_TRY(conv_gn(net->up2_1, P.b32, nullptr, C, 0, Bt, 0, H1, W1, 1, 1, nullptr, nullptr, P.a32, gn, &ns, st,
                    SC(7), SH(7), nullptr, nullptr, h2));
    // us1: GN+SiLU of up2's output, bilinear x2 into the free b64, conv.  Split path: the banded
    // upsample applies the GroupNorm+SiLU once per source element while staging (no apply pass);
    // fp32 path: the apply pass in place, then the plain upsample
    // (r03_o, one lane, alternating: 72.7 vs 72.3 images/s against the separate apply pass)
    if (h2.on && upsample_fused_ok(H1, W1, C)) {
        TCX_TRY(gn_tab(net, P, 8, P.P1, C, gn, ns, st));
        TCX_TRY(upsample2x_h2(P.a32, P.b64, Bt, H1, W1, C, P.sc(8), P.sh(8), h2.ovf, fmt, st));
    } else {
        TCX_TRY(norm(8, P.a32, P.P1, C, false));
        if (h2.on) TCX_TRY(upsample2x_h2(P.a32, P.b64, Bt, H1, W1, C, nullptr, nullptr, h2.ovf, fmt, st));
        else TCX_TRY(tcx_upsample2x(P.a32, P.b64, Bt, H1, W1, C, nullptr, nullptr, st));
    }
    TCX_TRY(conv_gn(net->us1, P.b64, nullptr, C, 0, Bt, 0, H, W, 1, 1, nullptr, nullptr, P.a64, nullptr, &ns, st,
                    nullptr, nullptr, nullptr, nullptr, h2, 1));
    // up1 on cat[a64, silu(gn(h1))]
    TCX_TRY(conv_gn(net->up1_0, P.a64, P.h1, C, C, Bt, 0, H, W, 1, 1, nullptr, nullptr, P.b64, gn, &ns, st, nullptr,
                    nullptr, SC(1), SH(1), cm1 ? h2cc : h2, pre_b2));
    TCX_TRY(norm(9, P.b64, P.P0, C));
    TCX_TRY(conv_gn(net->up1_1, P.b64, nullptr, C, 0, Bt, 0, H, W, 1, 1, nullptr, nullptr, P.a64, gn, &ns, st,
                    SC(9), SH(9), nullptr, nullptr, h2, pre_b2));  // b2: the head reads it as bf16
    // head: GN(up1.net.4)+SiLU fused with the out conv's channel reduction
    {
        TCX_TRY(gn_tab(net, P, 10, P.P0, C, gn, ns, st));
        TCX_REQUIRE(C % 4 == 0, "head: C %% 4");
        // up1_1 wrote its output as 2-byte bf16 (pre_b2) at fmt 2, which only k_head8r<3, true> reads: a
        // caller's out_w without 16-B alignment (that kernel's constant loads) is an error, never a
        // fall-through to a head that reads the tensor as fp32
        TCX_REQUIRE(fmt != 2 || (P.P0 % HPR == 0 && C == 96 && aligned16(net->out_w)),
                    "tcx_unet: the 2-byte bf16 head needs out_w 16-byte aligned and H*W %% %d == 0", HPR);
        // register-weight head (r03_ag: 124 -> 118 us at 64^2); k_head8 for other widths / shapes
        if (P.P0 % HPR == 0 && (C == 96 || C == 64 || C == 32) && aligned16(net->out_w)) {  // (16-B constant loads)
            const dim3 gr(Bt * P.P0 / HPR);
            if (C == 96 && fmt == 2)
                hipLaunchKernelGGL((k_head8r<3, true>), gr, dim3(256), 0, st, P.a64, P.P0, P.sc(10), P.sh(10), net->out_w, P.r);
            else if (C == 96) hipLaunchKernelGGL(k_head8r<3>, gr, dim3(256), 0, st, P.a64, P.P0, P.sc(10), P.sh(10), net->out_w, P.r);
            else if (C == 64) hipLaunchKernelGGL(k_head8r<2>, gr, dim3(256), 0, st, P.a64, P.P0, P.sc(10), P.sh(10), net->out_w, P.r);
            else hipLaunchKernelGGL(k_head8r<1>, gr, dim3(256), 0, st, P.a64, P.P0, P.sc(10), P.sh(10), net->out_w, P.r);
            TCX_TRY(check_launch("k_head8r"));
        } else if (P.P0 % HP8 == 0 && (C == 96 || C == 64 || C == 128 || C == 32)) {
            const dim3 g8(Bt * P.P0 / HP8);
            if (C == 96) hipLaunchKernelGGL(k_head8<3>, g8, dim3(256), 0, st, P.a64, P.P0, P.sc(10), P.sh(10), net->out_w, P.r);
            else if (C == 64) hipLaunchKernelGGL(k_head8<2>, g8, dim3(256), 0, st, P.a64, P.P0, P.sc(10), P.sh(10), net->out_w, P.r);
            else if (C == 128) hipLaunchKernelGGL(k_head8<4>, g8, dim3(256), 0, st, P.a64, P.P0, P.sc(10), P.sh(10), net->out_w, P.r);
            else hipLaunchKernelGGL(k_head8<1>, g8, dim3(256), 0, st, P.a64, P.P0, P.sc(10), P.sh(10), net->out_w, P.r);
            TCX_TRY(check_launch("k_head8"));
        } else {
            const size_t shm = ((size_t)HEAD_PX * (C + 4) + 11 * (size_t)C) * sizeof(float);
            const dim3 grid(cdiv(P.P0, HEAD_PX), Bt);
            hipLaunchKernelGGL(k_head, grid, dim3(256), shm, st, P.a64, P.P0, C, P.sc(10), P.sh(10), net->out_w, P.r);
            TCX_TRY(check_launch("k_head"));
        }
    }
    return TCX_OK;
}

int validate(const tcx_unet* net, int B, int H, int W) {
    TCX_REQUIRE(net, "tcx_unet: null net");
    TCX_REQUIRE(B > 0 && H % 4 == 0 && W % 4 == 0 && H >= 8 && W >= 8, "tcx_unet: need B>0 and H,W multiples of 4 (>=8)");
    TCX_REQUIRE(net->base_ch % 4 == 0 && net->base_ch >= 4, "tcx_unet: base_ch must be a multiple of 4");
    TCX_REQUIRE(net->emb_dim <= 256 && net->emb_dim % 2 == 0, "tcx_unet: emb_dim must be even and <= 256");
    TCX_REQUIRE(net->time_ch + net->cond_ch <= 64 && net->y_cont_dim >= 3 && net->y_cont_dim <= 16, "tcx_unet: bad cond dims");
    TCX_REQUIRE((H / 4) * (W / 4) <= 256 || ((H / 4) * (W / 4)) % 256 == 0,
                "tcx_unet: bottleneck attention needs N <= 256 or N %% 256 == 0 tokens");
    TCX_REQUIRE(net->precision >= 0 && net->precision <= 2,
                "tcx_unet: precision must be 0 (fp32), 1 (f16x3) or 2 (bf16)");
    TCX_REQUIRE(net->precision == 0 || (net->base_ch % 32 == 0 && ((H / 4) * (W / 4)) % 32 == 0),
                "tcx_unet: the split paths need base_ch %% 32 == 0 and (H/4)*(W/4) %% 32 == 0");
    TCX_REQUIRE(net->precision != 2 || ((H / 4) * (W / 4)) % 256 == 0,
                "tcx_unet: bf16 precision needs (H/4)*(W/4) %% 256 == 0 (the split attention)");
    return TCX_OK;
}

int launch_step(const StepArgs& a, hipStream_t st) {
    const size_t n = (size_t)a.B * a.H * a.W;
    const int blocks = (int)std::min<size_t>((n + 255) / 256, 16384);
    hipLaunchKernelGGL(k_step, dim3(blocks), dim3(256), 0, st, a);
    return check_launch("k_step");
}

// Batch chunking: one evaluation of B images can run as ceil(B / Bc) passes of Bc images (2*Bc
// U-Net rows with CFG; per-image arithmetic unchanged: GroupNorm is per sample, CFG pairs stay in
// one pass, in-kernel noise is keyed by the global element index).  Meant to keep a pass's
// producer -> consumer hand-offs inside the 256 MB Infinity Cache; measured at B = 128
// (profiles/r01_w_chunk_ab.txt) it LOSES: 59.9 img/s unchunked vs 56.6 / 49.3 / 37.2 at
// Bc = 64 / 32 / 16 (the smaller conv grids lose more than the memory-bound passes gain), so the
// default is one pass (the chunking knob was removed in round 3).
// A pass is capped so that its largest activation (2*Bc*H*W*C fp32)
// stays below 2 GiB: the conv kernels address their operands with 32-bit buffer offsets (the
// 256x256 configuration at base_ch 96: at most 84 images, i.e. 2*42 with CFG, per pass).
int max_pass_rows(const tcx_unet* net, int H, int W) {
    const long long per_row = (long long)H * W * net->base_ch * 4;
    const long long rows = ((1ll << 31) - 1) / per_row;
    return (int)std::max(2ll, rows & ~1ll);
}

int chunk_images(int B, int cap_images) {
    return std::max(1, std::min(B, cap_images));
}

// Concurrent sampling lanes (TCX_LANES = L > 1, default 1): the batch is split into L contiguous
// groups of images, each an independent sampling chain (GroupNorm is per image, CFG pairs stay
// together) advanced step by step on its own HIP stream, so the HBM-bound passes of one lane
// (GroupNorm apply, upsample, head) can run beside the MFMA-bound convs of another.  The noise
// counters use absolute element offsets: the result is identical to one lane.
// Per host thread (round 6: no process-global sampler state besides the thread-local error string):
// tcx_set_sample_lanes sets the calling thread's lane count, which its later workspace queries and
// sampler calls use; 0 means TCX_LANES from the environment.
thread_local int g_lanes = 0;
int lanes_setting() {
    static const int env = [] {
        const char* e = getenv("TCX_LANES");
        return e ? atoi(e) : 1;
    }();
    const int v = g_lanes > 0 ? g_lanes : env;
    return v < 1 ? 1 : (v > 4 ? 4 : v);
}

struct LaneSync {
    hipStream_t s[4];
    hipEvent_t ev[5];
    bool ok = false;
};

// The lane streams and events of the CURRENT device, created on first use on that device (keyed by
// hipGetDevice, so a process sampling on two devices never enqueues one device's lane work on the
// other's streams) and kept for the process's life; guarded by a mutex for concurrent first calls.
LaneSync* lane_sync() {
    static std::mutex mu;
    static std::map<int, LaneSync> per_dev;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    std::lock_guard<std::mutex> lk(mu);
    auto it = per_dev.find(dev);
    if (it == per_dev.end()) {
        LaneSync ls;
        bool ok = true;
        // lane 0 runs on the caller's stream, so L lanes use L streams (the box has 4 hardware queues:
        // a fifth stream would share one and serialise)
        ls.s[0] = nullptr;
        for (int i = 1; i < 4; ++i) ok = ok && hipStreamCreateWithFlags(&ls.s[i], hipStreamNonBlocking) == hipSuccess;
        for (int i = 0; i < 5; ++i) ok = ok && hipEventCreateWithFlags(&ls.ev[i], hipEventDisableTiming) == hipSuccess;
        ls.ok = ok;
        it = per_dev.emplace(dev, ls).first;
    }
    return it->second.ok ? &it->second : nullptr;
}

// workspace of one lane (rows 2*ceil(Bt/(2L)) >= ceil(Bt/L): an upper bound for B or 2B rows)
size_t single_ws_bytes(const tcx_unet* net, int Bt, int H, int W) {
    // Bt = B or 2B (CFG): size for the largest pass of either reading
    const int cap = max_pass_rows(net, H, W);
    const int Btc = std::min(std::min(Bt, 2 * chunk_images(Bt, cap)), cap);
    return make_plan(net, Btc, H, W, nullptr).bytes + 256;
}

// workspace of one lane (rows 2*ceil(Bt/(2L)) >= ceil(Bt/L): an upper bound for B or 2B rows)
size_t lane_ws_bytes(const tcx_unet* net, int Bt, int H, int W, int L) {
    const int rows = 2 * ((Bt + 2 * L - 1) / (2 * L));
    return align_up(single_ws_bytes(net, rows, H, W), 256);
}

}  // namespace
}  // namespace tcx

using namespace tcx;

extern "C" int tcx_set_sample_lanes(int lanes) {
    const int prev = lanes_setting();
    g_lanes = lanes < 0 ? 0 : (lanes > 4 ? 4 : lanes);
    return prev;
}

extern "C" size_t tcx_unet_workspace_size(const tcx_unet* net, int Bt, int H, int W) {
    if (!net) return 0;
    const int L = lanes_setting();
    const size_t one = single_ws_bytes(net, Bt, H, W);
    return L > 1 ? std::max(one, (size_t)L * lane_ws_bytes(net, Bt, H, W, L) + 256) : one;
}

namespace tcx {
namespace {

// Fault injection for the sampler's error paths (tcx_debug_fail_eval): the k-th U-Net evaluation
// after arming returns TCX_EINVAL before launching anything (one shot).  Thread-local: arming it on
// one host thread never fails another thread's evaluations.
thread_local int g_fail_eval = 0;
int injected_failure() {
    if (g_fail_eval <= 0) return TCX_OK;
    if (--g_fail_eval > 0) return TCX_OK;
    set_error("tcx_unet_eval: injected failure (tcx_debug_fail_eval)");
    return TCX_EINVAL;
}

// One (possibly chunked) U-Net evaluation + sampler step.  e_base: element offset of x[0] within
// the whole sampling batch (the Philox noise counter of element i is e_base + i, so a batch
// evaluated in pieces — chunks or concurrent lanes — draws the same noise as in one piece).
int unet_eval_impl(const tcx_unet* net, const float* x, float* x2, const float* t, int t_per_sample,
                   const int64_t* y_cat, const float* y_cont, int B, int H, int W, float guidance, int mode,
                   const float* scal, const float* z, uint64_t seed, uint64_t step, float* x_inout, float* eps_out,
                   void* ws, size_t ws_bytes, hipStream_t st, size_t e_base, CondTab ct = {}) {
    TCX_TRY(validate(net, B, H, W));
    TCX_TRY(injected_failure());
    TCX_REQUIRE(x && t && y_cat && y_cont && ws, "tcx_unet_eval: null pointer");
    TCX_REQUIRE(mode >= 0 && mode <= 5, "tcx_unet_eval: bad mode");
    TCX_REQUIRE(mode == 0 || scal, "tcx_unet_eval: sampler modes need the step table row");
    TCX_REQUIRE(mode == 1 || eps_out, "tcx_unet_eval: eps_out needed");
    TCX_REQUIRE((mode != 1 && mode != 3 && mode != 4) || x_inout, "tcx_unet_eval: x_inout needed");
    TCX_REQUIRE(mode != 3 || x2, "tcx_unet_eval: Heun stage 1 needs x2");
    const int cfg = guidance > 0.f ? 1 : 0;
    const int Bc = chunk_images(B, max_pass_rows(net, H, W) / (cfg ? 2 : 1));
    const int Btc = cfg ? 2 * Bc : Bc;
    char* base = reinterpret_cast<char*>(align_up(reinterpret_cast<uintptr_t>(ws), 256));
    const size_t need = make_plan(net, Btc, H, W, nullptr).bytes;
    TCX_REQUIRE(need + (base - (char*)ws) <= ws_bytes, "tcx_unet_eval: workspace too small (%zu < %zu)", ws_bytes,
                need + 256);
    const size_t HW = (size_t)H * W;
    for (int c0 = 0; c0 < B; c0 += Bc) {
        const int bc = std::min(Bc, B - c0);
        const int Bt = cfg ? 2 * bc : bc;
        Plan P = make_plan(net, Bt, H, W, base);
        const size_t e0 = (size_t)c0 * HW;
        CondTab ctc = ct;
        if (ct.bias_img) ctc.bias_img = ct.bias_img + (size_t)c0 * net->base_ch;
        TCX_TRY(unet_body(net, P, x + e0, bc, t_per_sample ? t + c0 : t, t_per_sample, y_cat + c0,
                          y_cont + (size_t)c0 * net->y_cont_dim, cfg, st, ctc));
        StepArgs a{};
        a.r = P.r; a.out_b = net->out_b; a.B = bc; a.H = H; a.W = W; a.cfg = cfg; a.guidance = guidance;
        a.mode = mode; a.scal = scal; a.x = x + e0; a.x_inout = x_inout ? x_inout + e0 : nullptr;
        a.x2 = x2 ? x2 + e0 : nullptr; a.eps_out = eps_out ? eps_out + e0 : nullptr; a.z = z ? z + e0 : nullptr;
        a.seed = seed; a.step = step; a.e0 = e_base + e0;
        TCX_TRY(launch_step(a, st));
    }
    return TCX_OK;
}

// The sampler's conditioning tables (k_cond_maps + k_bias_table), carved from the CALLER's workspace
// (tcx_sde_workspace_size / tcx_ode_workspace_size size them; the library never allocates): tmaps
// [n_t][time_ch] for the step table's t values, cmaps [B + 1][cond_ch] (row B: null token), then the
// per-(step, image) first-conv bias rows [n_t][B + 1][base_ch].  They replace the reference's
// per-call _make_maps (sde_score_model.py:227-241).  TCX_COND_HOIST=0 keeps the per-evaluation k_cond
// (A/B; the tables are then left unused).
size_t cond_tab_floats(const tcx_unet* net, int B, int n_t) {
    return (size_t)n_t * net->time_ch + (size_t)(B + 1) * net->cond_ch + (size_t)n_t * (B + 1) * net->base_ch;
}
size_t cond_tab_bytes(const tcx_unet* net, int B, int n_t) { return align_up(cond_tab_floats(net, B, n_t) * 4, 256); }

struct CondMaps {
    float* buf = nullptr;
    int time_ch = 0, cond_ch = 0, C0 = 0, B = 0, n_t = 0;
    float* tmaps() const { return buf; }
    float* cmaps() const { return buf + (size_t)n_t * time_ch; }
    float* bias() const { return cmaps() + (size_t)(B + 1) * cond_ch; }
    CondTab at(int step, int b0) const {
        if (!buf) return CondTab{};
        const float* row0 = bias() + (size_t)step * (B + 1) * C0;
        return CondTab{row0 + (size_t)b0 * C0, row0 + (size_t)B * C0};
    }
};

// tab: cond_tab_bytes(net, B, n_t) bytes of the caller's workspace, 256-B aligned
int make_cond_maps(const tcx_unet* net, const float* scal_table, int n_t, const int64_t* y_cat, const float* y_cont,
                   int B, hipStream_t st, void* tab, CondMaps& cm) {
    static const bool on = [] {
        const char* e = getenv("TCX_COND_HOIST");
        return !(e && e[0] == '0');
    }();
    if (!on) return TCX_OK;
    cm.time_ch = net->time_ch; cm.cond_ch = net->cond_ch; cm.C0 = net->base_ch; cm.B = B; cm.n_t = n_t;
    const size_t nbias = (size_t)n_t * (B + 1) * net->base_ch;
    cm.buf = reinterpret_cast<float*>(tab);
    CondArgs a{};
    a.time_w1t = net->time_w1t; a.time_b1 = net->time_b1; a.time_w2t = net->time_w2t; a.time_b2 = net->time_b2;
    a.ttm_wt = net->ttm_wt; a.ttm_b = net->ttm_b; a.tcm_wt = net->tcm_wt; a.tcm_b = net->tcm_b;
    a.cat_emb = net->cat_emb; a.cmlp_w1t = net->cmlp_w1t; a.cmlp_b1 = net->cmlp_b1;
    a.cmlp_w2t = net->cmlp_w2t; a.cmlp_b2 = net->cmlp_b2; a.cout_wt = net->cout_wt; a.cout_b = net->cout_b;
    a.map_wsum = net->map_wsum; a.conv_b = net->down1_0.b;
    a.E = net->emb_dim; a.n_types = net->n_types; a.ycd = net->y_cont_dim;
    a.time_ch = net->time_ch; a.cond_ch = net->cond_ch; a.C0 = net->base_ch;
    hipLaunchKernelGGL(k_cond_maps, dim3(n_t + B + 1), dim3(CT), 0, st, a, scal_table, TCX_SCAL, n_t, y_cat, y_cont, B,
                       cm.tmaps(), cm.cmaps());
    TCX_TRY(check_launch("k_cond_maps"));
    hipLaunchKernelGGL(k_bias_table, dim3((unsigned)((nbias + 255) / 256)), dim3(256), 0, st, cm.tmaps(), cm.cmaps(),
                       net->map_wsum, net->down1_0.b, net->time_ch, net->cond_ch, net->base_ch, B, n_t, cm.bias());
    return check_launch("k_bias_table");
}

// Joins sampling lanes 1..L-1 back into the caller's stream on EVERY exit of a sampler: on success
// through join() (errors reported), on an error return from the destructor (best effort), so no lane
// work is left unordered against the caller's later use or release of the workspace.
struct LaneJoin {
    LaneSync* ls = nullptr;
    int L = 0;
    hipStream_t st = nullptr;
    int join() {
        LaneSync* s = ls;
        ls = nullptr;
        if (!s) return TCX_OK;
        int rc = TCX_OK;
        for (int l = 1; l < L; ++l) {
            if (hipEventRecord(s->ev[l], s->s[l]) != hipSuccess || hipStreamWaitEvent(st, s->ev[l], 0) != hipSuccess) {
                set_error("tcx_sample: joining lane %d to the caller's stream failed", l);
                rc = TCX_EHIP;
            }
        }
        return rc;
    }
    ~LaneJoin() {
        if (ls) {
            const std::string keep = tcx_last_error();  // the error being returned stays the reported one
            (void)join();
            set_error("%s", keep.c_str());
        }
    }
};

}  // namespace
}  // namespace tcx

extern "C" int tcx_unet_eval(const tcx_unet* net, const float* x, float* x2, const float* t, int t_per_sample,
                             const int64_t* y_cat, const float* y_cont, int B, int H, int W, float guidance, int mode,
                             const float* scal, const float* z, uint64_t seed, uint64_t step, float* x_inout,
                             float* eps_out, void* ws, size_t ws_bytes, void* stream) {
    return unet_eval_impl(net, x, x2, t, t_per_sample, y_cat, y_cont, B, H, W, guidance, mode, scal, z, seed, step,
                          x_inout, eps_out, ws, ws_bytes, (hipStream_t)stream, 0);
}

// Workspace of the samplers (one caller allocation; the library allocates nothing): the U-Net
// evaluations' workspace for the (CFG-doubled) rows under the current lane setting, then the
// conditioning tables of the call's n_steps + 1 step-table rows (and for the PF-ODE the drift d and
// the Euler point x_e between them).
namespace tcx {
namespace {
size_t sde_ws_parts(const tcx_unet* net, int B, int H, int W, int n_steps, float guidance, size_t* unet_part) {
    const size_t u = align_up(tcx_unet_workspace_size(net, guidance > 0.f ? 2 * B : B, H, W), 256);
    if (unet_part) *unet_part = u;
    return u + cond_tab_bytes(net, B, n_steps + 1) + 256;
}
size_t ode_ws_parts(const tcx_unet* net, int B, int H, int W, int n_steps, float guidance, size_t* unet_part,
                    size_t* img_part) {
    const size_t u = align_up(tcx_unet_workspace_size(net, guidance > 0.f ? 2 * B : B, H, W), 256);
    const size_t im = align_up((size_t)B * H * W * sizeof(float), 256);
    if (unet_part) *unet_part = u;
    if (img_part) *img_part = im;
    return u + 2 * im + cond_tab_bytes(net, B, n_steps + 1) + 256;
}
}  // namespace
}  // namespace tcx

extern "C" size_t tcx_sde_workspace_size(const tcx_unet* net, int B, int H, int W, int n_steps, float guidance) {
    if (!net || B <= 0 || n_steps < 0) return 0;
    return sde_ws_parts(net, B, H, W, n_steps, guidance, nullptr);
}

extern "C" size_t tcx_ode_workspace_size(const tcx_unet* net, int B, int H, int W, int n_steps, float guidance) {
    if (!net || B <= 0 || n_steps < 0) return 0;
    return ode_ws_parts(net, B, H, W, n_steps, guidance, nullptr, nullptr);
}

extern "C" int tcx_debug_fail_eval(int k) {
    g_fail_eval = k < 0 ? 0 : k;
    return TCX_OK;
}

extern "C" int tcx_sde_sample_shard(const tcx_unet* net, float* x, const int64_t* y_cat, const float* y_cont, int B,
                                    int H, int W, int n_steps, float guidance, const float* scal_table,
                                    const float* noise, uint64_t seed, int flags, uint64_t e_base, void* ws,
                                    size_t ws_bytes, void* stream) {
    TCX_REQUIRE(x && scal_table && n_steps >= 0 && ws, "tcx_sde_sample: bad args");
    TCX_REQUIRE((flags & ~TCX_SAMPLE_X0_HAT) == 0, "tcx_sde_sample: unknown flags %d", flags);
    TCX_TRY(validate(net, B, H, W));
    const int fmode = (flags & TCX_SAMPLE_X0_HAT) ? 5 : 2;
    const size_t img = (size_t)B * H * W;
    size_t ubytes = 0;
    const size_t need = sde_ws_parts(net, B, H, W, n_steps, guidance, &ubytes);
    if (ws_bytes < need) {
        set_error("tcx_sde_sample: workspace too small (%zu < %zu, tcx_sde_workspace_size)", ws_bytes, need);
        return TCX_EWS;
    }
    char* wbase = reinterpret_cast<char*>(align_up(reinterpret_cast<uintptr_t>(ws), 256));
    hipStream_t st = (hipStream_t)stream;
    CondMaps cmap;
    TCX_TRY(make_cond_maps(net, scal_table, n_steps + 1, y_cat, y_cont, B, st, wbase + ubytes, cmap));
    const int L = std::min(lanes_setting(), B);
    const int rows = guidance > 0.f ? 2 * B : B;
    LaneSync* ls = L > 1 ? lane_sync() : nullptr;
    if (ls && ubytes >= (size_t)L * lane_ws_bytes(net, rows, H, W, L)) {
        const size_t HW = (size_t)H * W;
        const size_t lws = lane_ws_bytes(net, rows, H, W, L);
        auto lst = [&](int l) { return l == 0 ? st : ls->s[l]; };
        TCX_REQUIRE(hipEventRecord(ls->ev[4], st) == hipSuccess, "tcx_sde_sample: event record");
        LaneJoin lj;
        for (int l = 1; l < L; ++l)
            TCX_REQUIRE(hipStreamWaitEvent(ls->s[l], ls->ev[4], 0) == hipSuccess, "tcx_sde_sample: stream wait");
        lj.ls = ls; lj.L = L; lj.st = st;
        for (int i = 0; i <= n_steps; ++i) {
            const float* row = scal_table + (size_t)i * TCX_SCAL;
            for (int l = 0; l < L; ++l) {
                const int b0 = (int)((long long)B * l / L), b1 = (int)((long long)B * (l + 1) / L);
                const size_t e = (size_t)b0 * HW;
                if (i < n_steps) {
                    TCX_TRY(unet_eval_impl(net, x + e, nullptr, row, 0, y_cat + b0, y_cont + (size_t)b0 * net->y_cont_dim,
                                           b1 - b0, H, W, guidance, 1, row,
                                           noise ? noise + (size_t)i * img + e : nullptr, seed, (uint64_t)i, x + e,
                                           nullptr, wbase + l * lws, lws, lst(l), e_base + e, cmap.at(i, b0)));
                } else {  // final projection -> image written over x
                    TCX_TRY(unet_eval_impl(net, x + e, nullptr, row, 0, y_cat + b0, y_cont + (size_t)b0 * net->y_cont_dim,
                                           b1 - b0, H, W, guidance, fmode, row, nullptr, seed, 0, nullptr, x + e,
                                           wbase + l * lws, lws, lst(l), e_base + e, cmap.at(i, b0)));
                }
            }
        }
        return lj.join();
    }
    for (int i = 0; i < n_steps; ++i) {
        const float* row = scal_table + (size_t)i * TCX_SCAL;
        TCX_TRY(unet_eval_impl(net, x, nullptr, row, 0, y_cat, y_cont, B, H, W, guidance, 1, row,
                               noise ? noise + (size_t)i * img : nullptr, seed, (uint64_t)i, x, nullptr, wbase, ubytes,
                               st, e_base, cmap.at(i, 0)));
    }
    // final projection -> image written over x
    const float* row = scal_table + (size_t)n_steps * TCX_SCAL;
    return unet_eval_impl(net, x, nullptr, row, 0, y_cat, y_cont, B, H, W, guidance, fmode, row, nullptr, seed, 0,
                          nullptr, x, wbase, ubytes, st, e_base, cmap.at(n_steps, 0));
}

extern "C" int tcx_sde_sample_ex(const tcx_unet* net, float* x, const int64_t* y_cat, const float* y_cont, int B,
                                 int H, int W, int n_steps, float guidance, const float* scal_table, const float* noise,
                                 uint64_t seed, int flags, void* ws, size_t ws_bytes, void* stream) {
    return tcx_sde_sample_shard(net, x, y_cat, y_cont, B, H, W, n_steps, guidance, scal_table, noise, seed, flags, 0,
                                ws, ws_bytes, stream);
}

extern "C" int tcx_sde_sample(const tcx_unet* net, float* x, const int64_t* y_cat, const float* y_cont, int B, int H,
                              int W, int n_steps, float guidance, const float* scal_table, const float* noise,
                              uint64_t seed, void* ws, size_t ws_bytes, void* stream) {
    return tcx_sde_sample_ex(net, x, y_cat, y_cont, B, H, W, n_steps, guidance, scal_table, noise, seed, 0, ws,
                             ws_bytes, stream);
}

extern "C" int tcx_ode_sample_ex(const tcx_unet* net, float* x, const int64_t* y_cat, const float* y_cont, int B,
                                 int H, int W, int n_steps, float guidance, const float* scal_table, int flags, void* ws,
                                 size_t ws_bytes, void* stream) {
    TCX_REQUIRE(x && scal_table && n_steps >= 0 && ws, "tcx_ode_sample: bad args");
    TCX_REQUIRE((flags & ~TCX_SAMPLE_X0_HAT) == 0, "tcx_ode_sample: unknown flags %d", flags);
    TCX_TRY(validate(net, B, H, W));
    const int fmode = (flags & TCX_SAMPLE_X0_HAT) ? 5 : 2;
    size_t ubytes = 0, ibytes = 0;
    const size_t need = ode_ws_parts(net, B, H, W, n_steps, guidance, &ubytes, &ibytes);
    if (ws_bytes < need) {
        set_error("tcx_ode_sample: workspace too small (%zu < %zu, tcx_ode_workspace_size)", ws_bytes, need);
        return TCX_EWS;
    }
    char* wbase = reinterpret_cast<char*>(align_up(reinterpret_cast<uintptr_t>(ws), 256));
    hipStream_t st = (hipStream_t)stream;
    // [U-Net workspace][d][x_e][conditioning tables]
    float* d = reinterpret_cast<float*>(wbase + ubytes);
    float* xe = reinterpret_cast<float*>(wbase + ubytes + ibytes);
    CondMaps cmap;  // stage 2 of step i evaluates at t_{i+1}: table row i + 1
    TCX_TRY(make_cond_maps(net, scal_table, n_steps + 1, y_cat, y_cont, B, st, wbase + ubytes + 2 * ibytes, cmap));
    // concurrent lanes (tcx_set_sample_lanes): image groups on their own streams, d / x_e sliced
    const int L = std::min(lanes_setting(), B);
    const int rows = guidance > 0.f ? 2 * B : B;
    LaneSync* ls = L > 1 ? lane_sync() : nullptr;
    if (ls && ubytes >= (size_t)L * lane_ws_bytes(net, rows, H, W, L)) {
        const size_t HW = (size_t)H * W;
        const size_t lws = lane_ws_bytes(net, rows, H, W, L);
        auto lst = [&](int l) { return l == 0 ? st : ls->s[l]; };
        TCX_REQUIRE(hipEventRecord(ls->ev[4], st) == hipSuccess, "tcx_ode_sample: event record");
        LaneJoin lj;
        for (int l = 1; l < L; ++l)
            TCX_REQUIRE(hipStreamWaitEvent(ls->s[l], ls->ev[4], 0) == hipSuccess, "tcx_ode_sample: stream wait");
        lj.ls = ls; lj.L = L; lj.st = st;
        for (int i = 0; i <= n_steps; ++i) {
            const float* row = scal_table + (size_t)i * TCX_SCAL;
            for (int l = 0; l < L; ++l) {
                const int b0 = (int)((long long)B * l / L), b1 = (int)((long long)B * (l + 1) / L);
                const size_t e = (size_t)b0 * HW;
                const int64_t* yc = y_cat + b0;
                const float* yv = y_cont + (size_t)b0 * net->y_cont_dim;
                char* w = wbase + l * lws;
                if (i < n_steps) {
                    TCX_TRY(unet_eval_impl(net, x + e, xe + e, row, 0, yc, yv, b1 - b0, H, W, guidance, 3, row, nullptr,
                                           0, 0, x + e, d + e, w, lws, lst(l), e, cmap.at(i, b0)));
                    TCX_TRY(unet_eval_impl(net, xe + e, nullptr, row + TCX_SCAL, 0, yc, yv, b1 - b0, H, W, guidance, 4,
                                           row, nullptr, 0, 0, x + e, d + e, w, lws, lst(l), e, cmap.at(i + 1, b0)));
                } else {
                    TCX_TRY(unet_eval_impl(net, x + e, nullptr, row, 0, yc, yv, b1 - b0, H, W, guidance, fmode, row,
                                           nullptr, 0, 0, nullptr, x + e, w, lws, lst(l), e, cmap.at(i, b0)));
                }
            }
        }
        return lj.join();
    }
    for (int i = 0; i < n_steps; ++i) {
        const float* row = scal_table + (size_t)i * TCX_SCAL;
        TCX_TRY(unet_eval_impl(net, x, xe, row, 0, y_cat, y_cont, B, H, W, guidance, 3, row, nullptr, 0, 0, x, d, wbase,
                               ubytes, st, 0, cmap.at(i, 0)));
        const float* row_n = row + TCX_SCAL;  // t_{i+1}
        TCX_TRY(unet_eval_impl(net, xe, nullptr, row_n, 0, y_cat, y_cont, B, H, W, guidance, 4, row, nullptr, 0, 0, x,
                               d, wbase, ubytes, st, 0, cmap.at(i + 1, 0)));
    }
    const float* row = scal_table + (size_t)n_steps * TCX_SCAL;
    return unet_eval_impl(net, x, nullptr, row, 0, y_cat, y_cont, B, H, W, guidance, fmode, row, nullptr, 0, 0, nullptr,
                          x, wbase, ubytes, st, 0, cmap.at(n_steps, 0));
}

extern "C" int tcx_ode_sample(const tcx_unet* net, float* x, const int64_t* y_cat, const float* y_cont, int B, int H,
                              int W, int n_steps, float guidance, const float* scal_table, void* ws, size_t ws_bytes,
                              void* stream) {
    return tcx_ode_sample_ex(net, x, y_cat, y_cont, B, H, W, n_steps, guidance, scal_table, 0, ws, ws_bytes, stream);
}

extern "C" int tcx_randn_at(float* out, size_t n, uint64_t seed, uint64_t stream_id, uint64_t e_off, void* stream) {
    TCX_REQUIRE(out, "tcx_randn: null pointer");
    if (n == 0) return TCX_OK;
    const int blocks = (int)std::min<size_t>((n + 255) / 256, 8192);
    hipLaunchKernelGGL(k_randn, dim3(blocks), dim3(256), 0, (hipStream_t)stream, out, n, seed, stream_id, e_off);
    return check_launch("tcx_randn");
}

extern "C" int tcx_randn(float* out, size_t n, uint64_t seed, uint64_t stream_id, void* stream) {
    return tcx_randn_at(out, n, seed, stream_id, 0, stream);
}
