// Training-path kernels (gfx950): the backward of every non-GEMM op on the three models, the
// loss reductions and the optimiser.  Reference ops (file:line in /root/reference):
//   GroupNorm(+SiLU) fwd stats / bwd ...... src/toycrystals/models/sde_score_model.py:97-111,150
//   bilinear x2 upsample bwd .............. sde_score_model.py:217-222 (nn.Upsample, align_corners=False)
//   attention softmax fwd/bwd ............. sde_score_model.py:150-157 (SDPA math)
//   SiLU / ReLU / Sigmoid fwd/bwd ......... sde_score_model.py:59-60,196; models/vae.py:19-42
//   nn.Embedding bwd ...................... sde_score_model.py:58; models/diffusion_prior.py:80
//   LayerNorm + FiLM fwd/bwd .............. models/diffusion_prior.py:39-54,113
//   MSE loss .............................. sde_score_model.py:399; scripts/train_vae.py:309;
//                                           scripts/train_diffusion_prior.py:265
//   Adam (torch.optim.Adam defaults) ...... scripts/train_sde_score_model.py:160,233-234
//   EMA ................................... scripts/train_sde_score_model.py:236-240
// Reductions are fp64 and in a fixed order (deterministic, run to run).
#include "common.hpp"

#include <cmath>

namespace tcx {
namespace {

__device__ __forceinline__ float sigmoid_f(float v) { return 1.0f / (1.0f + expf(-v)); }

// ---------------------------------------------------------------- GroupNorm forward statistics
// From the fp64 partials [Bt][nsplit][C][2] (conv epilogue or tcx_gn_partials): scale/shift tables
// [Bt][C] (y = x*sc + sh) and the per-(batch, group) mean / rstd kept for the backward.
__global__ __launch_bounds__(256) void k_gn_stats(const double* __restrict__ part, int nsplit, int HW, int C,
                                                  int groups, const float* __restrict__ gamma,
                                                  const float* __restrict__ beta, float eps, float* __restrict__ sc,
                                                  float* __restrict__ sh, float* __restrict__ mean,
                                                  float* __restrict__ rstd) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float* lsc = reinterpret_cast<float*>(smem);
    float* lsh = lsc + ((C + 3) & ~3);
    double* gstat = reinterpret_cast<double*>(lsh + ((C + 3) & ~3));
    double* csum = gstat + 2 * groups;
    const int b = blockIdx.x;
    gn_scale_shift(part, b, nsplit, C, groups, HW, gamma, beta, eps, lsc, lsh, gstat, csum);
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
        sc[(size_t)b * C + c] = lsc[c];
        sh[(size_t)b * C + c] = lsh[c];
    }
    for (int g = threadIdx.x; g < groups; g += blockDim.x) {
        mean[(size_t)b * groups + g] = (float)gstat[2 * g];
        rstd[(size_t)b * groups + g] = (float)gstat[2 * g + 1];
    }
}

// ---------------------------------------------------------------- GroupNorm(+SiLU) backward
// y = act(z), z = x*sc + sh (sc = gamma*rstd, sh = beta - mean*rstd*gamma).  dz = dy * act'(z).
// Pass 1: per (batch, split, channel) fp64 sums of dz and dz*x over a pixel range.
__device__ __forceinline__ float dsilu(float z) {
    const float s = sigmoid_f(z);
    return s * (1.0f + z * (1.0f - s));
}

__global__ __launch_bounds__(256) void k_gn_bwd_partials(const float* __restrict__ x, const float* __restrict__ dy,
                                                         const float* __restrict__ sc, const float* __restrict__ sh,
                                                         int HW, int C, int nsplit, int silu,
                                                         double* __restrict__ part) {
    // grid (nsplit, Bt); thread (channel quad c4, pixel lane) — C/4 quads x (256 / (C/4)) pixel lanes
    extern __shared__ __attribute__((aligned(16))) double red[];  // [lanes][C][2]
    const int b = blockIdx.y, sp = blockIdx.x;
    const int C4 = C / 4;
    const int lanes = max(1, 256 / C4);
    const int tid = threadIdx.x;
    const int c4 = tid % C4, ln = tid / C4;
    const int p0 = (int)((long long)HW * sp / nsplit), p1 = (int)((long long)HW * (sp + 1) / nsplit);
    double s1[4] = {0, 0, 0, 0}, s2[4] = {0, 0, 0, 0};
    if (ln < lanes) {
        const float4 a = *reinterpret_cast<const float4*>(sc + (size_t)b * C + 4 * c4);
        const float4 o = *reinterpret_cast<const float4*>(sh + (size_t)b * C + 4 * c4);
        const float av[4] = {a.x, a.y, a.z, a.w}, ov[4] = {o.x, o.y, o.z, o.w};
        for (int pp = p0 + ln; pp < p1; pp += lanes) {
            const size_t off = ((size_t)b * HW + pp) * C + 4 * c4;
            const float4 xv = *reinterpret_cast<const float4*>(x + off);
            const float4 gv = *reinterpret_cast<const float4*>(dy + off);
            const float xs[4] = {xv.x, xv.y, xv.z, xv.w}, gs[4] = {gv.x, gv.y, gv.z, gv.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float z = fmaf(xs[e], av[e], ov[e]);
                const float dz = silu ? gs[e] * dsilu(z) : gs[e];
                s1[e] += (double)dz;
                s2[e] += (double)dz * (double)xs[e];
            }
        }
    }
    if (ln < lanes) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            red[((size_t)ln * C + 4 * c4 + e) * 2] = s1[e];
            red[((size_t)ln * C + 4 * c4 + e) * 2 + 1] = s2[e];
        }
    }
    __syncthreads();
    for (int c = tid; c < C; c += 256) {
        double a = 0, q = 0;
        for (int l = 0; l < lanes; ++l) {
            a += red[((size_t)l * C + c) * 2];
            q += red[((size_t)l * C + c) * 2 + 1];
        }
        double* d = part + (((size_t)b * nsplit + sp) * C + c) * 2;
        d[0] = a;
        d[1] = q;
    }
}

// Pass 2 (one block per batch): per-channel totals S1 = sum dz, S2 = sum dz*xhat, then
// dx = k1*dz + k2*x + k3 with k1 = rstd*gamma, k2 = a3*rstd, k3 = a2 - a3*rstd*mean,
// a2 = -rstd*A/n, a3 = -rstd*Bg/n, A = sum_{c in g} gamma_c S1_c, Bg = sum gamma_c S2_c.
// Also writes S1/S2 per (batch, channel) for the affine-parameter gradients.
__global__ __launch_bounds__(256) void k_gn_bwd_finalize(const double* __restrict__ part, int nsplit, int HW, int C,
                                                         int groups, const float* __restrict__ mean,
                                                         const float* __restrict__ rstd,
                                                         const float* __restrict__ gamma, float* __restrict__ k1,
                                                         float* __restrict__ k2, float* __restrict__ k3,
                                                         double* __restrict__ s12) {
    extern __shared__ __attribute__((aligned(16))) double sm[];  // [C][2] totals | [groups][2]
    double* tot = sm;
    double* gs = sm + 2 * C;
    const int b = blockIdx.x;
    const int cpg = C / groups;
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
        double a = 0, q = 0;
        for (int sp = 0; sp < nsplit; ++sp) {
            const double* d = part + (((size_t)b * nsplit + sp) * C + c) * 2;
            a += d[0];
            q += d[1];
        }
        const int g = c / cpg;
        const double mu = mean[(size_t)b * groups + g], rs = rstd[(size_t)b * groups + g];
        const double s2 = rs * (q - mu * a);  // sum dz * xhat
        tot[2 * c] = a;
        tot[2 * c + 1] = s2;
        s12[((size_t)b * C + c) * 2] = a;
        s12[((size_t)b * C + c) * 2 + 1] = s2;
    }
    __syncthreads();
    for (int g = threadIdx.x; g < groups; g += blockDim.x) {
        double A = 0, Bg = 0;
        for (int c = g * cpg; c < (g + 1) * cpg; ++c) {
            const double gm = gamma ? gamma[c] : 1.0;
            A += gm * tot[2 * c];
            Bg += gm * tot[2 * c + 1];
        }
        gs[2 * g] = A;
        gs[2 * g + 1] = Bg;
    }
    __syncthreads();
    const double n = (double)HW * cpg;
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
        const int g = c / cpg;
        const double mu = mean[(size_t)b * groups + g], rs = rstd[(size_t)b * groups + g];
        const double gm = gamma ? gamma[c] : 1.0;
        const double a2 = -rs * gs[2 * g] / n, a3 = -rs * gs[2 * g + 1] / n;
        k1[(size_t)b * C + c] = (float)(rs * gm);
        k2[(size_t)b * C + c] = (float)(a3 * rs);
        k3[(size_t)b * C + c] = (float)(a2 - a3 * rs * mu);
    }
}

__global__ __launch_bounds__(256) void k_gn_bwd_apply(const float* __restrict__ x, const float* __restrict__ dy,
                                                      const float* __restrict__ sc, const float* __restrict__ sh,
                                                      const float* __restrict__ k1, const float* __restrict__ k2,
                                                      const float* __restrict__ k3, int Bt, int HW, int C, int silu,
                                                      float* __restrict__ dx, unsigned* __restrict__ amax) {
    const size_t n4 = (size_t)Bt * HW * C / 4;
    const int C4 = C / 4;
    float m = 0.f;  // max |dx| of this thread's elements (reported when amax is given)
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
        const size_t pix = i / C4;
        const int c = (int)(i - pix * C4) * 4;
        const int b = (int)(pix / HW);
        const size_t t = (size_t)b * C + c;
        const float4 xv = reinterpret_cast<const float4*>(x)[i];
        const float4 gv = reinterpret_cast<const float4*>(dy)[i];
        const float xs[4] = {xv.x, xv.y, xv.z, xv.w}, gs[4] = {gv.x, gv.y, gv.z, gv.w};
        float o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const float z = fmaf(xs[e], sc[t + e], sh[t + e]);
            const float dz = silu ? gs[e] * dsilu(z) : gs[e];
            o[e] = fmaf(k1[t + e], dz, fmaf(k2[t + e], xs[e], k3[t + e]));
        }
        reinterpret_cast<float4*>(dx)[i] = make_float4(o[0], o[1], o[2], o[3]);
        m = fmaxf(m, fmaxf(fmaxf(fabsf(o[0]), fabsf(o[1])), fmaxf(fabsf(o[2]), fabsf(o[3]))));
    }
    if (amax) block_amax_publish(m, amax);
}

// d gamma[c] = sum_b S2[b][c], d beta[c] = sum_b S1[b][c]  (32-lane group per channel, fixed tree)
__device__ __forceinline__ double group32_sum_d(double v) {
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o, 32);
    return v;
}

__global__ __launch_bounds__(256) void k_gn_bwd_affine(const double* __restrict__ s12, int Bt, int C,
                                                       float* __restrict__ dgamma, float* __restrict__ dbeta) {
    const int lane = threadIdx.x & 31;
    for (int c = blockIdx.x * 8 + (threadIdx.x >> 5); c < C; c += gridDim.x * 8) {
        double a = 0, q = 0;
        for (int b = lane; b < Bt; b += 32) {
            a += s12[((size_t)b * C + c) * 2];
            q += s12[((size_t)b * C + c) * 2 + 1];
        }
        a = group32_sum_d(a);
        q = group32_sum_d(q);
        if (lane == 0) {
            if (dgamma) dgamma[c] = (float)q;
            if (dbeta) dbeta[c] = (float)a;
        }
    }
}

// ---------------------------------------------------------------- bilinear x2 upsample backward
// Gather form of the adjoint of ATen's upsample_bilinear2d (align_corners=False): low-res row y
// receives from output rows oy in [2y-1, 2y+2] whose (i0, i1) taps hit y, with the same clamped
// source coordinates as the forward (src = max(0, (oy+0.5)/2 - 0.5)).
__device__ __forceinline__ void up_axis(int d, int n, int& i0, int& i1, float& l0, float& l1) {
    float s = 0.5f * ((float)d + 0.5f) - 0.5f;
    s = s < 0.f ? 0.f : s;
    i0 = (int)s;
    i1 = i0 + (i0 < n - 1 ? 1 : 0);
    l1 = s - (float)i0;
    l0 = 1.f - l1;
}

__global__ __launch_bounds__(256) void k_upsample2x_bwd(const float* __restrict__ dy, float* __restrict__ dx, int Bt,
                                                        int H, int W, int C) {
    const int C4 = C / 4;
    const size_t n4 = (size_t)Bt * H * W * C4;
    const int Ho = 2 * H, Wo = 2 * W;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
        const size_t pix = i / C4;
        const int c = (int)(i - pix * C4) * 4;
        const int b = (int)(pix / (H * W));
        const int r = (int)(pix - (size_t)b * H * W);
        const int y = r / W, x = r - (r / W) * W;
        float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int oy = max(0, 2 * y - 1); oy <= min(Ho - 1, 2 * y + 2); ++oy) {
            int a0, a1;
            float w0, w1;
            up_axis(oy, H, a0, a1, w0, w1);
            const float wy = (a0 == y ? w0 : 0.f) + (a1 == y ? w1 : 0.f);
            if (wy == 0.f) continue;
            for (int ox = max(0, 2 * x - 1); ox <= min(Wo - 1, 2 * x + 2); ++ox) {
                int b0, b1;
                float v0, v1;
                up_axis(ox, W, b0, b1, v0, v1);
                const float wx = (b0 == x ? v0 : 0.f) + (b1 == x ? v1 : 0.f);
                if (wx == 0.f) continue;
                const float wgt = wy * wx;
                const float4 g = *reinterpret_cast<const float4*>(dy + (((size_t)b * Ho + oy) * Wo + ox) * C + c);
                acc.x = fmaf(wgt, g.x, acc.x);
                acc.y = fmaf(wgt, g.y, acc.y);
                acc.z = fmaf(wgt, g.z, acc.z);
                acc.w = fmaf(wgt, g.w, acc.w);
            }
        }
        reinterpret_cast<float4*>(dx)[i] = acc;
    }
}

// ---------------------------------------------------------------- column sums (bias grads)
// x [Bt][HW][C] -> part[b][split][C] (fp64).  Block = 256 threads as (channel quad, row lane):
// float4 loads along C, rows strided by the lane count, then an LDS reduction over lanes.
// Scalar variant (C % 4 != 0 or unaligned): (channel, row lane).
template <bool VEC>
__global__ __launch_bounds__(256) void k_colsum_part(const float* __restrict__ x, int HW, int C, int nsplit,
                                                     double* __restrict__ part) {
    extern __shared__ __attribute__((aligned(16))) double cs_red[];  // [lanes][cols]
    const int b = blockIdx.y, sp = blockIdx.x;
    const int p0 = (int)((long long)HW * sp / nsplit), p1 = (int)((long long)HW * (sp + 1) / nsplit);
    const int W = VEC ? 4 : 1;
    const int ncol = C / W;                        // columns handled as units
    const int cpb = ncol < 256 ? ncol : 256;       // columns per pass
    const int lanes = 256 / cpb;
    const int tid = threadIdx.x;
    const int cu = tid % cpb, ln = tid / cpb;
    for (int c0 = 0; c0 < ncol; c0 += cpb) {
        const int col = c0 + cu;
        double s[4] = {0, 0, 0, 0};
        if (ln < lanes && col < ncol) {
#pragma unroll 4
            for (int pp = p0 + ln; pp < p1; pp += lanes) {
                const float* r = x + ((size_t)b * HW + pp) * C + (size_t)col * W;
                if (VEC) {
                    const float4 v = *reinterpret_cast<const float4*>(r);
                    s[0] += v.x; s[1] += v.y; s[2] += v.z; s[3] += v.w;
                } else {
                    s[0] += r[0];
                }
            }
        }
        __syncthreads();
        if (ln < lanes)
            for (int e = 0; e < W; ++e) cs_red[(size_t)ln * cpb * W + cu * W + e] = s[e];
        __syncthreads();
        for (int j = tid; j < cpb * W; j += 256) {
            const int c = c0 * W + j;
            if (c >= C) continue;
            double t = 0;
            for (int l = 0; l < lanes; ++l) t += cs_red[(size_t)l * cpb * W + j];
            part[((size_t)b * nsplit + sp) * C + c] = t;
        }
    }
}

// per (b, c): fold the splits -> per_b (float) and a double row for the total.  One 32-lane group
// per output: lane l sums splits l, l+32, ... then a fixed xor-shuffle tree (deterministic).
__device__ __forceinline__ double group32_sum(double v) {
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o, 32);
    return v;
}

__global__ __launch_bounds__(256) void k_colsum_fold(const double* __restrict__ part, int Bt, int nsplit, int C,
                                                     float* __restrict__ per_b, double* __restrict__ tot_b) {
    const size_t n = (size_t)Bt * C;
    const int lane = threadIdx.x & 31;
    for (size_t i = blockIdx.x * (size_t)8 + (threadIdx.x >> 5); i < n; i += (size_t)gridDim.x * 8) {
        const int b = (int)(i / C), c = (int)(i - (size_t)b * C);
        const double* pp = part + (size_t)b * nsplit * C + c;
        double s = 0;
        for (int sp = lane; sp < nsplit; sp += 32) s += pp[(size_t)sp * C];
        s = group32_sum(s);
        if (lane == 0) {
            if (per_b) per_b[i] = (float)s;
            tot_b[i] = s;
        }
    }
}

// Column sums of one short [rows][C] matrix (a Linear bias gradient over the batch, rows <= 4096)
// in ONE launch: block = 32 float4 column quads x 8 row groups; each thread sums its rows in fp64,
// then a fixed-order fold over the 8 groups (deterministic).  The general path (partials, fold,
// total) launched 4 blocks for a 256 x 4096 matrix and three kernels per bias.
__global__ __launch_bounds__(256) void k_colsum_small(const float* __restrict__ x, int rows, int C,
                                                      float* __restrict__ total, float beta) {
    __shared__ double red[8][32][4];
    const int q = blockIdx.x * 32 + (threadIdx.x & 31);  // column quad
    const int rg = threadIdx.x >> 5;
    const bool ok = q * 4 < C;
    double s0 = 0, s1 = 0, s2 = 0, s3 = 0;
    if (ok) {
#pragma unroll 8
        for (int r = rg; r < rows; r += 8) {
            const float4 v = *reinterpret_cast<const float4*>(x + (size_t)r * C + q * 4);
            s0 += v.x; s1 += v.y; s2 += v.z; s3 += v.w;
        }
    }
    red[rg][threadIdx.x & 31][0] = s0;
    red[rg][threadIdx.x & 31][1] = s1;
    red[rg][threadIdx.x & 31][2] = s2;
    red[rg][threadIdx.x & 31][3] = s3;
    __syncthreads();
    if (threadIdx.x < 128) {
        const int cq = threadIdx.x >> 2, e = threadIdx.x & 3;
        const int c = (blockIdx.x * 32 + cq) * 4 + e;
        if (c < C) {
            double t = 0;
#pragma unroll
            for (int g = 0; g < 8; ++g) t += red[g][cq][e];
            total[c] = beta != 0.f ? beta * total[c] + (float)t : (float)t;
        }
    }
}

// fold for many splits (a flattened [rows][C] matrix: Bt = 1, nsplit up to 4096): one block per
// (b, c), 256 threads striding the splits, then a fixed wave-xor + cross-wave fold.  The 32-lane
// fold above left one lane group per output walking 64 strided partials each (~46 us per bias).
__global__ __launch_bounds__(256) void k_colsum_fold_wide(const double* __restrict__ part, int nsplit, int C,
                                                          float* __restrict__ per_b, double* __restrict__ tot_b) {
    __shared__ double wsum[4];
    const size_t i = blockIdx.x;  // b * C + c
    const int b = (int)(i / C), c = (int)(i - (size_t)b * C);
    const double* pp = part + (size_t)b * nsplit * C + c;
    double s = 0;
    for (int sp = threadIdx.x; sp < nsplit; sp += 256) s += pp[(size_t)sp * C];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        const double t = (wsum[0] + wsum[1]) + (wsum[2] + wsum[3]);
        if (per_b) per_b[i] = (float)t;
        tot_b[i] = t;
    }
}

__global__ __launch_bounds__(256) void k_colsum_total(const double* __restrict__ tot_b, int Bt, int C,
                                                      float* __restrict__ total, float beta) {
    const int lane = threadIdx.x & 31;
    for (int c = blockIdx.x * 8 + (threadIdx.x >> 5); c < C; c += gridDim.x * 8) {
        double t = 0;
        for (int b = lane; b < Bt; b += 32) t += tot_b[(size_t)b * C + c];
        t = group32_sum(t);
        if (lane == 0) total[c] = beta != 0.f ? beta * total[c] + (float)t : (float)t;
    }
}

// ---------------------------------------------------------------- softmax rows (attention)
// One wave per row; rows of length n <= 1024.  P = softmax(S) ; dS = P * (dP - sum_j dP_j P_j).
__global__ __launch_bounds__(256) void k_softmax_rows(const float* __restrict__ S, float* __restrict__ P, long long rows,
                                                      int n) {
    const long long row = blockIdx.x * 4LL + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (row >= rows) return;
    const float* s = S + row * n;
    float* pr = P + row * n;
    float mx = -INFINITY;
    for (int j = lane; j < n; j += 64) mx = fmaxf(mx, s[j]);
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
    float sum = 0.f;
    for (int j = lane; j < n; j += 64) sum += expf(s[j] - mx);
    for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
    const float inv = 1.0f / sum;
    for (int j = lane; j < n; j += 64) pr[j] = expf(s[j] - mx) * inv;
}

__global__ __launch_bounds__(256) void k_softmax_bwd_rows(const float* __restrict__ P, const float* __restrict__ dP,
                                                          float* __restrict__ dS, long long rows, int n) {
    const long long row = blockIdx.x * 4LL + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (row >= rows) return;
    const float* pr = P + row * n;
    const float* g = dP + row * n;
    float dot = 0.f;
    for (int j = lane; j < n; j += 64) dot = fmaf(pr[j], g[j], dot);
    for (int o = 32; o > 0; o >>= 1) dot += __shfl_xor(dot, o);
    float* d = dS + row * n;
    for (int j = lane; j < n; j += 64) d[j] = pr[j] * (g[j] - dot);
}

// ---------------------------------------------------------------- activations
// act: 1 relu, 2 sigmoid, 3 silu.  Backward takes the pre-activation z.
__global__ void k_act_fwd(const float* __restrict__ z, float* __restrict__ y, size_t n, int act) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const float v = z[i];
        y[i] = act == 1 ? fmaxf(v, 0.f) : act == 2 ? sigmoid_f(v) : silu_f(v);
    }
}

__global__ void k_act_bwd(const float* __restrict__ z, const float* __restrict__ dy, float* __restrict__ dz, size_t n,
                          int act) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const float v = z[i], g = dy[i];
        float d;
        if (act == 1) d = v > 0.f ? g : 0.f;
        else if (act == 2) {
            const float s = sigmoid_f(v);
            d = g * (s * (1.0f - s));
        } else d = g * dsilu(v);
        dz[i] = d;
    }
}

// ---------------------------------------------------------------- MSE loss
// loss = mean((a - b)^2): per-block fp64 partials, then one block folds them in order.
__global__ __launch_bounds__(256) void k_sqdiff_part(const float* __restrict__ a, const float* __restrict__ b, size_t n,
                                                     double* __restrict__ part) {
    __shared__ double red[256];
    double s = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const float d = a[i] - b[i];
        s += (double)(d * d);
    }
    red[threadIdx.x] = s;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

__global__ void k_sqdiff_fold(const double* __restrict__ part, int nb, size_t n, float* __restrict__ out) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        double s = 0;
        for (int i = 0; i < nb; ++i) s += part[i];
        out[0] = (float)(s / (double)n);
    }
}

// d = g * 2 (a - b) / n   (grad of mean((a-b)^2) w.r.t. a; g is a device scalar)
__global__ void k_mse_bwd(const float* __restrict__ a, const float* __restrict__ b, size_t n,
                          const float* __restrict__ g, float* __restrict__ da) {
    const float s = 2.0f * g[0] / (float)n;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        da[i] = s * (a[i] - b[i]);
}

// ---------------------------------------------------------------- embedding backward
// dW[r][j] = sum_{b: idx[b] == r} dout[b][j]  (gather per row: deterministic)
__global__ void k_embedding_bwd(const int64_t* __restrict__ idx, const float* __restrict__ dout, int B, int rows,
                                int E, float* __restrict__ dW) {
    const size_t n = (size_t)rows * E;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const int r = (int)(i / E), j = (int)(i - (size_t)r * E);
        float s = 0.f;
        for (int b = 0; b < B; ++b)
            if (idx[b] == r) s += dout[(size_t)b * E + j];
        dW[i] = s;
    }
}

// ---------------------------------------------------------------- LayerNorm (+FiLM)
// y = l*(1+gm) + bt with l = (x*rstd - mean*rstd)*w + b (ATen's CPU LayerNorm form), gm/bt the
// two halves of a FiLM row gb[r][0:Wd | Wd:2Wd] (null: plain LayerNorm).  One block per row.
__global__ __launch_bounds__(256) void k_ln_fwd(const float* __restrict__ x, float* __restrict__ y, int Wd,
                                                const float* __restrict__ w, const float* __restrict__ bb,
                                                const float* __restrict__ gb, int ld_gb, float eps,
                                                float* __restrict__ mean, float* __restrict__ rstd) {
    __shared__ double red[2][256];
    const int r = blockIdx.x;
    const float* xr = x + (size_t)r * Wd;
    double s = 0, q = 0;
    for (int c = threadIdx.x; c < Wd; c += 256) {
        const double v = xr[c];
        s += v;
        q += v * v;
    }
    red[0][threadIdx.x] = s;
    red[1][threadIdx.x] = q;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) {
            red[0][threadIdx.x] += red[0][threadIdx.x + o];
            red[1][threadIdx.x] += red[1][threadIdx.x + o];
        }
        __syncthreads();
    }
    const double mu = red[0][0] / Wd;
    double var = red[1][0] / Wd - mu * mu;
    var = var < 0 ? 0 : var;
    const float rs = (float)(1.0 / sqrt(var + (double)eps));
    const float muf = (float)mu;
    if (threadIdx.x == 0) {
        mean[r] = muf;
        rstd[r] = rs;
    }
    const float sft = -muf * rs;
    for (int c = threadIdx.x; c < Wd; c += 256) {
        float l = fmaf(xr[c], rs, sft) * w[c] + bb[c];
        if (gb) l = l * (1.0f + gb[(size_t)r * ld_gb + c]) + gb[(size_t)r * ld_gb + Wd + c];
        y[(size_t)r * Wd + c] = l;
    }
}

// Backward of k_ln_fwd: dx, and per-row products for the column reductions: dwrow = dl*xhat,
// dbrow = dl (summed over rows by tcx_colsum), dgb row = [dh*l | dh] (the FiLM linear's output grad).
__global__ __launch_bounds__(256) void k_ln_bwd(const float* __restrict__ x, const float* __restrict__ dh, int Wd,
                                                const float* __restrict__ w, const float* __restrict__ bb,
                                                const float* __restrict__ gb, int ld_gb,
                                                const float* __restrict__ mean, const float* __restrict__ rstd,
                                                float* __restrict__ dx, float* __restrict__ dwrow,
                                                float* __restrict__ dbrow, float* __restrict__ dgb) {
    __shared__ double red[2][256];
    const int r = blockIdx.x;
    const float mu = mean[r], rs = rstd[r];
    const float* xr = x + (size_t)r * Wd;
    const float* gr = dh + (size_t)r * Wd;
    double s1 = 0, s2 = 0;
    for (int c = threadIdx.x; c < Wd; c += 256) {
        const float xh = (xr[c] - mu) * rs;
        float dl = gr[c];
        if (gb) {
            const float l = xh * w[c] + bb[c];
            dgb[(size_t)r * 2 * Wd + c] = dl * l;
            dgb[(size_t)r * 2 * Wd + Wd + c] = dl;
            dl = dl * (1.0f + gb[(size_t)r * ld_gb + c]);
        }
        dwrow[(size_t)r * Wd + c] = dl * xh;
        dbrow[(size_t)r * Wd + c] = dl;
        const float dxh = dl * w[c];
        s1 += dxh;
        s2 += (double)dxh * xh;
    }
    red[0][threadIdx.x] = s1;
    red[1][threadIdx.x] = s2;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) {
            red[0][threadIdx.x] += red[0][threadIdx.x + o];
            red[1][threadIdx.x] += red[1][threadIdx.x + o];
        }
        __syncthreads();
    }
    const float m1 = (float)(red[0][0] / Wd), m2 = (float)(red[1][0] / Wd);
    for (int c = threadIdx.x; c < Wd; c += 256) {
        const float xh = (xr[c] - mu) * rs;
        float dl = gr[c];
        if (gb) dl = dl * (1.0f + gb[(size_t)r * ld_gb + c]);
        const float dxh = dl * w[c];
        dx[(size_t)r * Wd + c] = rs * (dxh - m1 - xh * m2);
    }
}

// ---------------------------------------------------------------- optimiser
// torch.optim.Adam single-tensor step (torch/optim/adam.py, weight_decay folded into the grad):
//   m.lerp_(g, 1-b1); v = v*b2 + (1-b2)*g*g; denom = sqrt(v)/bc2_sqrt + eps; p += (-step_size)*m/denom
constexpr int kMaxAdamTensors = 48;  // tensors per launch, passed by value in the kernel arguments
struct AdamArgs {
    tcx_adam_tensor t[kMaxAdamTensors];
    float w1, b2, w2, bc2s, eps, neg_step, wd;
};

__global__ __launch_bounds__(256) void k_adam(AdamArgs a) {
    const tcx_adam_tensor T = a.t[blockIdx.y];
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < T.n; i += (long long)gridDim.x * blockDim.x) {
        float g = T.g[i];
        const float p = T.p[i];
        if (a.wd != 0.f) g = g + a.wd * p;
        float m = T.m[i];
        // ATen lerp: weight < 0.5 ? self + w*(end-self) : end - (end-self)*(1-w)
        m = a.w1 < 0.5f ? m + a.w1 * (g - m) : g - (g - m) * (1.0f - a.w1);
        float v = T.v[i] * a.b2;
        v = v + (a.w2 * g) * g;
        const float denom = sqrtf(v) / a.bc2s + a.eps;
        T.m[i] = m;
        T.v[i] = v;
        T.p[i] = p + (a.neg_step * m) / denom;
    }
}

// p_ema = p_ema * d + (1-d) * p   (mul_(decay).add_(p, alpha=1-decay))
struct EmaArgs {
    tcx_adam_tensor t[kMaxAdamTensors];
    float d, w;
};

__global__ __launch_bounds__(256) void k_ema(EmaArgs a) {
    const tcx_adam_tensor T = a.t[blockIdx.y];
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < T.n; i += (long long)gridDim.x * blockDim.x)
        T.p[i] = T.p[i] * a.d + a.w * T.g[i];
}

// ---------------------------------------------------------------- conditioning inputs (score net)
// te = timestep_embedding(t, E) (sde_score_model.py:17-32: [cos, sin] of (2 pi t) * freqs),
// yv = y_cont with y[1] = sin(theta), y[2] = cos(y[1]) (the view quirk, :75-78), yc = clamp(y_cat, 0, n_types).
__global__ void k_cond_inputs(const float* __restrict__ t, const int64_t* __restrict__ y_cat,
                              const float* __restrict__ y_cont, int B, int E, int n_types, int ycd,
                              float* __restrict__ te, float* __restrict__ yv, int64_t* __restrict__ yc) {
    const int b = blockIdx.x;
    const int half = E / 2;
    for (int j = threadIdx.x; j < E; j += blockDim.x) {
        const int k = j < half ? j : j - half;
        const float fr = expf((-9.210340371976184f * (float)k) / (float)(half > 1 ? half - 1 : 1));
        const float arg = (6.283185307179586f * t[b]) * fr;
        te[(size_t)b * E + j] = (j < half) ? cosf(arg) : (j < 2 * half ? sinf(arg) : 0.f);
    }
    for (int j = threadIdx.x; j < ycd; j += blockDim.x) {
        float v = y_cont[(size_t)b * ycd + j];
        const float th = y_cont[(size_t)b * ycd + 1];
        if (j == 1) v = sinf(th);
        if (j == 2) v = cosf(sinf(th));
        yv[(size_t)b * ycd + j] = v;
    }
    if (threadIdx.x == 0) {
        long long c = y_cat[b];
        yc[b] = c < 0 ? 0 : (c > n_types ? n_types : c);
    }
}

// prior timestep embedding (diffusion_prior.py:11-25): freqs = exp(-linspace(0, ln 1e4, half)),
// args = t * freqs (no 2 pi), [sin, cos].  freqs come from the host (torch.linspace bits).
__global__ void k_prior_temb(const int64_t* __restrict__ t, const float* __restrict__ freqs, int B, int E,
                             float* __restrict__ te) {
    const int b = blockIdx.x, half = E / 2;
    for (int j = threadIdx.x; j < E; j += blockDim.x) {
        const int k = j < half ? j : j - half;
        const float arg = (float)t[b] * freqs[k];
        te[(size_t)b * E + j] = j < half ? sinf(arg) : (j < 2 * half ? cosf(arg) : 0.f);
    }
}

__global__ void k_embedding_fwd(const int64_t* __restrict__ idx, const float* __restrict__ W, int B, int E,
                                float* __restrict__ out) {
    const size_t n = (size_t)B * E;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const int b = (int)(i / E), j = (int)(i - (size_t)b * E);
        out[i] = W[(size_t)idx[b] * E + j];
    }
}

// dst[r][c] = beta * dst[r][c] + src[r][c] with row strides (concat / split of feature columns)
__global__ void k_copy2d(const float* __restrict__ src, long long lds, float* __restrict__ dst, long long ldd, int rows,
                         int cols, float beta) {
    const size_t n = (size_t)rows * cols;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const int r = (int)(i / cols), c = (int)(i - (size_t)r * cols);
        const float v = src[r * lds + c];
        float* d = dst + r * ldd + c;
        *d = beta != 0.f ? beta * *d + v : v;
    }
}

// [B][HW][C] <-> [B][C][HW]
__global__ void k_transpose_bhc(const float* __restrict__ src, float* __restrict__ dst, int B, int R, int C) {
    // dst[b][c][r] = src[b][r][c]
    const size_t n = (size_t)B * R * C;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const int b = (int)(i / ((size_t)R * C));
        const size_t rem = i - (size_t)b * R * C;
        const int c = (int)(rem / R), r = (int)(rem - (size_t)c * R);
        dst[i] = src[((size_t)b * R + r) * C + c];
    }
}

// First conv of down1 with the spatially-constant map channels folded (sde_score_model.py:246):
// bias_b[b][co] = bias[co] + sum_c maps[b][c] * sum_tap w[co][1+c][tap]   (w [C0][1+nm][ks][ks])
__global__ void k_first_conv_bias(const float* __restrict__ maps, const float* __restrict__ w,
                                  const float* __restrict__ bias, int B, int C0, int nm, int ks,
                                  float* __restrict__ bias_b) {
    const int n = B * C0, kk = ks * ks;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const int b = i / C0, co = i - (i / C0) * C0;
        float s = bias ? bias[co] : 0.f;
        for (int c = 0; c < nm; ++c) {
            float ws = 0.f;
            for (int tp = 0; tp < kk; ++tp) ws += w[((size_t)co * (1 + nm) + 1 + c) * kk + tp];
            s = fmaf(maps[(size_t)b * nm + c], ws, s);
        }
        bias_b[i] = s;
    }
}

// Its backward from S[b][co] = sum_p dY[b,p,co]:  dmaps[b][c] = sum_co S[b][co] * wsum[co][c];
// dw[co][1+c][tap] = sum_b S[b][co] maps[b][c] (every tap; circular padding keeps the map
// constant); dw[co][0][tap] = dwx[co][tap] (the x_t channel from tcx_conv_wgrad); db[co] = sum_b S.
__global__ void k_first_conv_bwd(const float* __restrict__ S, const float* __restrict__ maps,
                                 const float* __restrict__ w, const float* __restrict__ dwx, int B, int C0, int nm,
                                 int ks, float* __restrict__ dmaps, float* __restrict__ dw, float* __restrict__ db) {
    const int kk = ks * ks;
    const int tid = blockIdx.x * blockDim.x + threadIdx.x, nth = gridDim.x * blockDim.x;
    if (dmaps)
        for (int i = tid; i < B * nm; i += nth) {
            const int b = i / nm, c = i - (i / nm) * nm;
            float s = 0.f;
            for (int co = 0; co < C0; ++co) {
                float ws = 0.f;
                for (int tp = 0; tp < kk; ++tp) ws += w[((size_t)co * (1 + nm) + 1 + c) * kk + tp];
                s = fmaf(S[(size_t)b * C0 + co], ws, s);
            }
            dmaps[i] = s;
        }
    if (dw)
        for (int i = tid; i < C0 * (1 + nm); i += nth) {
            const int co = i / (1 + nm), c = i - (i / (1 + nm)) * (1 + nm);
            if (c == 0) {
                for (int tp = 0; tp < kk; ++tp) dw[(size_t)i * kk + tp] = dwx[(size_t)co * kk + tp];
            } else {
                float s = 0.f;
                for (int b = 0; b < B; ++b) s = fmaf(S[(size_t)b * C0 + co], maps[(size_t)b * nm + c - 1], s);
                for (int tp = 0; tp < kk; ++tp) dw[(size_t)i * kk + tp] = s;
            }
        }
    if (db)
        for (int co = tid; co < C0; co += nth) {
            float s = 0.f;
            for (int b = 0; b < B; ++b) s += S[(size_t)b * C0 + co];
            db[co] = s;
        }
}

// diffusion_loss_eps forward data path (sde_score_model.py:380-389): t = u^p; int_beta =
// bmin t + c2 t^2; a = exp(-0.5 int_beta); s = sqrt(max(1 - a^2, 1e-8)); x_t = a (2 x0 - 1) + s eps.
__global__ void k_qsample_vp(const float* __restrict__ x0, const float* __restrict__ eps, const float* __restrict__ u,
                             float t_power, float bmin, float c2, int B, int HW, float* __restrict__ t_out,
                             float* __restrict__ x_t) {
    const size_t n = (size_t)B * HW;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const int b = (int)(i / HW);
        const float uv = u[b];
        const float t = t_power == 1.0f ? uv : (t_power == 2.0f ? uv * uv : powf(uv, t_power));
        const float ib = bmin * t + c2 * (t * t);
        const float a = expf(-0.5f * ib);
        const float s = sqrtf(fmaxf(1.0f - a * a, 1e-8f));
        const float xv = x0[i] * 2.0f - 1.0f;
        x_t[i] = a * xv + s * eps[i];
        if (i - (size_t)b * HW == 0) t_out[b] = t;
    }
}

// CFG condition dropout (sde_score_model.py:392-397): drop = r < p -> y_cat = n_types, y_cont = 0
__global__ void k_cond_drop(const int64_t* __restrict__ y_cat, const float* __restrict__ y_cont,
                            const float* __restrict__ r, float p, int B, int ycd, int n_types,
                            int64_t* __restrict__ oc, float* __restrict__ ov) {
    for (int b = blockIdx.x * blockDim.x + threadIdx.x; b < B; b += gridDim.x * blockDim.x) {
        const bool d = r && r[b] < p;
        oc[b] = d ? (int64_t)n_types : y_cat[b];
        for (int j = 0; j < ycd; ++j) ov[(size_t)b * ycd + j] = d ? 0.f : y_cont[(size_t)b * ycd + j];
    }
}

// prior training q_sample (train_diffusion_prior.py:256-260): t = clamp(long(u^2 * T), 0, T-1);
// z_t = sqrt_ab[t] z0 + sqrt_1mab[t] eps
__global__ void k_prior_qsample(const float* __restrict__ z0, const float* __restrict__ eps, const float* __restrict__ u,
                                const float* __restrict__ sab, const float* __restrict__ s1mab, int T, int B, int Z,
                                int64_t* __restrict__ t_out, float* __restrict__ z_t) {
    const size_t n = (size_t)B * Z;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const int b = (int)(i / Z);
        const float uv = u[b];
        long long t = (long long)((uv * uv) * (float)T);
        t = t < 0 ? 0 : (t > T - 1 ? T - 1 : t);
        z_t[i] = sab[t] * z0[i] + s1mab[t] * eps[i];
        if (i - (size_t)b * Z == 0) t_out[b] = t;
    }
}

// VAE reparameterise (vae.py:57-60): z = mu + exp(0.5 lv) * eps; backward adds into dmu/dlv.
__global__ void k_reparam(const float* __restrict__ mu, const float* __restrict__ lv, const float* __restrict__ eps,
                          size_t n, float* __restrict__ z) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        z[i] = mu[i] + expf(0.5f * lv[i]) * eps[i];
}

__global__ void k_reparam_bwd(const float* __restrict__ lv, const float* __restrict__ eps, const float* __restrict__ dz,
                              size_t n, float* __restrict__ dmu, float* __restrict__ dlv, float beta) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const float g = dz[i];
        const float dl = g * eps[i] * (0.5f * expf(0.5f * lv[i]));
        dmu[i] = beta != 0.f ? beta * dmu[i] + g : g;
        dlv[i] = beta != 0.f ? beta * dlv[i] + dl : dl;
    }
}

// kl_stats (train_vae.py:17-36): kl_dim = 0.5 (mu^2 + e^lv - 1 - lv); out = {mean_b sum_d max(kl_dim, fb),
// mean_b sum_d kl_dim}.  One block, fixed-order fp64.
__global__ __launch_bounds__(256) void k_vae_kl(const float* __restrict__ mu, const float* __restrict__ lv, int B, int Z,
                                                float fb, float* __restrict__ out) {
    __shared__ double red[2][256];
    double s_used = 0, s_raw = 0;
    for (int i = threadIdx.x; i < B * Z; i += 256) {
        const float m = mu[i], l = lv[i];
        const float kd = 0.5f * (m * m + expf(l) - 1.0f - l);
        s_raw += kd;
        s_used += fb > 0.f ? fmaxf(kd, fb) : kd;
    }
    red[0][threadIdx.x] = s_used;
    red[1][threadIdx.x] = s_raw;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) {
            red[0][threadIdx.x] += red[0][threadIdx.x + o];
            red[1][threadIdx.x] += red[1][threadIdx.x + o];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        out[0] = (float)(red[0][0] / B);
        out[1] = (float)(red[1][0] / B);
    }
}

// grad of g * kl_used w.r.t. mu / lv (torch.maximum passes 1 where kl_dim > fb, 0.5 on ties)
__global__ void k_vae_kl_bwd(const float* __restrict__ mu, const float* __restrict__ lv, int B, int Z, float fb,
                             const float* __restrict__ g, float* __restrict__ dmu, float* __restrict__ dlv, float beta) {
    const float s = g[0] / (float)B;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < B * Z; i += gridDim.x * blockDim.x) {
        const float m = mu[i], l = lv[i];
        float w = 1.f;
        if (fb > 0.f) {
            const float kd = 0.5f * (m * m + expf(l) - 1.0f - l);
            w = kd > fb ? 1.f : (kd == fb ? 0.5f : 0.f);
        }
        const float gm = s * w * m, gl = s * w * 0.5f * (expf(l) - 1.0f);
        dmu[i] = beta != 0.f ? beta * dmu[i] + gm : gm;
        dlv[i] = beta != 0.f ? beta * dlv[i] + gl : gl;
    }
}

// CondVAE._y_vec (vae.py:45-48): [one_hot(y_cat, n_types) | y_cont], times the training-time keep
// mask (keep_u >= cond_drop, vae.py:65-67) when keep_u is given.
__global__ void k_vae_yvec(const int64_t* __restrict__ y_cat, const float* __restrict__ y_cont,
                           const float* __restrict__ keep_u, float cond_drop, int B, int n_types, int ycd,
                           float* __restrict__ out) {
    const int D = n_types + ycd;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < B * D; i += gridDim.x * blockDim.x) {
        const int b = i / D, j = i - (i / D) * D;
        float v = j < n_types ? (y_cat[b] == j ? 1.f : 0.f) : y_cont[(size_t)b * ycd + (j - n_types)];
        if (keep_u) v = v * (keep_u[b] >= cond_drop ? 1.f : 0.f);
        out[i] = v;
    }
}

// DDIM eta = 0 step (diffusion_prior.py:226-250): z0 = (z - sqrt(1-abar_t) eps) / (sqrt(abar_t) + 1e-8);
// last step returns z0, else z = sqrt(abar_prev) z0 + sqrt(1-abar_prev) eps.
__global__ void k_ddim_step(float* __restrict__ z, const float* __restrict__ eps, size_t n, float abar_t,
                            float abar_prev, int last) {
    const float sa = sqrtf(abar_t), s1 = sqrtf(1.0f - abar_t);
    const float sp = sqrtf(abar_prev), s1p = sqrtf(1.0f - abar_prev);
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const float e = eps[i];
        const float z0 = (z[i] - s1 * e) / (sa + 1e-8f);
        z[i] = last ? z0 : sp * z0 + s1p * e;
    }
}

// DiffusionSchedule.q_sample (diffusion_prior.py:194-201) with a given t
__global__ void k_q_sample_t(const float* __restrict__ z0, const int64_t* __restrict__ t, const float* __restrict__ eps,
                             const float* __restrict__ sab, const float* __restrict__ s1mab, int B, int Z,
                             float* __restrict__ out) {
    const size_t n = (size_t)B * Z;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const int b = (int)(i / Z);
        const long long tt = t[b];
        out[i] = sab[tt] * z0[i] + s1mab[tt] * eps[i];
    }
}

// Device-side data pipeline (ToyCrystalsDiskDataset.__getitem__, disk_data.py:27-31):
// out[b][p] = x_u8[idx[b]][p] / 255.0 for a shuffled batch of indices.
__global__ void k_u8_gather(const uint8_t* __restrict__ x, const int64_t* __restrict__ idx, int B, int npix,
                            float* __restrict__ out) {
    const size_t n = (size_t)B * npix;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const int b = (int)(i / npix), p = (int)(i - (size_t)b * npix);
        out[i] = (float)x[(size_t)idx[b] * npix + p] / 255.0f;
    }
}

int grid1d(size_t n, int cap = 8192) { return (int)std::max<size_t>(1, std::min<size_t>((n + 255) / 256, cap)); }

}  // namespace
}  // namespace tcx

using namespace tcx;

extern "C" int tcx_gn_stats(const double* part, int Bt, int HW, int C, int groups, int nsplit, const float* gamma,
                            const float* beta, float eps, float* scale, float* shift, float* mean, float* rstd,
                            void* stream) {
    TCX_REQUIRE(part && scale && shift && mean && rstd && Bt >= 0 && C > 0 && groups > 0 && C % groups == 0,
                "tcx_gn_stats: bad args");
    if (Bt == 0) return TCX_OK;
    hipLaunchKernelGGL(k_gn_stats, dim3(Bt), dim3(256), gn_fold_lds_bytes(C, groups), (hipStream_t)stream, part,
                       nsplit, HW, C, groups, gamma, beta, eps, scale, shift, mean, rstd);
    return check_launch("tcx_gn_stats");
}

extern "C" size_t tcx_gn_bwd_workspace(int Bt, int HW, int C) {
    const int nsplit = std::max(1, std::min(64, HW / 64));
    return ((size_t)Bt * nsplit * C * 2 + (size_t)Bt * C * 2) * sizeof(double) + (size_t)3 * Bt * C * sizeof(float) + 1024;
}

extern "C" int tcx_gn_bwd_absmax(const float* x, const float* dy, const float* scale, const float* shift,
                                 const float* mean, const float* rstd, const float* gamma, int Bt, int HW, int C,
                                 int groups, int silu, float* dx, float* dgamma, float* dbeta, unsigned* amax, void* ws,
                                 size_t ws_bytes, void* stream) {
    TCX_REQUIRE(x && dy && scale && shift && mean && rstd && dx && ws, "tcx_gn_bwd: null pointer");
    TCX_REQUIRE(C % 4 == 0 && groups > 0 && C % groups == 0 && Bt >= 0 && HW > 0, "tcx_gn_bwd: need C %% 4 == 0");
    TCX_REQUIRE(ws_bytes >= tcx_gn_bwd_workspace(Bt, HW, C), "tcx_gn_bwd: workspace too small");
    TCX_REQUIRE(aligned16(x) && aligned16(dy) && aligned16(dx) && aligned16(scale) && aligned16(shift),
                "tcx_gn_bwd: 16-B alignment");
    if (Bt == 0) return TCX_OK;
    const int nsplit = std::max(1, std::min(64, HW / 64));
    char* base = reinterpret_cast<char*>(align_up(reinterpret_cast<uintptr_t>(ws), 256));
    double* part = reinterpret_cast<double*>(base);
    double* s12 = part + (size_t)Bt * nsplit * C * 2;
    float* k1 = reinterpret_cast<float*>(s12 + (size_t)Bt * C * 2);
    float* k2 = k1 + (size_t)Bt * C;
    float* k3 = k2 + (size_t)Bt * C;
    hipStream_t st = (hipStream_t)stream;
    const int lanes = std::max(1, 256 / (C / 4));
    hipLaunchKernelGGL(k_gn_bwd_partials, dim3(nsplit, Bt), dim3(256), (size_t)lanes * C * 2 * sizeof(double), st, x,
                       dy, scale, shift, HW, C, nsplit, silu, part);
    TCX_TRY(check_launch("tcx_gn_bwd partials"));
    hipLaunchKernelGGL(k_gn_bwd_finalize, dim3(Bt), dim3(256), (size_t)(2 * C + 2 * groups) * sizeof(double), st, part,
                       nsplit, HW, C, groups, mean, rstd, gamma, k1, k2, k3, s12);
    TCX_TRY(check_launch("tcx_gn_bwd finalize"));
    const size_t n4 = (size_t)Bt * HW * C / 4;
    // with amax: at most 2048 workgroups (grid-stride), one atomic each
    hipLaunchKernelGGL(k_gn_bwd_apply, dim3(grid1d(n4, amax ? 2048 : 16384)), dim3(256), 0, st, x, dy, scale, shift, k1, k2, k3, Bt,
                       HW, C, silu, dx, amax);
    TCX_TRY(check_launch("tcx_gn_bwd apply"));
    if (dgamma || dbeta) {
        hipLaunchKernelGGL(k_gn_bwd_affine, dim3(cdiv(C, 8)), dim3(256), 0, st, s12, Bt, C, dgamma, dbeta);
        TCX_TRY(check_launch("tcx_gn_bwd affine"));
    }
    return TCX_OK;
}

extern "C" int tcx_gn_bwd(const float* x, const float* dy, const float* scale, const float* shift, const float* mean,
                          const float* rstd, const float* gamma, int Bt, int HW, int C, int groups, int silu, float* dx,
                          float* dgamma, float* dbeta, void* ws, size_t ws_bytes, void* stream) {
    return tcx_gn_bwd_absmax(x, dy, scale, shift, mean, rstd, gamma, Bt, HW, C, groups, silu, dx, dgamma, dbeta, nullptr,
                             ws, ws_bytes, stream);
}

extern "C" int tcx_upsample2x_bwd(const float* dy, float* dx, int Bt, int H, int W, int C, void* stream) {
    TCX_REQUIRE(dy && dx && C % 4 == 0 && aligned16(dy) && aligned16(dx), "tcx_upsample2x_bwd: bad args");
    const size_t n4 = (size_t)Bt * H * W * C / 4;
    if (n4 == 0) return TCX_OK;
    hipLaunchKernelGGL(k_upsample2x_bwd, dim3(grid1d(n4, 16384)), dim3(256), 0, (hipStream_t)stream, dy, dx, Bt, H, W, C);
    return check_launch("tcx_upsample2x_bwd");
}

static int colsum_nsplit(int Bt, int HW) {
    // ~>= 2048 blocks overall, >= 64 rows per block
    int ns = std::max(1, cdiv(2048, std::max(Bt, 1)));
    ns = std::min(ns, std::max(1, HW / 64));
    return std::min(ns, 4096);
}

extern "C" size_t tcx_colsum_workspace(int Bt, int HW, int C) {
    const int nsplit = colsum_nsplit(Bt, HW);
    return ((size_t)Bt * nsplit * C + (size_t)Bt * C) * sizeof(double) + 512;
}

extern "C" int tcx_colsum(const float* x, int Bt, int HW, int C, float* per_batch, float* total, float beta, void* ws,
                          size_t ws_bytes, void* stream) {
    TCX_REQUIRE(x && ws && Bt >= 0 && HW >= 0 && C > 0, "tcx_colsum: bad args");
    TCX_REQUIRE(ws_bytes >= tcx_colsum_workspace(Bt, HW, C), "tcx_colsum: workspace too small");
    const int nsplit = colsum_nsplit(Bt, HW);
    double* part = reinterpret_cast<double*>(align_up(reinterpret_cast<uintptr_t>(ws), 256));
    double* tot_b = part + (size_t)Bt * nsplit * C;
    hipStream_t st = (hipStream_t)stream;
    if (Bt == 1 && !per_batch && total && HW <= 4096 && C % 4 == 0 && aligned16(x)) {
        hipLaunchKernelGGL(k_colsum_small, dim3(cdiv(C / 4, 32)), dim3(256), 0, st, x, HW, C, total, beta);
        return check_launch("tcx_colsum small");
    }
    if (Bt > 0) {
        const bool vec = C % 4 == 0 && aligned16(x);
        const int ncol = vec ? C / 4 : C;
        const int cpb = std::min(ncol, 256);
        const size_t shm = (size_t)(256 / cpb) * cpb * (vec ? 4 : 1) * sizeof(double);
        if (vec) hipLaunchKernelGGL(k_colsum_part<true>, dim3(nsplit, Bt), dim3(256), shm, st, x, HW, C, nsplit, part);
        else hipLaunchKernelGGL(k_colsum_part<false>, dim3(nsplit, Bt), dim3(256), shm, st, x, HW, C, nsplit, part);
        TCX_TRY(check_launch("tcx_colsum part"));
        const size_t n = (size_t)Bt * C;
        if (nsplit > 256 && n <= 65535)
            hipLaunchKernelGGL(k_colsum_fold_wide, dim3((unsigned)n), dim3(256), 0, st, part, nsplit, C, per_batch, tot_b);
        else
            hipLaunchKernelGGL(k_colsum_fold, dim3((unsigned)std::min<size_t>((n + 7) / 8, 16384)), dim3(256), 0, st,
                               part, Bt, nsplit, C, per_batch, tot_b);
        TCX_TRY(check_launch("tcx_colsum fold"));
    }
    if (total) {
        hipLaunchKernelGGL(k_colsum_total, dim3(cdiv(C, 8)), dim3(256), 0, st, tot_b, Bt, C, total, beta);
        TCX_TRY(check_launch("tcx_colsum total"));
    }
    return TCX_OK;
}

extern "C" int tcx_softmax_rows(const float* S, float* P, long long rows, int n, void* stream) {
    TCX_REQUIRE(S && P && n > 0 && rows >= 0, "tcx_softmax_rows: bad args");
    if (rows == 0) return TCX_OK;
    hipLaunchKernelGGL(k_softmax_rows, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, (hipStream_t)stream, S, P, rows, n);
    return check_launch("tcx_softmax_rows");
}

extern "C" int tcx_softmax_bwd_rows(const float* P, const float* dP, float* dS, long long rows, int n, void* stream) {
    TCX_REQUIRE(P && dP && dS && n > 0 && rows >= 0, "tcx_softmax_bwd_rows: bad args");
    if (rows == 0) return TCX_OK;
    hipLaunchKernelGGL(k_softmax_bwd_rows, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, (hipStream_t)stream, P, dP,
                       dS, rows, n);
    return check_launch("tcx_softmax_bwd_rows");
}

extern "C" int tcx_act_fwd(const float* z, float* y, size_t n, int act, void* stream) {
    TCX_REQUIRE(z && y && act >= 1 && act <= 3, "tcx_act_fwd: bad args");
    if (n == 0) return TCX_OK;
    hipLaunchKernelGGL(k_act_fwd, dim3(grid1d(n)), dim3(256), 0, (hipStream_t)stream, z, y, n, act);
    return check_launch("tcx_act_fwd");
}

extern "C" int tcx_act_bwd(const float* z, const float* dy, float* dz, size_t n, int act, void* stream) {
    TCX_REQUIRE(z && dy && dz && act >= 1 && act <= 3, "tcx_act_bwd: bad args");
    if (n == 0) return TCX_OK;
    hipLaunchKernelGGL(k_act_bwd, dim3(grid1d(n)), dim3(256), 0, (hipStream_t)stream, z, dy, dz, n, act);
    return check_launch("tcx_act_bwd");
}

extern "C" int tcx_mse_loss(const float* a, const float* b, size_t n, float* out, void* ws, size_t ws_bytes,
                            void* stream) {
    TCX_REQUIRE(a && b && out && ws && n > 0, "tcx_mse_loss: bad args");
    const int nb = grid1d(n, 1024);
    TCX_REQUIRE(ws_bytes >= (size_t)nb * sizeof(double) + 256, "tcx_mse_loss: workspace too small");
    double* part = reinterpret_cast<double*>(align_up(reinterpret_cast<uintptr_t>(ws), 256));
    hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL(k_sqdiff_part, dim3(nb), dim3(256), 0, st, a, b, n, part);
    TCX_TRY(check_launch("tcx_mse_loss part"));
    hipLaunchKernelGGL(k_sqdiff_fold, dim3(1), dim3(64), 0, st, part, nb, n, out);
    return check_launch("tcx_mse_loss fold");
}

extern "C" int tcx_mse_bwd(const float* a, const float* b, size_t n, const float* grad_out, float* da, void* stream) {
    TCX_REQUIRE(a && b && grad_out && da, "tcx_mse_bwd: bad args");
    if (n == 0) return TCX_OK;
    hipLaunchKernelGGL(k_mse_bwd, dim3(grid1d(n)), dim3(256), 0, (hipStream_t)stream, a, b, n, grad_out, da);
    return check_launch("tcx_mse_bwd");
}

extern "C" int tcx_embedding_bwd(const int64_t* idx, const float* dout, int B, int rows, int E, float* dW,
                                 void* stream) {
    TCX_REQUIRE(idx && dout && dW && B >= 0 && rows > 0 && E > 0, "tcx_embedding_bwd: bad args");
    const size_t n = (size_t)rows * E;
    hipLaunchKernelGGL(k_embedding_bwd, dim3(grid1d(n)), dim3(256), 0, (hipStream_t)stream, idx, dout, B, rows, E, dW);
    return check_launch("tcx_embedding_bwd");
}

extern "C" int tcx_ln_fwd(const float* x, float* y, int M, int Wd, const float* w, const float* b, const float* gb,
                          int ld_gb, float eps, float* mean, float* rstd, void* stream) {
    TCX_REQUIRE(x && y && w && b && mean && rstd && M >= 0 && Wd > 0, "tcx_ln_fwd: bad args");
    if (M == 0) return TCX_OK;
    hipLaunchKernelGGL(k_ln_fwd, dim3(M), dim3(256), 0, (hipStream_t)stream, x, y, Wd, w, b, gb, ld_gb, eps, mean, rstd);
    return check_launch("tcx_ln_fwd");
}

extern "C" int tcx_ln_bwd(const float* x, const float* dh, int M, int Wd, const float* w, const float* b,
                          const float* gb, int ld_gb, const float* mean, const float* rstd, float* dx, float* dwrow,
                          float* dbrow, float* dgb, void* stream) {
    TCX_REQUIRE(x && dh && w && b && mean && rstd && dx && dwrow && dbrow && (!gb || dgb) && M >= 0 && Wd > 0,
                "tcx_ln_bwd: bad args");
    if (M == 0) return TCX_OK;
    hipLaunchKernelGGL(k_ln_bwd, dim3(M), dim3(256), 0, (hipStream_t)stream, x, dh, Wd, w, b, gb, ld_gb, mean, rstd, dx,
                       dwrow, dbrow, dgb);
    return check_launch("tcx_ln_bwd");
}

extern "C" int tcx_adam(const tcx_adam_tensor* table, int ntensors, long long max_n, float lr, float beta1,
                        float beta2, float eps, float weight_decay, long long step, void* stream) {
    TCX_REQUIRE((table || ntensors == 0) && ntensors >= 0 && step >= 1, "tcx_adam: bad args");
    AdamArgs a{};
    // host scalars in double as torch's Python-side arithmetic, then cast to the tensor dtype
    const double b1 = beta1, b2 = beta2;
    const double bc1 = 1.0 - std::pow(b1, (double)step), bc2 = 1.0 - std::pow(b2, (double)step);
    a.w1 = (float)(1.0 - b1);
    a.b2 = (float)b2;
    a.w2 = (float)(1.0 - b2);
    a.bc2s = (float)std::sqrt(bc2);
    a.eps = eps;
    a.neg_step = (float)(-((double)lr / bc1));
    a.wd = weight_decay;
    const int gx = (int)std::max<long long>(1, std::min<long long>((max_n + 255) / 256, 1024));
    for (int t0 = 0; t0 < ntensors; t0 += kMaxAdamTensors) {
        const int nt = std::min(kMaxAdamTensors, ntensors - t0);
        for (int i = 0; i < nt; ++i) a.t[i] = table[t0 + i];
        hipLaunchKernelGGL(k_adam, dim3(gx, nt), dim3(256), 0, (hipStream_t)stream, a);
        TCX_TRY(check_launch("tcx_adam"));
    }
    return TCX_OK;
}

extern "C" int tcx_ema(const tcx_adam_tensor* table, int ntensors, long long max_n, float decay, void* stream) {
    TCX_REQUIRE((table || ntensors == 0) && ntensors >= 0, "tcx_ema: bad args");
    EmaArgs a{};
    const double d = decay;
    a.d = (float)d;
    a.w = (float)(1.0 - d);
    const int gx = (int)std::max<long long>(1, std::min<long long>((max_n + 255) / 256, 1024));
    for (int t0 = 0; t0 < ntensors; t0 += kMaxAdamTensors) {
        const int nt = std::min(kMaxAdamTensors, ntensors - t0);
        for (int i = 0; i < nt; ++i) a.t[i] = table[t0 + i];
        hipLaunchKernelGGL(k_ema, dim3(gx, nt), dim3(256), 0, (hipStream_t)stream, a);
        TCX_TRY(check_launch("tcx_ema"));
    }
    return TCX_OK;
}

extern "C" int tcx_cond_inputs(const float* t, const int64_t* y_cat, const float* y_cont, int B, int E, int n_types,
                               int ycd, float* te, float* yv, int64_t* yc, void* stream) {
    TCX_REQUIRE(t && y_cat && y_cont && te && yv && yc && B >= 0 && E > 0 && ycd >= 3, "tcx_cond_inputs: bad args");
    if (B == 0) return TCX_OK;
    hipLaunchKernelGGL(k_cond_inputs, dim3(B), dim3(128), 0, (hipStream_t)stream, t, y_cat, y_cont, B, E, n_types, ycd,
                       te, yv, yc);
    return check_launch("tcx_cond_inputs");
}

extern "C" int tcx_prior_temb(const int64_t* t, const float* freqs, int B, int E, float* te, void* stream) {
    TCX_REQUIRE(t && freqs && te && B >= 0 && E > 0, "tcx_prior_temb: bad args");
    if (B == 0) return TCX_OK;
    hipLaunchKernelGGL(k_prior_temb, dim3(B), dim3(64), 0, (hipStream_t)stream, t, freqs, B, E, te);
    return check_launch("tcx_prior_temb");
}

extern "C" int tcx_embedding_fwd(const int64_t* idx, const float* W, int B, int E, float* out, void* stream) {
    TCX_REQUIRE(idx && W && out && B >= 0 && E > 0, "tcx_embedding_fwd: bad args");
    if (B == 0) return TCX_OK;
    hipLaunchKernelGGL(k_embedding_fwd, dim3(grid1d((size_t)B * E)), dim3(256), 0, (hipStream_t)stream, idx, W, B, E, out);
    return check_launch("tcx_embedding_fwd");
}

extern "C" int tcx_copy2d(const float* src, long long ld_src, float* dst, long long ld_dst, int rows, int cols,
                          float beta, void* stream) {
    TCX_REQUIRE(src && dst && rows >= 0 && cols >= 0, "tcx_copy2d: bad args");
    const size_t n = (size_t)rows * cols;
    if (n == 0) return TCX_OK;
    hipLaunchKernelGGL(k_copy2d, dim3(grid1d(n)), dim3(256), 0, (hipStream_t)stream, src, ld_src, dst, ld_dst, rows, cols,
                       beta);
    return check_launch("tcx_copy2d");
}

extern "C" int tcx_transpose_bhc(const float* src, float* dst, int B, int R, int C, void* stream) {
    TCX_REQUIRE(src && dst && B >= 0 && R >= 0 && C >= 0, "tcx_transpose_bhc: bad args");
    const size_t n = (size_t)B * R * C;
    if (n == 0) return TCX_OK;
    hipLaunchKernelGGL(k_transpose_bhc, dim3(grid1d(n)), dim3(256), 0, (hipStream_t)stream, src, dst, B, R, C);
    return check_launch("tcx_transpose_bhc");
}

extern "C" int tcx_first_conv_bias(const float* maps, const float* w, const float* bias, int B, int C0, int nm, int ks,
                                   float* bias_b, void* stream) {
    TCX_REQUIRE(maps && w && bias_b && B >= 0 && C0 > 0 && nm >= 0, "tcx_first_conv_bias: bad args");
    if (B == 0) return TCX_OK;
    hipLaunchKernelGGL(k_first_conv_bias, dim3(cdiv(B * C0, 256)), dim3(256), 0, (hipStream_t)stream, maps, w, bias, B,
                       C0, nm, ks, bias_b);
    return check_launch("tcx_first_conv_bias");
}

extern "C" int tcx_first_conv_bwd(const float* S, const float* maps, const float* w, const float* dwx, int B, int C0,
                                  int nm, int ks, float* dmaps, float* dw, float* db, void* stream) {
    TCX_REQUIRE(S && maps && w && (!dw || dwx) && B >= 0 && C0 > 0, "tcx_first_conv_bwd: bad args");
    hipLaunchKernelGGL(k_first_conv_bwd, dim3(std::max(1, cdiv(std::max(B * nm, C0 * (1 + nm)), 256))), dim3(256), 0,
                       (hipStream_t)stream, S, maps, w, dwx, B, C0, nm, ks, dmaps, dw, db);
    return check_launch("tcx_first_conv_bwd");
}

extern "C" int tcx_qsample_vp(const float* x0, const float* eps, const float* u, float t_power, float beta_min,
                              float half_dbeta, int B, int HW, float* t_out, float* x_t, void* stream) {
    TCX_REQUIRE(x0 && eps && u && t_out && x_t && B >= 0 && HW > 0, "tcx_qsample_vp: bad args");
    const size_t n = (size_t)B * HW;
    if (n == 0) return TCX_OK;
    hipLaunchKernelGGL(k_qsample_vp, dim3(grid1d(n)), dim3(256), 0, (hipStream_t)stream, x0, eps, u, t_power, beta_min,
                       half_dbeta, B, HW, t_out, x_t);
    return check_launch("tcx_qsample_vp");
}

extern "C" int tcx_cond_drop(const int64_t* y_cat, const float* y_cont, const float* r, float p, int B, int ycd,
                             int n_types, int64_t* out_cat, float* out_cont, void* stream) {
    TCX_REQUIRE(y_cat && y_cont && out_cat && out_cont && B >= 0 && ycd > 0, "tcx_cond_drop: bad args");
    if (B == 0) return TCX_OK;
    hipLaunchKernelGGL(k_cond_drop, dim3(cdiv(B, 256)), dim3(256), 0, (hipStream_t)stream, y_cat, y_cont, r, p, B, ycd,
                       n_types, out_cat, out_cont);
    return check_launch("tcx_cond_drop");
}

extern "C" int tcx_prior_qsample(const float* z0, const float* eps, const float* u, const float* sqrt_ab,
                                 const float* sqrt_1mab, int T, int B, int Z, int64_t* t_out, float* z_t, void* stream) {
    TCX_REQUIRE(z0 && eps && u && sqrt_ab && sqrt_1mab && t_out && z_t && T > 0 && B >= 0 && Z > 0,
                "tcx_prior_qsample: bad args");
    const size_t n = (size_t)B * Z;
    if (n == 0) return TCX_OK;
    hipLaunchKernelGGL(k_prior_qsample, dim3(grid1d(n)), dim3(256), 0, (hipStream_t)stream, z0, eps, u, sqrt_ab,
                       sqrt_1mab, T, B, Z, t_out, z_t);
    return check_launch("tcx_prior_qsample");
}

extern "C" int tcx_reparam(const float* mu, const float* lv, const float* eps, size_t n, float* z, void* stream) {
    TCX_REQUIRE(mu && lv && eps && z, "tcx_reparam: bad args");
    if (n == 0) return TCX_OK;
    hipLaunchKernelGGL(k_reparam, dim3(grid1d(n)), dim3(256), 0, (hipStream_t)stream, mu, lv, eps, n, z);
    return check_launch("tcx_reparam");
}

extern "C" int tcx_reparam_bwd(const float* lv, const float* eps, const float* dz, size_t n, float* dmu, float* dlv,
                               float beta, void* stream) {
    TCX_REQUIRE(lv && eps && dz && dmu && dlv, "tcx_reparam_bwd: bad args");
    if (n == 0) return TCX_OK;
    hipLaunchKernelGGL(k_reparam_bwd, dim3(grid1d(n)), dim3(256), 0, (hipStream_t)stream, lv, eps, dz, n, dmu, dlv, beta);
    return check_launch("tcx_reparam_bwd");
}

extern "C" int tcx_vae_kl(const float* mu, const float* lv, int B, int Z, float free_bits, float* out, void* stream) {
    TCX_REQUIRE(mu && lv && out && B > 0 && Z > 0, "tcx_vae_kl: bad args");
    hipLaunchKernelGGL(k_vae_kl, dim3(1), dim3(256), 0, (hipStream_t)stream, mu, lv, B, Z, free_bits, out);
    return check_launch("tcx_vae_kl");
}

extern "C" int tcx_vae_kl_bwd(const float* mu, const float* lv, int B, int Z, float free_bits, const float* grad_out,
                              float* dmu, float* dlv, float beta, void* stream) {
    TCX_REQUIRE(mu && lv && grad_out && dmu && dlv && B > 0 && Z > 0, "tcx_vae_kl_bwd: bad args");
    hipLaunchKernelGGL(k_vae_kl_bwd, dim3(cdiv(B * Z, 256)), dim3(256), 0, (hipStream_t)stream, mu, lv, B, Z, free_bits,
                       grad_out, dmu, dlv, beta);
    return check_launch("tcx_vae_kl_bwd");
}

extern "C" int tcx_vae_yvec(const int64_t* y_cat, const float* y_cont, const float* keep_u, float cond_drop, int B,
                            int n_types, int ycd, float* out, void* stream) {
    TCX_REQUIRE(y_cat && y_cont && out && B >= 0 && n_types > 0 && ycd >= 0, "tcx_vae_yvec: bad args");
    if (B == 0) return TCX_OK;
    hipLaunchKernelGGL(k_vae_yvec, dim3(cdiv(B * (n_types + ycd), 256)), dim3(256), 0, (hipStream_t)stream, y_cat,
                       y_cont, keep_u, cond_drop, B, n_types, ycd, out);
    return check_launch("tcx_vae_yvec");
}

extern "C" int tcx_ddim_step(float* z, const float* eps, size_t n, float abar_t, float abar_prev, int last,
                             void* stream) {
    TCX_REQUIRE(z && eps, "tcx_ddim_step: bad args");
    if (n == 0) return TCX_OK;
    hipLaunchKernelGGL(k_ddim_step, dim3(grid1d(n)), dim3(256), 0, (hipStream_t)stream, z, eps, n, abar_t, abar_prev,
                       last);
    return check_launch("tcx_ddim_step");
}

extern "C" int tcx_q_sample(const float* z0, const int64_t* t, const float* eps, const float* sqrt_ab,
                            const float* sqrt_1mab, int B, int Z, float* out, void* stream) {
    TCX_REQUIRE(z0 && t && eps && sqrt_ab && sqrt_1mab && out && B >= 0 && Z > 0, "tcx_q_sample: bad args");
    const size_t n = (size_t)B * Z;
    if (n == 0) return TCX_OK;
    hipLaunchKernelGGL(k_q_sample_t, dim3(grid1d(n)), dim3(256), 0, (hipStream_t)stream, z0, t, eps, sqrt_ab, sqrt_1mab,
                       B, Z, out);
    return check_launch("tcx_q_sample");
}

extern "C" int tcx_u8_gather(const uint8_t* x_u8, const int64_t* idx, int B, int npix, float* out, void* stream) {
    TCX_REQUIRE(x_u8 && idx && out && B >= 0 && npix > 0, "tcx_u8_gather: bad args");
    const size_t n = (size_t)B * npix;
    if (n == 0) return TCX_OK;
    hipLaunchKernelGGL(k_u8_gather, dim3(grid1d(n)), dim3(256), 0, (hipStream_t)stream, x_u8, idx, B, npix, out);
    return check_launch("tcx_u8_gather");
}
