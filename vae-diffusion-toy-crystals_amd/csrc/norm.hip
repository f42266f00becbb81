// GroupNorm (+SiLU), LayerNorm/FiLM, bilinear x2 upsample — HBM-bound kernels, NHWC fp32.
//
// GroupNorm(8, C, eps=1e-5) of CondUNetTiny (/root/reference/src/toycrystals/models/
// sde_score_model.py:103,106,130 via _gn_groups :89-94) is split in two phases so that the
// statistics can come either from tcx_gn_partials or from the producing conv's epilogue
// (tcx_conv2d gn_stats): partial {sum, sumsq} per (batch, split, channel) in fp64, then an
// apply pass that folds mean/rstd/gamma/beta into one per-channel scale/shift and fuses SiLU.
#include "common.hpp"

namespace tcx {
namespace {

// part[b][split][c][2]; grid (nsplit, Bt); block 256.  Threads: c4 = tid % TPR (channel quad),
// row = tid / TPR (pixel lane); each thread streams pixels row, row + RP, ... of its split.
__global__ __launch_bounds__(256) void k_gn_partials(const float* __restrict__ x, int HW, int C, int nsplit,
                                                     double* __restrict__ part) {
    extern __shared__ __attribute__((aligned(16))) double sred[];  // [RP][C][2]
    const int b = blockIdx.y, split = blockIdx.x;
    const int TPR = C >> 2;
    const int RP = 256 / TPR;
    const int tid = threadIdx.x;
    const int c4 = tid % TPR, row = tid / TPR;
    const int per = (HW + nsplit - 1) / nsplit;
    const int p0 = split * per, p1 = min(HW, p0 + per);
    double s[4] = {0, 0, 0, 0}, ss[4] = {0, 0, 0, 0};
    if (row < RP) {
        const float* base = x + (size_t)b * HW * C + c4 * 4;
        int p = p0 + row;
        for (; p + 3 * RP < p1; p += 4 * RP) {  // 4 loads in flight per thread
            float4 v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const float4*>(base + (size_t)(p + u * RP) * C);
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                s[0] += v[u].x; s[1] += v[u].y; s[2] += v[u].z; s[3] += v[u].w;
                ss[0] += (double)v[u].x * v[u].x; ss[1] += (double)v[u].y * v[u].y;
                ss[2] += (double)v[u].z * v[u].z; ss[3] += (double)v[u].w * v[u].w;
            }
        }
        for (; p < p1; p += RP) {
            const float4 v = *reinterpret_cast<const float4*>(base + (size_t)p * C);
            s[0] += v.x; s[1] += v.y; s[2] += v.z; s[3] += v.w;
            ss[0] += (double)v.x * v.x; ss[1] += (double)v.y * v.y;
            ss[2] += (double)v.z * v.z; ss[3] += (double)v.w * v.w;
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            sred[(row * C + c4 * 4 + e) * 2 + 0] = s[e];
            sred[(row * C + c4 * 4 + e) * 2 + 1] = ss[e];
        }
    }
    __syncthreads();
    for (int c = tid; c < C; c += 256) {
        double a = 0, q = 0;
        for (int r = 0; r < RP; ++r) {
            a += sred[(r * C + c) * 2 + 0];
            q += sred[(r * C + c) * 2 + 1];
        }
        double* dst = part + (((size_t)b * nsplit + split) * C + c) * 2;
        dst[0] = a;
        dst[1] = q;
    }
}

// Per-channel scale/shift of batch b into LDS from the partials.
__device__ void gn_scale_shift(const double* __restrict__ part, int b, int nsplit, int C, int groups, int HW,
                               const float* __restrict__ gamma, const float* __restrict__ beta, float eps,
                               float* sc, float* sh, double* gstat) {
    const int cpg = C / groups;
    const int tid = threadIdx.x;
    for (int g = tid; g < groups; g += blockDim.x) {
        double a = 0, q = 0;
        for (int sp = 0; sp < nsplit; ++sp) {
            const double* src = part + (((size_t)b * nsplit + sp) * C + g * cpg) * 2;
            for (int c = 0; c < cpg; ++c) {
                a += src[2 * c];
                q += src[2 * c + 1];
            }
        }
        const double n = (double)HW * cpg;
        const double mean = a / n;
        double var = q / n - mean * mean;
        var = var < 0 ? 0 : var;
        gstat[2 * g] = mean;
        gstat[2 * g + 1] = 1.0 / sqrt(var + (double)eps);
    }
    __syncthreads();
    for (int c = tid; c < C; c += blockDim.x) {
        const int g = c / cpg;
        const float rstd = (float)gstat[2 * g + 1];
        const float mean = (float)gstat[2 * g];
        const float gm = gamma ? gamma[c] : 1.f;
        const float bt = beta ? beta[c] : 0.f;
        const float scl = rstd * gm;
        sc[c] = scl;
        sh[c] = bt - mean * scl;
    }
    __syncthreads();
}

// grid (chunks, Bt); each block normalises pixels [chunk*ppb, ...) of image b.
__global__ __launch_bounds__(256) void k_gn_apply(const float* __restrict__ x, float* __restrict__ y, int HW, int C,
                                                  int groups, const double* __restrict__ part, int nsplit,
                                                  const float* __restrict__ gamma, const float* __restrict__ beta,
                                                  float eps, int silu, int ppb) {
    extern __shared__ __attribute__((aligned(16))) float lsm[];  // sc[C], sh[C], gstat (double) [2*groups]
    float* sc = lsm;
    float* sh = lsm + C;
    double* gstat = reinterpret_cast<double*>(lsm + 2 * ((C + 1) & ~1));
    const int b = blockIdx.y;
    gn_scale_shift(part, b, nsplit, C, groups, HW, gamma, beta, eps, sc, sh, gstat);
    const int p0 = blockIdx.x * ppb;
    const int p1 = min(HW, p0 + ppb);
    const size_t base = ((size_t)b * HW + p0) * C;
    const int n4 = (p1 - p0) * C / 4;
    const int C4 = C / 4;
    for (int i = threadIdx.x; i < n4; i += 256) {
        const int c = (i % C4) * 4;
        float4 v = *reinterpret_cast<const float4*>(x + base + (size_t)i * 4);
        v.x = fmaf(v.x, sc[c + 0], sh[c + 0]);
        v.y = fmaf(v.y, sc[c + 1], sh[c + 1]);
        v.z = fmaf(v.z, sc[c + 2], sh[c + 2]);
        v.w = fmaf(v.w, sc[c + 3], sh[c + 3]);
        if (silu) {
            v.x = silu_f(v.x); v.y = silu_f(v.y); v.z = silu_f(v.z); v.w = silu_f(v.w);
        }
        *reinterpret_cast<float4*>(y + base + (size_t)i * 4) = v;
    }
}

__global__ __launch_bounds__(256) void k_upsample2x(const float* __restrict__ x, float* __restrict__ y, int Bt, int H,
                                                    int W, int C) {
    const int C4 = C / 4;
    const size_t n = (size_t)Bt * 4 * H * W * C4;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const int c4 = (int)(i % C4);
        size_t r = i / C4;
        const int ox = (int)(r % (2 * W));
        r /= (2 * W);
        const int oy = (int)(r % (2 * H));
        const int b = (int)(r / (2 * H));
        float sy = 0.5f * ((float)oy + 0.5f) - 0.5f;
        sy = sy < 0.f ? 0.f : sy;
        float sx = 0.5f * ((float)ox + 0.5f) - 0.5f;
        sx = sx < 0.f ? 0.f : sx;
        const int y0 = (int)sy, x0 = (int)sx;
        const int y1 = y0 + (y0 < H - 1 ? 1 : 0), x1 = x0 + (x0 < W - 1 ? 1 : 0);
        const float ly1 = sy - (float)y0, ly0 = 1.f - ly1;
        const float lx1 = sx - (float)x0, lx0 = 1.f - lx1;
        const float* src = x + (size_t)b * H * W * C + c4 * 4;
        const float4 a = *reinterpret_cast<const float4*>(src + (size_t)(y0 * W + x0) * C);
        const float4 bq = *reinterpret_cast<const float4*>(src + (size_t)(y0 * W + x1) * C);
        const float4 c = *reinterpret_cast<const float4*>(src + (size_t)(y1 * W + x0) * C);
        const float4 d = *reinterpret_cast<const float4*>(src + (size_t)(y1 * W + x1) * C);
        float4 o;
        o.x = ly0 * (lx0 * a.x + lx1 * bq.x) + ly1 * (lx0 * c.x + lx1 * d.x);
        o.y = ly0 * (lx0 * a.y + lx1 * bq.y) + ly1 * (lx0 * c.y + lx1 * d.y);
        o.z = ly0 * (lx0 * a.z + lx1 * bq.z) + ly1 * (lx0 * c.z + lx1 * d.z);
        o.w = ly0 * (lx0 * a.w + lx1 * bq.w) + ly1 * (lx0 * c.w + lx1 * d.w);
        *reinterpret_cast<float4*>(y + i * 4) = o;
    }
}

// LayerNorm over rows of width Wd (+ optional FiLM h*(1+gamma)+beta), one wave per row.
__global__ __launch_bounds__(256) void k_layernorm_film(const float* __restrict__ x, float* __restrict__ y, int M,
                                                        int Wd, const float* __restrict__ lw,
                                                        const float* __restrict__ lb, const float* __restrict__ gb,
                                                        int ld_gb, float eps) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (row >= M) return;
    const float* xr = x + (size_t)row * Wd;
    double s = 0, q = 0;
    for (int i = lane; i < Wd; i += 64) {
        const double v = xr[i];
        s += v;
        q += v * v;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        s += __shfl_xor(s, o);
        q += __shfl_xor(q, o);
    }
    const double mean = s / Wd;
    double var = q / Wd - mean * mean;
    var = var < 0 ? 0 : var;
    const float rstd = (float)(1.0 / sqrt(var + (double)eps));
    const float mf = (float)mean;
    float* yr = y + (size_t)row * Wd;
    for (int i = lane; i < Wd; i += 64) {
        float h = (xr[i] - mf) * rstd * lw[i] + lb[i];
        if (gb) {
            const float g = gb[(size_t)row * ld_gb + i];
            const float be = gb[(size_t)row * ld_gb + Wd + i];
            h = h * (1.f + g) + be;
        }
        yr[i] = h;
    }
}

}  // namespace
}  // namespace tcx

using namespace tcx;

extern "C" int tcx_gn_partials(const float* x, int Bt, int HW, int C, int nsplit, double* part, void* stream) {
    TCX_REQUIRE(x && part, "tcx_gn_partials: null pointer");
    TCX_REQUIRE(C % 4 == 0 && C / 4 <= 256 && nsplit >= 1 && HW > 0, "tcx_gn_partials: need C%%4==0, C<=1024");
    TCX_REQUIRE(aligned16(x), "tcx_gn_partials: x must be 16-B aligned");
    if (Bt == 0) return TCX_OK;
    const int RP = 256 / (C / 4);
    const size_t shm = (size_t)RP * C * 2 * sizeof(double);
    hipLaunchKernelGGL(k_gn_partials, dim3(nsplit, Bt), dim3(256), shm, (hipStream_t)stream, x, HW, C, nsplit, part);
    return check_launch("tcx_gn_partials");
}

extern "C" int tcx_gn_apply(const float* x, float* y, int Bt, int HW, int C, int groups, const double* part,
                            int nsplit, const float* gamma, const float* beta, float eps, int silu, void* stream) {
    TCX_REQUIRE(x && y && part, "tcx_gn_apply: null pointer");
    TCX_REQUIRE(C % 4 == 0 && groups > 0 && C % groups == 0, "tcx_gn_apply: bad C/groups");
    TCX_REQUIRE(aligned16(x) && aligned16(y), "tcx_gn_apply: x/y must be 16-B aligned");
    if (Bt == 0) return TCX_OK;
    const int ppb = std::max(1, 16384 / C);  // ~64 KB of activations per block
    const int chunks = cdiv(HW, ppb);
    const size_t shm = (size_t)2 * ((C + 1) & ~1) * sizeof(float) + (size_t)2 * groups * sizeof(double);
    hipLaunchKernelGGL(k_gn_apply, dim3(chunks, Bt), dim3(256), shm, (hipStream_t)stream, x, y, HW, C, groups, part,
                       nsplit, gamma, beta, eps, silu, ppb);
    return check_launch("tcx_gn_apply");
}

extern "C" int tcx_upsample2x(const float* x, float* y, int Bt, int H, int W, int C, void* stream) {
    TCX_REQUIRE(x && y && C % 4 == 0 && aligned16(x) && aligned16(y), "tcx_upsample2x: bad args");
    const size_t n = (size_t)Bt * 4 * H * W * (C / 4);
    if (n == 0) return TCX_OK;
    const int blocks = (int)std::min<size_t>((n + 255) / 256, 8192);
    hipLaunchKernelGGL(k_upsample2x, dim3(blocks), dim3(256), 0, (hipStream_t)stream, x, y, Bt, H, W, C);
    return check_launch("tcx_upsample2x");
}

extern "C" int tcx_layernorm_film(const float* x, float* y, int M, int Wd, const float* ln_w, const float* ln_b,
                                  const float* gb, int ld_gb, float eps, void* stream) {
    TCX_REQUIRE(x && y && ln_w && ln_b && M >= 0 && Wd > 0, "tcx_layernorm_film: bad args");
    if (M == 0) return TCX_OK;
    hipLaunchKernelGGL(k_layernorm_film, dim3(cdiv(M, 4)), dim3(256), 0, (hipStream_t)stream, x, y, M, Wd, ln_w, ln_b,
                       gb, ld_gb, eps);
    return check_launch("tcx_layernorm_film");
}
