// Implicit-GEMM 2-D convolution on fp32 MFMA (v_mfma_f32_32x32x2_f32), NHWC, gfx950.
//
// GEMM view: out[m = pixel][co] = sum_k A[m][k] * B[k][co],  k = (dy*ks + dx)*Cin + ci,
//   A[m][k] = x[b, wrap(oy*s - pad + dy), wrap(ox*s - pad + dx), ci]   (im2col, never stored)
//   B[k][co] = packed weight wpk[co][k]   (tcx_pack_conv_weight)
// Replaces nn.Conv2d(..., padding_mode="circular") of CondUNetTiny
// (/root/reference/src/toycrystals/models/sde_score_model.py:102,105,133-134,208,210,218,222,225)
// and the zero-padded Conv2d / ConvTranspose2d of CondVAE (models/vae.py:19-26,35-42).
//
// Tile: BM = 128 pixels x BN = 32*NT output channels, BK = 32; 4 waves, each owning a
// 32-pixel x BN slab (NT 32x32 accumulators = 16*NT AGPR/VGPR).  K is consumed in 32-deep
// chunks staged through LDS (register-staged double buffer: the next chunk's global loads are
// in flight while the current chunk's MFMAs run).  Inside a chunk the K order is permuted so
// that lane half h owns k = 16h + s (s = 0..15): each lane reads 4 consecutive k with one
// ds_read_b128, and A/B rows padded to 36 floats keep those reads bank-conflict free
// (row stride 144 B -> 9r mod 16 distinct in every 16-lane group).
// Fusions: channel concat (two sources), CFG batch aliasing (bmod), bilinear x2 upsample on
// the A load, bias / per-batch bias / residual / activation epilogue, and GroupNorm partial
// statistics of the output (fp64) for the following GroupNorm.
#include "common.hpp"

namespace tcx {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int BM = 128;
constexpr int BK = 32;
constexpr int LDA = 36;  // padded LDS row (floats)

struct ConvParams {
    const float* x1;
    const float* x2;
    int C1, C2, Cin;
    int bmod, H, W;    // source image dims (pre-upsample)
    int Hi, Wi;        // im2col input dims (2H,2W when upsampling)
    int Ho, Wo, HoWo, M;
    const float* w;
    const float* bias;
    const float* bias_b;
    const float* resid;
    float* y;
    int Cout, kpad, nchunks;
    int ks, stride, pad_y, pad_x, circular;
    // output placement (sub-pixel phases of a transposed conv): row = oy*osy + ooy
    int Hy, Wy, osy, ooy, osx, oox;
    int act;       // 0 none, 1 relu, 2 sigmoid, 3 silu
    double* gn;    // [Bt][nsplit][Cout][2] or null
    int nsplit;
    int n_nblk;
};

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

__device__ __forceinline__ float4 f4_fma(float s, float4 a, float4 acc) {
    return make_float4(fmaf(s, a.x, acc.x), fmaf(s, a.y, acc.y), fmaf(s, a.z, acc.z), fmaf(s, a.w, acc.w));
}

// Bilinear x2 (align_corners=False) tap: mirrors ATen's upsample_bilinear2d CPU kernel:
// src = 0.5*(d+0.5)-0.5 clamped at 0, i1 = i0 + (i0 < n-1), l1 = src - i0, l0 = 1 - l1,
// out = l0y*(l0x*a00 + l1x*a01) + l1y*(l0x*a10 + l1x*a11).
__device__ __forceinline__ void bilin_axis(int d, int n, int& i0, int& i1, float& l0, float& l1) {
    float s = 0.5f * ((float)d + 0.5f) - 0.5f;
    s = s < 0.f ? 0.f : s;
    i0 = (int)s;
    i1 = i0 + (i0 < n - 1 ? 1 : 0);
    l1 = s - (float)i0;
    l0 = 1.f - l1;
}

template <int NT, int MODE>  // MODE 0: float4 loads (Cin%4==0); 1: scalar (any Cin); 2: upsample
__global__ __launch_bounds__(256, 2) void k_conv(ConvParams p) {
    constexpr int BN = 32 * NT;
    __shared__ __attribute__((aligned(16))) float As[2][BM * LDA];
    __shared__ __attribute__((aligned(16))) float Bs[2][BN * LDA];

    const int nwg = gridDim.x;
    const int tile = xcd_remap(blockIdx.x, nwg);
    const int mblk = tile / p.n_nblk;
    const int nblk = tile - mblk * p.n_nblk;
    const int m0 = mblk * BM;
    const int n0 = nblk * BN;

    const int tid = threadIdx.x;
    const int k4 = tid & 7;
    const int prow = tid >> 3;  // 0..31

    // per-thread pixel decode (4 pixel rows of the A tile)
    int pbase[4], piy[4], pix[4];
    bool pv[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int m = m0 + prow + 32 * i;
        pv[i] = m < p.M;
        const int mm = pv[i] ? m : 0;
        const int b = mm / p.HoWo;
        const int r = mm - b * p.HoWo;
        const int oy = r / p.Wo;
        const int ox = r - oy * p.Wo;
        const int bs = p.bmod > 0 ? b % p.bmod : b;
        pbase[i] = bs * p.H * p.W;
        piy[i] = oy * p.stride - p.pad_y;
        pix[i] = ox * p.stride - p.pad_x;
    }

    float4 ra[4];
    float4 rb[NT];

    auto load_chunk = [&](int c) {
        // ---- A (im2col gather)
        if constexpr (MODE == 1) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                float v[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int k = c * BK + k4 * 4 + e;
                    const int tap = k / p.Cin;
                    const int ci = k - tap * p.Cin;
                    const int dy = tap / p.ks, dx = tap - (tap / p.ks) * p.ks;
                    int yy = piy[i] + dy, xx = pix[i] + dx;
                    bool ok = pv[i] && tap < p.ks * p.ks;
                    if (p.circular) {
                        yy = wrap_idx(yy, p.Hi);
                        xx = wrap_idx(xx, p.Wi);
                    } else {
                        ok = ok && yy >= 0 && yy < p.Hi && xx >= 0 && xx < p.Wi;
                    }
                    v[e] = ok ? p.x1[(size_t)(pbase[i] + yy * p.W + xx) * p.C1 + ci] : 0.f;
                }
                ra[i] = make_float4(v[0], v[1], v[2], v[3]);
            }
        } else {
            const int k = c * BK + k4 * 4;
            const int tap = k / p.Cin;
            const int ci = k - tap * p.Cin;
            const bool kval = tap < p.ks * p.ks;
            const int dy = tap / p.ks, dx = tap - (tap / p.ks) * p.ks;
            const float* src;
            int cs, cc;
            if (ci < p.C1) {
                src = p.x1; cs = p.C1; cc = ci;
            } else {
                src = p.x2; cs = p.C2; cc = ci - p.C1;
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                int yy = piy[i] + dy, xx = pix[i] + dx;
                bool ok = pv[i] && kval;
                if (p.circular) {
                    yy = wrap_idx(yy, p.Hi);
                    xx = wrap_idx(xx, p.Wi);
                } else {
                    ok = ok && yy >= 0 && yy < p.Hi && xx >= 0 && xx < p.Wi;
                }
                if constexpr (MODE == 0) {
                    ra[i] = ok ? ld4(src + (size_t)(pbase[i] + yy * p.W + xx) * cs + cc)
                               : make_float4(0.f, 0.f, 0.f, 0.f);
                } else {  // MODE 2: read through the bilinear x2 upsample of a HxW source
                    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
                    if (ok) {
                        int y0, y1, x0, x1;
                        float ly0, ly1, lx0, lx1;
                        bilin_axis(yy, p.H, y0, y1, ly0, ly1);
                        bilin_axis(xx, p.W, x0, x1, lx0, lx1);
                        const float* b0 = src + (size_t)pbase[i] * cs + cc;
                        const float4 a00 = ld4(b0 + (size_t)(y0 * p.W + x0) * cs);
                        const float4 a01 = ld4(b0 + (size_t)(y0 * p.W + x1) * cs);
                        const float4 a10 = ld4(b0 + (size_t)(y1 * p.W + x0) * cs);
                        const float4 a11 = ld4(b0 + (size_t)(y1 * p.W + x1) * cs);
                        float4 r0 = make_float4(lx0 * a00.x, lx0 * a00.y, lx0 * a00.z, lx0 * a00.w);
                        r0 = f4_fma(lx1, a01, r0);
                        float4 r1 = make_float4(lx0 * a10.x, lx0 * a10.y, lx0 * a10.z, lx0 * a10.w);
                        r1 = f4_fma(lx1, a11, r1);
                        acc = make_float4(ly0 * r0.x, ly0 * r0.y, ly0 * r0.z, ly0 * r0.w);
                        acc = f4_fma(ly1, r1, acc);
                    }
                    ra[i] = acc;
                }
            }
        }
        // ---- B (packed weights, zero padded to kpad x cout_pad)
#pragma unroll
        for (int j = 0; j < NT; ++j) {
            const int co = n0 + prow + 32 * j;
            rb[j] = ld4(p.w + (size_t)co * p.kpad + c * BK + k4 * 4);
        }
    };

    auto store_chunk = [&](int buf) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
            *reinterpret_cast<float4*>(&As[buf][(prow + 32 * i) * LDA + k4 * 4]) = ra[i];
#pragma unroll
        for (int j = 0; j < NT; ++j)
            *reinterpret_cast<float4*>(&Bs[buf][(prow + 32 * j) * LDA + k4 * 4]) = rb[j];
    };

    f32x16 acc[NT];
#pragma unroll
    for (int n = 0; n < NT; ++n) acc[n] = (f32x16){};

    const int lane = tid & 63;
    const int wv = tid >> 6;
    const int li = lane & 31;
    const int lh = lane >> 5;

    load_chunk(0);
    store_chunk(0);
    __syncthreads();

    for (int c = 0; c < p.nchunks; ++c) {
        const int cur = c & 1;
        const bool more = c + 1 < p.nchunks;
        if (more) load_chunk(c + 1);
        const float* Ab = &As[cur][(wv * 32 + li) * LDA + lh * 16];
        const float* Bb = &Bs[cur][li * LDA + lh * 16];
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
            const float4 a = ld4(Ab + s4 * 4);
            float4 b[NT];
#pragma unroll
            for (int n = 0; n < NT; ++n) b[n] = ld4(Bb + n * 32 * LDA + s4 * 4);
#pragma unroll
            for (int n = 0; n < NT; ++n) acc[n] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, b[n].x, acc[n], 0, 0, 0);
#pragma unroll
            for (int n = 0; n < NT; ++n) acc[n] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, b[n].y, acc[n], 0, 0, 0);
#pragma unroll
            for (int n = 0; n < NT; ++n) acc[n] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, b[n].z, acc[n], 0, 0, 0);
#pragma unroll
            for (int n = 0; n < NT; ++n) acc[n] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, b[n].w, acc[n], 0, 0, 0);
        }
        if (more) store_chunk(cur ^ 1);
        __syncthreads();
    }

    // ---- epilogue: C/D map of 32x32 f32 MFMA: col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
    const bool gn = p.gn != nullptr;
    double* red = reinterpret_cast<double*>(&As[0][0]);  // [4 waves][BN][2] (LDS free after the loop)
#pragma unroll
    for (int n = 0; n < NT; ++n) {
        const int co = n0 + n * 32 + li;
        const bool cv = co < p.Cout;
        const float bco = (cv && p.bias) ? p.bias[co] : 0.f;
        double s = 0.0, ss = 0.0;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int row = (r & 3) + 8 * (r >> 2) + 4 * lh;
            const int m = m0 + wv * 32 + row;
            if (m < p.M && cv) {
                const int b = m / p.HoWo;
                float v = acc[n][r] + bco;
                if (p.bias_b) v += p.bias_b[(size_t)b * p.Cout + co];
                size_t oidx;
                if (p.osy == 1 && p.osx == 1) {
                    oidx = (size_t)m * p.Cout + co;
                } else {
                    const int rr = m - b * p.HoWo;
                    const int oy = rr / p.Wo, ox = rr - (rr / p.Wo) * p.Wo;
                    oidx = ((size_t)b * p.Hy * p.Wy + (size_t)(oy * p.osy + p.ooy) * p.Wy + (ox * p.osx + p.oox)) * p.Cout + co;
                }
                if (p.resid) v += p.resid[oidx];
                if (p.act == 1) v = fmaxf(v, 0.f);
                else if (p.act == 2) v = 1.f / (1.f + expf(-v));
                else if (p.act == 3) v = silu_f(v);
                p.y[oidx] = v;
                s += (double)v;
                ss += (double)v * (double)v;
            }
        }
        if (gn) {
            s += __shfl_xor(s, 32);
            ss += __shfl_xor(ss, 32);
            if (lh == 0) {
                red[(wv * BN + n * 32 + li) * 2 + 0] = s;
                red[(wv * BN + n * 32 + li) * 2 + 1] = ss;
            }
        }
    }
    if (gn) {
        __syncthreads();
        if (tid < BN) {
            const int co = n0 + tid;
            if (co < p.Cout) {
                double s = 0.0, ss = 0.0;
#pragma unroll
                for (int w = 0; w < 4; ++w) {
                    s += red[(w * BN + tid) * 2 + 0];
                    ss += red[(w * BN + tid) * 2 + 1];
                }
                const int b = m0 / p.HoWo;
                const int split = (m0 - b * p.HoWo) / BM;
                double* dst = p.gn + (((size_t)b * p.nsplit + split) * p.Cout + co) * 2;
                dst[0] = s;
                dst[1] = ss;
            }
        }
    }
}

template <int NT>
int launch_nt(const ConvParams& p, int mode, hipStream_t st) {
    const int nm = cdiv(p.M, BM);
    const dim3 grid(nm * p.n_nblk), block(256);
    if (mode == 0) hipLaunchKernelGGL((k_conv<NT, 0>), grid, block, 0, st, p);
    else if (mode == 1) hipLaunchKernelGGL((k_conv<NT, 1>), grid, block, 0, st, p);
    else hipLaunchKernelGGL((k_conv<NT, 2>), grid, block, 0, st, p);
    return check_launch("tcx_conv2d");
}

int launch_conv(ConvParams& p, int cout_pad, int mode, hipStream_t st) {
    // BN choice: 96 when it tiles Cout exactly (96, 192, 576 ...), else 64 / 32.
    int nt = (cout_pad % 96 == 0) ? 3 : (cout_pad % 64 == 0 ? 2 : 1);
    p.n_nblk = cout_pad / (32 * nt);
    if (p.M == 0) return TCX_OK;
    prof_begin(st);
    int rc;
    if (nt == 3) rc = launch_nt<3>(p, mode, st);
    else if (nt == 2) rc = launch_nt<2>(p, mode, st);
    else rc = launch_nt<1>(p, mode, st);
    // algorithmic work of this launch: 2 * pixels * Cout * ks^2 * Cin (no padding counted)
    prof_end(st, 2.0 * (double)p.M * p.Cout * p.ks * p.ks * p.Cin);
    return rc;
}

__global__ void k_pack_conv(const float* __restrict__ w, float* __restrict__ wpk, int Cout, int Cin, int ks,
                            int cout_pad, int kpad) {
    const size_t n = (size_t)cout_pad * kpad;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const int co = (int)(i / kpad);
        const int k = (int)(i - (size_t)co * kpad);
        const int tap = k / Cin, ci = k - (k / Cin) * Cin;
        float v = 0.f;
        if (co < Cout && tap < ks * ks) {
            const int dy = tap / ks, dx = tap - (tap / ks) * ks;
            v = w[(((size_t)co * Cin + ci) * ks + dy) * ks + dx];
        }
        wpk[i] = v;
    }
}

// ConvTranspose2d(k=4, s=2, p=1) as 4 sub-pixel 2x2 convs.  Output row oy = 2a + ry reads
// input rows a - 1 + dy (ry = 0: dy 0 -> ky 3, dy 1 -> ky 1) and a + dy (ry = 1: dy 0 -> ky 2,
// dy 1 -> ky 0); the same along x.  w [Cin][Cout][4][4] -> wpk[phase][cout_pad][kpad].
__global__ void k_pack_convT(const float* __restrict__ w, float* __restrict__ wpk, int Cin, int Cout,
                             int cout_pad, int kpad) {
    const size_t per = (size_t)cout_pad * kpad;
    const size_t n = 4 * per;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const int ph = (int)(i / per);
        const size_t rem = i - (size_t)ph * per;
        const int co = (int)(rem / kpad);
        const int k = (int)(rem - (size_t)co * kpad);
        const int tap = k / Cin, ci = k - (k / Cin) * Cin;
        float v = 0.f;
        if (co < Cout && tap < 4) {
            const int ry = ph >> 1, rx = ph & 1;
            const int dy = tap >> 1, dx = tap & 1;
            const int ky = ry == 0 ? (dy == 0 ? 3 : 1) : (dy == 0 ? 2 : 0);
            const int kx = rx == 0 ? (dx == 0 ? 3 : 1) : (dx == 0 ? 2 : 0);
            v = w[(((size_t)ci * Cout + co) * 4 + ky) * 4 + kx];
        }
        wpk[i] = v;
    }
}

}  // namespace
}  // namespace tcx

using namespace tcx;

extern "C" int tcx_conv2d(const float* x1, const float* x2, int Bt, int bmod, int H, int W, int C1, int C2,
                          const float* wpk, const float* bias, const float* bias_b, const float* resid,
                          float* y, int Cout, int cout_pad, int kpad, int ks, int stride, int pad,
                          int circular, int upsample, int act, double* gn_stats, void* stream) {
    TCX_REQUIRE(x1 && wpk && y, "tcx_conv2d: null pointer");
    TCX_REQUIRE(Bt >= 0 && H > 0 && W > 0 && C1 > 0 && C2 >= 0 && Cout > 0, "tcx_conv2d: bad shape");
    TCX_REQUIRE((C2 == 0) == (x2 == nullptr), "tcx_conv2d: x2/C2 mismatch");
    TCX_REQUIRE(cout_pad >= Cout && cout_pad % 32 == 0, "tcx_conv2d: cout_pad must be a multiple of 32 >= Cout");
    const int Cin = C1 + C2;
    TCX_REQUIRE(kpad % BK == 0 && kpad >= ks * ks * Cin, "tcx_conv2d: kpad must be a multiple of 32 >= ks*ks*Cin");
    TCX_REQUIRE(ks >= 1 && stride >= 1 && pad >= 0, "tcx_conv2d: bad geometry");
    ConvParams p{};
    p.x1 = x1; p.x2 = x2; p.C1 = C1; p.C2 = C2; p.Cin = Cin;
    p.bmod = bmod; p.H = H; p.W = W;
    p.Hi = upsample ? 2 * H : H;
    p.Wi = upsample ? 2 * W : W;
    p.Ho = (p.Hi + 2 * pad - ks) / stride + 1;
    p.Wo = (p.Wi + 2 * pad - ks) / stride + 1;
    TCX_REQUIRE(p.Ho > 0 && p.Wo > 0, "tcx_conv2d: empty output");
    p.HoWo = p.Ho * p.Wo;
    p.M = Bt * p.HoWo;
    p.w = wpk; p.bias = bias; p.bias_b = bias_b; p.resid = resid; p.y = y;
    p.Cout = Cout; p.kpad = kpad; p.nchunks = kpad / BK;
    p.ks = ks; p.stride = stride; p.pad_y = pad; p.pad_x = pad; p.circular = circular;
    TCX_REQUIRE(act >= 0 && act <= 3, "tcx_conv2d: bad act");
    p.Hy = p.Ho; p.Wy = p.Wo; p.osy = 1; p.ooy = 0; p.osx = 1; p.oox = 0; p.act = act;
    p.gn = gn_stats;
    p.nsplit = cdiv(p.HoWo, BM);
    int mode = 0;
    const bool vec_ok = (C1 % 4 == 0) && (C2 % 4 == 0) && aligned16(x1) && (!x2 || aligned16(x2));
    if (upsample) {
        TCX_REQUIRE(vec_ok && circular, "tcx_conv2d: upsample needs Cin%4==0, circular padding");
        mode = 2;
    } else if (!vec_ok) {
        TCX_REQUIRE(x2 == nullptr, "tcx_conv2d: scalar path supports a single source");
        mode = 1;
    }
    if (gn_stats) TCX_REQUIRE(p.HoWo % BM == 0, "tcx_conv2d: fused GN stats need Ho*Wo %% 128 == 0");
    TCX_REQUIRE(aligned16(wpk), "tcx_conv2d: packed weight must be 16-B aligned");
    return launch_conv(p, cout_pad, mode, (hipStream_t)stream);
}

extern "C" int tcx_convT2x(const float* x, int Bt, int H, int W, int Cin, const float* wpk4, const float* bias,
                           float* y, int Cout, int cout_pad, int kpad, int act, void* stream) {
    TCX_REQUIRE(x && wpk4 && y, "tcx_convT2x: null pointer");
    TCX_REQUIRE(cout_pad >= Cout && cout_pad % 32 == 0 && kpad % BK == 0 && kpad >= 4 * Cin, "tcx_convT2x: bad padding");
    for (int ph = 0; ph < 4; ++ph) {
        const int ry = ph >> 1, rx = ph & 1;
        ConvParams p{};
        p.x1 = x; p.x2 = nullptr; p.C1 = Cin; p.C2 = 0; p.Cin = Cin;
        p.bmod = 0; p.H = H; p.W = W; p.Hi = H; p.Wi = W;
        p.Ho = H; p.Wo = W; p.HoWo = H * W; p.M = Bt * H * W;
        p.w = wpk4 + (size_t)ph * cout_pad * kpad;
        p.bias = bias; p.bias_b = nullptr; p.resid = nullptr; p.y = y;
        p.Cout = Cout; p.kpad = kpad; p.nchunks = kpad / BK;
        p.ks = 2; p.stride = 1; p.pad_y = 1 - ry; p.pad_x = 1 - rx; p.circular = 0;
        p.Hy = 2 * H; p.Wy = 2 * W; p.osy = 2; p.ooy = ry; p.osx = 2; p.oox = rx;
        p.act = act; p.gn = nullptr; p.nsplit = 1;
        const bool vec_ok = (Cin % 4 == 0) && aligned16(x);
        TCX_TRY(launch_conv(p, cout_pad, vec_ok ? 0 : 1, (hipStream_t)stream));
    }
    return TCX_OK;
}

extern "C" int tcx_pack_conv_weight(const float* w, float* wpk, int Cout, int Cin, int ks, int cout_pad, int kpad,
                                    void* stream) {
    TCX_REQUIRE(w && wpk && cout_pad >= Cout && kpad >= ks * ks * Cin, "tcx_pack_conv_weight: bad args");
    const size_t n = (size_t)cout_pad * kpad;
    const int blocks = (int)std::min<size_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(k_pack_conv, dim3(blocks), dim3(256), 0, (hipStream_t)stream, w, wpk, Cout, Cin, ks, cout_pad, kpad);
    return check_launch("tcx_pack_conv_weight");
}

extern "C" int tcx_pack_convT_weight(const float* w, float* wpk, int Cin, int Cout, int cout_pad, int kpad,
                                     void* stream) {
    TCX_REQUIRE(w && wpk && cout_pad >= Cout && kpad >= 4 * Cin, "tcx_pack_convT_weight: bad args");
    const size_t n = 4 * (size_t)cout_pad * kpad;
    const int blocks = (int)std::min<size_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(k_pack_convT, dim3(blocks), dim3(256), 0, (hipStream_t)stream, w, wpk, Cin, Cout, cout_pad, kpad);
    return check_launch("tcx_pack_convT_weight");
}

extern "C" int tcx_linear(const float* x1, int K1, const float* x2, int K2, const float* wpk, const float* b,
                          const float* resid, float* y, int M, int N, int npad, int kpad, int act, void* stream) {
    const int K = K1 + K2;
    TCX_REQUIRE(x1 && wpk && y && M >= 0 && N > 0 && K1 > 0 && K2 >= 0, "tcx_linear: bad args");
    TCX_REQUIRE((K2 == 0) == (x2 == nullptr), "tcx_linear: x2/K2 mismatch");
    TCX_REQUIRE(npad >= N && npad % 32 == 0 && kpad >= K && kpad % BK == 0, "tcx_linear: bad padding");
    TCX_REQUIRE(act >= 0 && act <= 3, "tcx_linear: bad act");
    ConvParams p{};
    p.x1 = x1; p.x2 = x2; p.C1 = K1; p.C2 = K2; p.Cin = K;
    p.bmod = 0; p.H = 1; p.W = 1; p.Hi = 1; p.Wi = 1; p.Ho = 1; p.Wo = 1; p.HoWo = 1; p.M = M;
    p.w = wpk; p.bias = b; p.bias_b = nullptr; p.resid = resid; p.y = y;
    p.Cout = N; p.kpad = kpad; p.nchunks = kpad / BK;
    p.ks = 1; p.stride = 1; p.pad_y = 0; p.pad_x = 0; p.circular = 0;
    p.Hy = 1; p.Wy = 1; p.osy = 1; p.ooy = 0; p.osx = 1; p.oox = 0; p.act = act; p.gn = nullptr; p.nsplit = 1;
    const bool vec_ok = (K1 % 4 == 0) && (K2 % 4 == 0) && aligned16(x1) && (!x2 || aligned16(x2));
    TCX_REQUIRE(vec_ok || x2 == nullptr, "tcx_linear: two-source form needs K1,K2 %% 4 == 0 and aligned rows");
    return launch_conv(p, npad, vec_ok ? 0 : 1, (hipStream_t)stream);
}
