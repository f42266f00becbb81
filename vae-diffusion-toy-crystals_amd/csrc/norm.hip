// GroupNorm (+SiLU), LayerNorm/FiLM, bilinear x2 upsample — HBM-bound kernels, NHWC fp32.
//
// GroupNorm(8, C, eps=1e-5) of CondUNetTiny (/root/reference/src/toycrystals/models/
// sde_score_model.py:103,106,130 via _gn_groups :89-94) is split in two phases so that the
// statistics can come either from tcx_gn_partials or from the producing conv's epilogue
// (tcx_conv2d gn_stats): partial {sum, sumsq} per (batch, split, channel) in fp64, then an
// apply pass that folds mean/rstd/gamma/beta into one per-channel scale/shift and fuses SiLU.
#include "common.hpp"
#include "skinny.hpp"
#include "h2.hpp"

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

// grid (chunks, Bt); each block normalises pixels [chunk*ppb, ...) of image b.
__global__ __launch_bounds__(256) void k_gn_apply(const float* __restrict__ x, float* __restrict__ y, int HW, int C,
                                                  int groups, const double* __restrict__ part, int nsplit,
                                                  const float* __restrict__ gamma, const float* __restrict__ beta,
                                                  float eps, int silu, int ppb) {
    extern __shared__ __attribute__((aligned(16))) float lsm[];  // sc[C], sh[C], gstat, csum
    float* sc = lsm;
    float* sh = lsm + ((C + 3) & ~3);
    double* gstat = reinterpret_cast<double*>(lsm + 2 * ((C + 3) & ~3));
    double* csum = gstat + 2 * groups;
    const int b = blockIdx.y;
    gn_scale_shift(part, b, nsplit, C, groups, HW, gamma, beta, eps, sc, sh, gstat, csum);
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

// Streaming GroupNorm apply from per-(b, c) tables: y = act(x * scale + shift).  grid (chunks, Bt).
__global__ __launch_bounds__(256) void k_gn_apply_tab(const float* __restrict__ x, float* __restrict__ y, int HW, int C,
                                                      const float* __restrict__ tsc, const float* __restrict__ tsh,
                                                      int silu, int ppb, unsigned* __restrict__ amax) {
    extern __shared__ __attribute__((aligned(16))) float lsm[];
    float* sc = lsm;
    float* sh = lsm + ((C + 3) & ~3);
    const int b = blockIdx.y;
    for (int c = threadIdx.x; c < C; c += 256) {
        sc[c] = tsc[(size_t)b * C + c];
        sh[c] = tsh[(size_t)b * C + c];
    }
    __syncthreads();
    const int p0 = blockIdx.x * ppb;
    const int p1 = min(HW, p0 + ppb);
    const size_t base = ((size_t)b * HW + p0) * C;
    const int n4 = (p1 - p0) * C / 4;
    const int C4 = C / 4;
    int i = threadIdx.x;
    float m = 0.f;  // max |y| of this thread's elements (only reported when amax is given)
    for (; i + 256 < n4; i += 512) {  // two float4 in flight per thread
        const int c0 = (i % C4) * 4, c1 = ((i + 256) % C4) * 4;
        float4 v0 = *reinterpret_cast<const float4*>(x + base + (size_t)i * 4);
        float4 v1 = *reinterpret_cast<const float4*>(x + base + (size_t)(i + 256) * 4);
        v0.x = fmaf(v0.x, sc[c0], sh[c0]); v0.y = fmaf(v0.y, sc[c0 + 1], sh[c0 + 1]);
        v0.z = fmaf(v0.z, sc[c0 + 2], sh[c0 + 2]); v0.w = fmaf(v0.w, sc[c0 + 3], sh[c0 + 3]);
        v1.x = fmaf(v1.x, sc[c1], sh[c1]); v1.y = fmaf(v1.y, sc[c1 + 1], sh[c1 + 1]);
        v1.z = fmaf(v1.z, sc[c1 + 2], sh[c1 + 2]); v1.w = fmaf(v1.w, sc[c1 + 3], sh[c1 + 3]);
        if (silu) {
            v0.x = silu_f(v0.x); v0.y = silu_f(v0.y); v0.z = silu_f(v0.z); v0.w = silu_f(v0.w);
            v1.x = silu_f(v1.x); v1.y = silu_f(v1.y); v1.z = silu_f(v1.z); v1.w = silu_f(v1.w);
        }
        *reinterpret_cast<float4*>(y + base + (size_t)i * 4) = v0;
        *reinterpret_cast<float4*>(y + base + (size_t)(i + 256) * 4) = v1;
        m = fmaxf(m, fmaxf(absmax4(v0), absmax4(v1)));
    }
    for (; i < n4; i += 256) {
        const int c = (i % C4) * 4;
        float4 v = *reinterpret_cast<const float4*>(x + base + (size_t)i * 4);
        v.x = fmaf(v.x, sc[c], sh[c]); v.y = fmaf(v.y, sc[c + 1], sh[c + 1]);
        v.z = fmaf(v.z, sc[c + 2], sh[c + 2]); v.w = fmaf(v.w, sc[c + 3], sh[c + 3]);
        if (silu) {
            v.x = silu_f(v.x); v.y = silu_f(v.y); v.z = silu_f(v.z); v.w = silu_f(v.w);
        }
        *reinterpret_cast<float4*>(y + base + (size_t)i * 4) = v;
        m = fmaxf(m, absmax4(v));
    }
    if (amax) block_amax_publish(m, amax);
}

// One block per image: partials -> per-(b, c) scale/shift tables for a fused GN(+SiLU) prologue.
__global__ __launch_bounds__(1024) void k_gn_finalize(const double* __restrict__ part, int HW, int C, int groups,
                                                     int nsplit, const float* __restrict__ gamma,
                                                     const float* __restrict__ beta, float eps,
                                                     float* __restrict__ scale, float* __restrict__ shift) {
    extern __shared__ __attribute__((aligned(16))) float lsm[];
    float* sc = lsm;
    float* sh = lsm + ((C + 3) & ~3);
    double* gstat = reinterpret_cast<double*>(lsm + 2 * ((C + 3) & ~3));
    double* csum = gstat + 2 * groups;
    double* lsum = csum + 2 * C;  // [lanes][C][2]
    const int b = blockIdx.x;
    // 1024 threads: `lanes` threads per channel each sum a strided subset of the nsplit partials (the
    // one-thread-per-channel loop left 3/4 of a 256-thread block idle and was ~45 us at 256^2, where
    // nsplit is 512), then one thread per channel adds its lanes in lane order (deterministic)
    const int lanes = max(1, (int)blockDim.x / C);
    const double* pb = part + (size_t)b * nsplit * C * 2;
    for (int t = threadIdx.x; t < lanes * C; t += blockDim.x) {
        const int l = t / C, c = t - (t / C) * C;
        double a = 0, q = 0;
#pragma unroll 4
        for (int sp = l; sp < nsplit; sp += lanes) {
            const double2 v = *reinterpret_cast<const double2*>(pb + ((size_t)sp * C + c) * 2);
            a += v.x;
            q += v.y;
        }
        lsum[2 * t] = a;
        lsum[2 * t + 1] = q;
    }
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
        double a = 0, q = 0;
        for (int l = 0; l < lanes; ++l) {
            a += lsum[2 * (l * C + c)];
            q += lsum[2 * (l * C + c) + 1];
        }
        csum[2 * c] = a;
        csum[2 * c + 1] = q;
    }
    __syncthreads();
    gn_tables_from_csum(C, groups, HW, gamma, beta, eps, sc, sh, gstat, csum);
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
        scale[(size_t)b * C + c] = sc[c];
        shift[(size_t)b * C + c] = sh[c];
    }
}

constexpr int UPK = 4;  // output quads per thread of the upsample (4 x 4 float4 loads in flight)
template <bool OUTH2>
__global__ __launch_bounds__(256) void k_upsample2x(const float* __restrict__ x, float* __restrict__ y, int Bt, int H,
                                                    int W, int C, const float* __restrict__ tsc,
                                                    const float* __restrict__ tsh, unsigned* ovf, int bf) {
    // one output row (b, oy) per blockIdx.x, a chunk of UPK * 256 of its 2W * C/4 channel quads
    // per blockIdx.y.  The row's two source rows and weights are block-uniform (32-bit index
    // math only: the former flat 64-bit div/mod per element was the cost); the 4 x UPK source
    // loads of a thread are issued before any is used.
    bool bad = false;
    const int C4 = C / 4;
    const int oy = blockIdx.x % (2 * H), b = blockIdx.x / (2 * H);
    float sy = 0.5f * ((float)oy + 0.5f) - 0.5f;
    sy = sy < 0.f ? 0.f : sy;
    const int y0 = (int)sy;
    const int y1 = y0 + (y0 < H - 1 ? 1 : 0);
    const float ly1 = sy - (float)y0, ly0 = 1.f - ly1;
    const float* r0 = x + ((size_t)b * H + y0) * W * C;
    const float* r1 = x + ((size_t)b * H + y1) * W * C;
    const int nq = 2 * W * C4;
    const size_t orow = ((size_t)b * 2 * H + oy) * 2 * W * C4;  // first quad of the output row
    const int i0 = blockIdx.y * (UPK * 256) + threadIdx.x;
    float4 a[UPK], bq[UPK], c[UPK], d[UPK];
#pragma unroll
    for (int k = 0; k < UPK; ++k) {
        const int i = i0 + 256 * k;
        if (i < nq) {
            const int ox = i / C4, c4 = i - (i / C4) * C4;
            float sx = 0.5f * ((float)ox + 0.5f) - 0.5f;
            sx = sx < 0.f ? 0.f : sx;
            const int x0 = (int)sx, x1 = x0 + (x0 < W - 1 ? 1 : 0);
            a[k] = *reinterpret_cast<const float4*>(r0 + x0 * C + c4 * 4);
            bq[k] = *reinterpret_cast<const float4*>(r0 + x1 * C + c4 * 4);
            c[k] = *reinterpret_cast<const float4*>(r1 + x0 * C + c4 * 4);
            d[k] = *reinterpret_cast<const float4*>(r1 + x1 * C + c4 * 4);
        }
    }
#pragma unroll
    for (int k = 0; k < UPK; ++k) {
        const int i = i0 + 256 * k;
        if (i < nq) {
            const int ox = i / C4, c4 = i - (i / C4) * C4;
            float sx = 0.5f * ((float)ox + 0.5f) - 0.5f;
            sx = sx < 0.f ? 0.f : sx;
            const int x0 = (int)sx;
            const float lx1 = sx - (float)x0, lx0 = 1.f - lx1;
            if (tsc) {  // fused GN+SiLU of the source
                const float4 s4 = *reinterpret_cast<const float4*>(tsc + (size_t)b * C + c4 * 4);
                const float4 h4 = *reinterpret_cast<const float4*>(tsh + (size_t)b * C + c4 * 4);
                auto tr = [&](float4& v) {
                    v.x = silu_f(fmaf(v.x, s4.x, h4.x)); v.y = silu_f(fmaf(v.y, s4.y, h4.y));
                    v.z = silu_f(fmaf(v.z, s4.z, h4.z)); v.w = silu_f(fmaf(v.w, s4.w, h4.w));
                };
                tr(a[k]); tr(bq[k]); tr(c[k]); tr(d[k]);
            }
            // explicit fmaf: the same rounding in every instantiation (fp32 and h2 outputs)
            auto bl = [&](float va, float vb, float vc, float vd) {
                return fmaf(ly1, fmaf(lx1, vd, lx0 * vc), ly0 * fmaf(lx1, vb, lx0 * va));
            };
            float4 o;
            o.x = bl(a[k].x, bq[k].x, c[k].x, d[k].x);
            o.y = bl(a[k].y, bq[k].y, c[k].y, d[k].y);
            o.z = bl(a[k].z, bq[k].z, c[k].z, d[k].z);
            o.w = bl(a[k].w, bq[k].w, c[k].w, d[k].w);
            const size_t q = orow + i;
            if constexpr (OUTH2) {
                const size_t pix = ((size_t)b * 2 * H + oy) * 2 * W + ox;
                store4_h2x(reinterpret_cast<char*>(y), pix * C * 4, c4, o, bf != 0);
                bad = bad || h2_bad(o.x) || h2_bad(o.y) || h2_bad(o.z) || h2_bad(o.w);
            } else {
                *reinterpret_cast<float4*>(y + q * 4) = o;
            }
        }
    }
    h2_flag(ovf, bad && !bf);
}

// h2-output upsample with one 8-channel group per item: a thread reads 2 x 16 B per source tap and
// writes the group's 16-B hi and 16-B lo records (the quad form above writes 8-B halves).
typedef float f4v __attribute__((ext_vector_type(4)));
constexpr int UPG = 2;  // 8-channel groups per thread
__global__ __launch_bounds__(256) void k_upsample2x_g8(const float* __restrict__ x, char* __restrict__ y, int H, int W,
                                                       int C, const float* __restrict__ tsc,
                                                       const float* __restrict__ tsh, unsigned* ovf, int bf) {
    bool bad = false;
    const int C8 = C / 8;
    const int oy = blockIdx.x % (2 * H), b = blockIdx.x / (2 * H);
    float sy = 0.5f * ((float)oy + 0.5f) - 0.5f;
    sy = sy < 0.f ? 0.f : sy;
    const int y0 = (int)sy;
    const int y1 = y0 + (y0 < H - 1 ? 1 : 0);
    const float ly1 = sy - (float)y0, ly0 = 1.f - ly1;
    const float* r0 = x + ((size_t)b * H + y0) * W * C;
    const float* r1 = x + ((size_t)b * H + y1) * W * C;
    const int ng = 2 * W * C8;
    const int i0 = blockIdx.y * (UPG * 256) + threadIdx.x;
    f4v a[UPG][2], bq[UPG][2], c[UPG][2], d[UPG][2];
#pragma unroll
    for (int k = 0; k < UPG; ++k) {
        const int i = i0 + 256 * k;
        if (i < ng) {
            const int ox = i / C8, g = i - (i / C8) * C8;
            float sx = 0.5f * ((float)ox + 0.5f) - 0.5f;
            sx = sx < 0.f ? 0.f : sx;
            const int x0 = (int)sx, x1 = x0 + (x0 < W - 1 ? 1 : 0);
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                a[k][h] = *reinterpret_cast<const f4v*>(r0 + x0 * C + 8 * g + 4 * h);
                bq[k][h] = *reinterpret_cast<const f4v*>(r0 + x1 * C + 8 * g + 4 * h);
                c[k][h] = *reinterpret_cast<const f4v*>(r1 + x0 * C + 8 * g + 4 * h);
                d[k][h] = *reinterpret_cast<const f4v*>(r1 + x1 * C + 8 * g + 4 * h);
            }
        }
    }
#pragma unroll
    for (int k = 0; k < UPG; ++k) {
        const int i = i0 + 256 * k;
        if (i < ng) {
            const int ox = i / C8, g = i - (i / C8) * C8;
            float sx = 0.5f * ((float)ox + 0.5f) - 0.5f;
            sx = sx < 0.f ? 0.f : sx;
            const int x0 = (int)sx;
            const float lx1 = sx - (float)x0, lx0 = 1.f - lx1;
            uint2 hi[2], lo[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                f4v va = a[k][h], vb = bq[k][h], vc = c[k][h], vd = d[k][h];
                if (tsc) {  // fused GN+SiLU of the source
                    const f4v s4 = *reinterpret_cast<const f4v*>(tsc + (size_t)b * C + 8 * g + 4 * h);
                    const f4v h4 = *reinterpret_cast<const f4v*>(tsh + (size_t)b * C + 8 * g + 4 * h);
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        va[e] = silu_f(fmaf(va[e], s4[e], h4[e]));
                        vb[e] = silu_f(fmaf(vb[e], s4[e], h4[e]));
                        vc[e] = silu_f(fmaf(vc[e], s4[e], h4[e]));
                        vd[e] = silu_f(fmaf(vd[e], s4[e], h4[e]));
                    }
                }
                float o[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) {  // the quad kernel's fmaf order: identical values
                    o[e] = fmaf(ly1, fmaf(lx1, vd[e], lx0 * vc[e]), ly0 * fmaf(lx1, vb[e], lx0 * va[e]));
                    bad = bad || h2_bad(o[e]);
                }
                split4x(make_float4(o[0], o[1], o[2], o[3]), hi[h], lo[h], bf != 0);
            }
            const size_t pix = ((size_t)b * 2 * H + oy) * 2 * W + ox;
            if (bf == 2) {  // 2-byte bf16 (h2.hpp "b2"): the hi halves only
                *reinterpret_cast<uint4*>(y + (pix * C + 8 * (size_t)g) * 2) = make_uint4(hi[0].x, hi[0].y, hi[1].x, hi[1].y);
            } else {
                char* gp = y + pix * C * 4 + 32 * (size_t)g;
                *reinterpret_cast<uint4*>(gp) = make_uint4(hi[0].x, hi[0].y, hi[1].x, hi[1].y);
                *reinterpret_cast<uint4*>(gp + 16) = make_uint4(lo[0].x, lo[0].y, lo[1].x, lo[1].y);
            }
        }
    }
    h2_flag(ovf, bad && !bf);
}

// Banded bilinear x2 upsample -> h2 (us1 / us2 of sde_score_model.py:217-222, 256, 261): one workgroup
// per (image, band of ROWS output rows).  The band's ROWS / 2 + 2 source rows (one clamped halo row
// either side) are read from HBM once, put through the optional GroupNorm+SiLU of the source ONCE per
// element (the fused form of k_upsample2x_g8 recomputes it for each of the 4 taps of every output,
// 16x per element; SiLU here as in the conv prologues, y rcp(1 + exp2(-y log2 e))) and held in LDS as
// fp32; every output 8-channel group then reads its 4 taps from LDS (same fmaf order as
// k_upsample2x_g8) and is written as two 16-B pieces.
constexpr int UB_MAXWC = 3072;             // W * C of one source row (72 KB of LDS for an 8-row band)
// ROWS output rows per band (ROWS / 2 + 2 source rows staged); G8: one 8-channel group per item (two
// 16-B stores) instead of one 4-channel quad (two 8-B stores)
template <int ROWS, bool G8>
__global__ __launch_bounds__(256, 2) void k_upsample2x_band(const float* __restrict__ x, char* __restrict__ y, int H,
                                                           int W, int C, const float* __restrict__ tsc,
                                                           const float* __restrict__ tsh, unsigned* ovf, int bf) {
    constexpr int SRC = ROWS / 2 + 2;
    extern __shared__ __attribute__((aligned(16))) float ub[];  // [SRC][W][C]
    const int nband = 2 * H / ROWS;
    const int b = blockIdx.x / nband, band = blockIdx.x - (blockIdx.x / nband) * nband;
    const int ys0 = band * (ROWS / 2) - 1;  // source row of LDS row 0 (before clamping)
    const int WC = W * C, WC4 = WC / 4, C4 = C / 4;
    // phase 1: SRC source rows (clamped), GroupNorm+SiLU once per element, into LDS
    constexpr int NL = (SRC * UB_MAXWC / 4 + 255) / 256;
    f4v v[NL];
#pragma unroll
    for (int k = 0; k < NL; ++k) {
        const int i = threadIdx.x + 256 * k;
        if (i < SRC * WC4) {
            const int r = i / WC4, e = i - (i / WC4) * WC4;
            const int ysrc = min(max(ys0 + r, 0), H - 1);
            v[k] = *reinterpret_cast<const f4v*>(x + ((size_t)b * H + ysrc) * WC + 4 * e);
        }
    }
#pragma unroll
    for (int k = 0; k < NL; ++k) {
        const int i = threadIdx.x + 256 * k;
        if (i < SRC * WC4) {
            if (tsc) {
                const int c4 = (i - (i / C4) * C4) * 4;
                const f4v s4 = *reinterpret_cast<const f4v*>(tsc + (size_t)b * C + c4);
                const f4v h4 = *reinterpret_cast<const f4v*>(tsh + (size_t)b * C + c4);
#pragma unroll
                for (int e = 0; e < 4; ++e) {  // SiLU as y rcp(1 + exp2(-y log2 e)), as the conv prologues
                    const float yv = fmaf(v[k][e], s4[e], h4[e]);
                    v[k][e] = yv * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-1.4426950408889634f * yv));
                }
            }
            *reinterpret_cast<f4v*>(ub + 4 * i) = v[k];
        }
    }
    __syncthreads();
    // phase 2: output items (oy, ox, quad or group), channel index fastest
    bool bad = false;
    constexpr int CW = G8 ? 8 : 4;  // channels per item
    const int CI = C / CW;
    const int nq = ROWS * 2 * W * CI;
    for (int i = threadIdx.x; i < nq; i += 256) {
        const int q = i % CI, rest = i / CI;
        const int ox = rest % (2 * W), ry = rest / (2 * W);
        const int oy = band * ROWS + ry;
        float sy = 0.5f * ((float)oy + 0.5f) - 0.5f;
        sy = sy < 0.f ? 0.f : sy;
        const int y0 = (int)sy;
        const int y1 = y0 + (y0 < H - 1 ? 1 : 0);
        const float ly1 = sy - (float)y0, ly0 = 1.f - ly1;
        float sx = 0.5f * ((float)ox + 0.5f) - 0.5f;
        sx = sx < 0.f ? 0.f : sx;
        const int x0 = (int)sx, x1 = x0 + (x0 < W - 1 ? 1 : 0);
        const float lx1 = sx - (float)x0, lx0 = 1.f - lx1;
        const float* r0 = ub + (y0 - ys0) * WC + CW * q;
        const float* r1 = ub + (y1 - ys0) * WC + CW * q;
        const size_t pix = ((size_t)b * 2 * H + oy) * 2 * W + ox;
        uint2 hi[2], lo[2];
#pragma unroll
        for (int h = 0; h < CW / 4; ++h) {
            const f4v va = *reinterpret_cast<const f4v*>(r0 + x0 * C + 4 * h);
            const f4v vb = *reinterpret_cast<const f4v*>(r0 + x1 * C + 4 * h);
            const f4v vc = *reinterpret_cast<const f4v*>(r1 + x0 * C + 4 * h);
            const f4v vd = *reinterpret_cast<const f4v*>(r1 + x1 * C + 4 * h);
            float o[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                o[e] = fmaf(ly1, fmaf(lx1, vd[e], lx0 * vc[e]), ly0 * fmaf(lx1, vb[e], lx0 * va[e]));
                bad = bad || h2_bad(o[e]);
            }
            split4x(make_float4(o[0], o[1], o[2], o[3]), hi[h], lo[h], bf != 0);
        }
        if (bf == 2) {  // 2-byte bf16 (h2.hpp "b2"): the hi halves only
            char* gp = y + (pix * C + (size_t)CW * q) * 2;
            if constexpr (G8) *reinterpret_cast<uint4*>(gp) = make_uint4(hi[0].x, hi[0].y, hi[1].x, hi[1].y);
            else *reinterpret_cast<uint2*>(gp) = hi[0];
        } else if constexpr (G8) {
            char* gp = y + pix * C * 4 + 32 * (size_t)q;
            *reinterpret_cast<uint4*>(gp) = make_uint4(hi[0].x, hi[0].y, hi[1].x, hi[1].y);
            *reinterpret_cast<uint4*>(gp + 16) = make_uint4(lo[0].x, lo[0].y, lo[1].x, lo[1].y);
        } else {
            char* gp = y + pix * C * 4 + 32 * (size_t)(q >> 1) + 8 * (q & 1);
            *reinterpret_cast<uint2*>(gp) = hi[0];
            *reinterpret_cast<uint2*>(gp + 16) = lo[0];
        }
    }
    h2_flag(ovf, bad && !bf);
}

// Column-segmented form of k_upsample2x_band for source rows wider than the LDS holds (config 5's us1 /
// us2 at 256^2: 128 x 96 and 64 x 192 floats per source row): one workgroup per (image, band of ROWS
// output rows, segment of SW source columns).  The segment's SW columns and one clamped halo column
// either side (the bilinear taps of its 2 SW output columns) are staged; the arithmetic per output is
// that of k_upsample2x_band / k_upsample2x_g8 (same clamped coordinates, same fmaf order).
template <int ROWS>
__global__ __launch_bounds__(256, 2) void k_upsample2x_bandseg(const float* __restrict__ x, char* __restrict__ y,
                                                              int H, int W, int C, int SW,
                                                              const float* __restrict__ tsc,
                                                              const float* __restrict__ tsh, unsigned* ovf, int bf) {
    constexpr int SRC = ROWS / 2 + 2;
    extern __shared__ __attribute__((aligned(16))) float ub[];  // [SRC][SW + 2][C]
    const int nband = 2 * H / ROWS, nseg = W / SW;
    const int seg = blockIdx.x % nseg;
    const int rest = blockIdx.x / nseg;
    const int b = rest / nband, band = rest - (rest / nband) * nband;
    const int ys0 = band * (ROWS / 2) - 1;  // source row of LDS row 0 (before clamping)
    const int xs0 = seg * SW - 1;           // source column of LDS column 0 (before clamping)
    const int SC2 = SW + 2;
    const int RC4 = SC2 * C / 4, C4 = C / 4;
    constexpr int NL = (SRC * UB_MAXWC / 4 + 255) / 256;
    f4v v[NL];
#pragma unroll
    for (int k = 0; k < NL; ++k) {
        const int i = threadIdx.x + 256 * k;
        if (i < SRC * RC4) {
            const int r = i / RC4, e = i - (i / RC4) * RC4;
            const int col = e / C4, c4 = e - (e / C4) * C4;
            const int ysrc = min(max(ys0 + r, 0), H - 1);
            const int xsrc = min(max(xs0 + col, 0), W - 1);
            v[k] = *reinterpret_cast<const f4v*>(x + (((size_t)b * H + ysrc) * W + xsrc) * C + 4 * c4);
        }
    }
#pragma unroll
    for (int k = 0; k < NL; ++k) {
        const int i = threadIdx.x + 256 * k;
        if (i < SRC * RC4) {
            if (tsc) {
                const int c4 = (i - (i / C4) * C4) * 4;
                const f4v s4 = *reinterpret_cast<const f4v*>(tsc + (size_t)b * C + c4);
                const f4v h4 = *reinterpret_cast<const f4v*>(tsh + (size_t)b * C + c4);
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float yv = fmaf(v[k][e], s4[e], h4[e]);
                    v[k][e] = yv * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-1.4426950408889634f * yv));
                }
            }
            *reinterpret_cast<f4v*>(ub + 4 * i) = v[k];
        }
    }
    __syncthreads();
    bool bad = false;
    const int CI = C / 8;
    const int nq = ROWS * 2 * SW * CI;
    for (int i = threadIdx.x; i < nq; i += 256) {
        const int q = i % CI, r2 = i / CI;
        const int oxl = r2 % (2 * SW), ry = r2 / (2 * SW);
        const int ox = 2 * seg * SW + oxl;
        const int oy = band * ROWS + ry;
        float sy = 0.5f * ((float)oy + 0.5f) - 0.5f;
        sy = sy < 0.f ? 0.f : sy;
        const int y0 = (int)sy;
        const int y1 = y0 + (y0 < H - 1 ? 1 : 0);
        const float ly1 = sy - (float)y0, ly0 = 1.f - ly1;
        float sx = 0.5f * ((float)ox + 0.5f) - 0.5f;
        sx = sx < 0.f ? 0.f : sx;
        const int x0 = (int)sx, x1 = x0 + (x0 < W - 1 ? 1 : 0);
        const float lx1 = sx - (float)x0, lx0 = 1.f - lx1;
        const float* r0 = ub + (y0 - ys0) * SC2 * C + 8 * q;
        const float* r1 = ub + (y1 - ys0) * SC2 * C + 8 * q;
        const int c0 = (x0 - xs0) * C, c1 = (x1 - xs0) * C;
        const size_t pix = ((size_t)b * 2 * H + oy) * 2 * W + ox;
        uint2 hi[2], lo[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const f4v va = *reinterpret_cast<const f4v*>(r0 + c0 + 4 * h);
            const f4v vb = *reinterpret_cast<const f4v*>(r0 + c1 + 4 * h);
            const f4v vc = *reinterpret_cast<const f4v*>(r1 + c0 + 4 * h);
            const f4v vd = *reinterpret_cast<const f4v*>(r1 + c1 + 4 * h);
            float o[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                o[e] = fmaf(ly1, fmaf(lx1, vd[e], lx0 * vc[e]), ly0 * fmaf(lx1, vb[e], lx0 * va[e]));
                bad = bad || h2_bad(o[e]);
            }
            split4x(make_float4(o[0], o[1], o[2], o[3]), hi[h], lo[h], bf != 0);
        }
        if (bf == 2) {  // 2-byte bf16 (h2.hpp "b2"): the hi halves only
            *reinterpret_cast<uint4*>(y + (pix * C + 8 * (size_t)q) * 2) = make_uint4(hi[0].x, hi[0].y, hi[1].x, hi[1].y);
        } else {
            char* gp = y + pix * C * 4 + 32 * (size_t)q;
            *reinterpret_cast<uint4*>(gp) = make_uint4(hi[0].x, hi[0].y, hi[1].x, hi[1].y);
            *reinterpret_cast<uint4*>(gp + 16) = make_uint4(lo[0].x, lo[0].y, lo[1].x, lo[1].y);
        }
    }
    h2_flag(ovf, bad && !bf);
}

// GroupNorm (+ SiLU) apply from tables into 2-byte bf16 (h2.hpp "b2", config 5): one thread per (pixel,
// 8-channel group), the source fp32 (32 B) or itself b2 (16 B, in place: the conv wrote its pre-norm
// output as bf16), the result 16 B of bf16.  Loads of a batch of GU groups before any store, the next
// batch's loads before this batch's stores (k_gn_apply_tab_h2's order).
template <bool IN_B2>
__global__ __launch_bounds__(256) void k_gn_apply_b2(const char* x, char* y, int HW, int C,
                                                     const float* __restrict__ tsc, const float* __restrict__ tsh,
                                                     int silu, int ppb) {
    extern __shared__ __attribute__((aligned(16))) float lsm[];
    float* sc = lsm;
    float* sh = lsm + ((C + 3) & ~3);
    const int b = blockIdx.y;
    for (int c = threadIdx.x; c < C; c += 256) {
        sc[c] = tsc[(size_t)b * C + c];
        sh[c] = tsh[(size_t)b * C + c];
    }
    __syncthreads();
    const int p0 = blockIdx.x * ppb;
    const int p1 = min(HW, p0 + ppb);
    const size_t base = ((size_t)b * HW + p0) * C;  // element index of the block's first value
    const int C8 = C / 8;
    const int n8 = (p1 - p0) * C8;
    constexpr int GU = 4;
    uint4 n0[GU], n1[GU];
    auto ld = [&](int at, int k) {
        const size_t e = base + (size_t)(at + 256 * k) * 8;
        if constexpr (IN_B2) {
            n0[k] = *reinterpret_cast<const uint4*>(x + e * 2);
        } else {
            n0[k] = *reinterpret_cast<const uint4*>(x + e * 4);
            n1[k] = *reinterpret_cast<const uint4*>(x + e * 4 + 16);
        }
    };
    auto work = [&](int at, const uint4& a, const uint4& c) {
        float v[8];
        if constexpr (IN_B2) {
            v[0] = bf_lo(a.x); v[1] = bf_hi(a.x); v[2] = bf_lo(a.y); v[3] = bf_hi(a.y);
            v[4] = bf_lo(a.z); v[5] = bf_hi(a.z); v[6] = bf_lo(a.w); v[7] = bf_hi(a.w);
        } else {
            v[0] = __uint_as_float(a.x); v[1] = __uint_as_float(a.y); v[2] = __uint_as_float(a.z); v[3] = __uint_as_float(a.w);
            v[4] = __uint_as_float(c.x); v[5] = __uint_as_float(c.y); v[6] = __uint_as_float(c.z); v[7] = __uint_as_float(c.w);
        }
        const int c0 = (at % C8) * 8;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            v[e] = fmaf(v[e], sc[c0 + e], sh[c0 + e]);
            if (silu) v[e] = silu_hw(v[e]);
        }
        *reinterpret_cast<uint4*>(y + (base + (size_t)at * 8) * 2) =
            make_uint4(pack2_bf(v[0], v[1]), pack2_bf(v[2], v[3]), pack2_bf(v[4], v[5]), pack2_bf(v[6], v[7]));
    };
    int i = threadIdx.x;
    if (i + (GU - 1) * 256 < n8)
#pragma unroll
        for (int k = 0; k < GU; ++k) ld(i, k);
    for (; i + (GU - 1) * 256 < n8; i += GU * 256) {
        uint4 u0[GU], u1[GU];
#pragma unroll
        for (int k = 0; k < GU; ++k) {
            u0[k] = n0[k];
            u1[k] = n1[k];
        }
        if (i + GU * 256 + (GU - 1) * 256 < n8)
#pragma unroll
            for (int k = 0; k < GU; ++k) ld(i + GU * 256, k);
#pragma unroll
        for (int k = 0; k < GU; ++k) work(i + 256 * k, u0[k], u1[k]);
    }
    for (; i < n8; i += 256) {
        ld(i, 0);
        work(i, n0[0], n1[0]);
    }
}

// LayerNorm over rows of width Wd (+ optional FiLM h*(1+gamma)+beta), one wave per row.
// gamma = gb[row][i] (+ gt[i]), beta = gb[row][Wd + i] (+ gt[Wd + i]): gt is one row broadcast over
// all rows (the prior DDIM's per-step time half of the FiLM projection, prior.hip).
__global__ __launch_bounds__(256) void k_layernorm_film(const float* __restrict__ x, float* __restrict__ y, int M,
                                                        int Wd, const float* __restrict__ lw,
                                                        const float* __restrict__ lb, const float* __restrict__ gb,
                                                        int ld_gb, const float* __restrict__ gt, float eps) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (row >= M) return;
    const float* xr = x + (size_t)row * Wd;
    if (Wd == 1024 && (ld_gb & 3) == 0 &&
        ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y) | reinterpret_cast<uintptr_t>(gb) |
          reinterpret_cast<uintptr_t>(gt) | reinterpret_cast<uintptr_t>(lw) | reinterpret_cast<uintptr_t>(lb)) & 15) == 0) {
        // the prior's width: 16 values per lane loaded as 4 float4 at once (the scalar loop below
        // waits out one load latency per element: 16 us per 36-row call in the DDIM)
        float4 v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = *reinterpret_cast<const float4*>(xr + 4 * lane + 256 * j);
        double s = 0, q = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const double a = v[j].x, b2 = v[j].y, c = v[j].z, d = v[j].w;
            s += (a + b2) + (c + d);
            q += (a * a + b2 * b2) + (c * c + d * d);
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
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int i = 4 * lane + 256 * j;
            const float4 w4 = *reinterpret_cast<const float4*>(lw + i);
            const float4 b4 = *reinterpret_cast<const float4*>(lb + i);
            float h[4] = {(v[j].x - mf) * rstd * w4.x + b4.x, (v[j].y - mf) * rstd * w4.y + b4.y,
                          (v[j].z - mf) * rstd * w4.z + b4.z, (v[j].w - mf) * rstd * w4.w + b4.w};
            if (gb) {
                float4 g4 = *reinterpret_cast<const float4*>(gb + (size_t)row * ld_gb + i);
                float4 e4 = *reinterpret_cast<const float4*>(gb + (size_t)row * ld_gb + Wd + i);
                if (gt) {
                    const float4 tg = *reinterpret_cast<const float4*>(gt + i);
                    const float4 te = *reinterpret_cast<const float4*>(gt + Wd + i);
                    g4.x += tg.x; g4.y += tg.y; g4.z += tg.z; g4.w += tg.w;
                    e4.x += te.x; e4.y += te.y; e4.z += te.z; e4.w += te.w;
                }
                h[0] = h[0] * (1.f + g4.x) + e4.x; h[1] = h[1] * (1.f + g4.y) + e4.y;
                h[2] = h[2] * (1.f + g4.z) + e4.z; h[3] = h[3] * (1.f + g4.w) + e4.w;
            }
            *reinterpret_cast<float4*>(yr + i) = make_float4(h[0], h[1], h[2], h[3]);
        }
        return;
    }
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
            const float g = gb[(size_t)row * ld_gb + i] + (gt ? gt[i] : 0.f);
            const float be = gb[(size_t)row * ld_gb + Wd + i] + (gt ? gt[Wd + i] : 0.f);
            h = h * (1.f + g) + be;
        }
        yr[i] = h;
    }
}

// GroupNorm apply from tables with the output in the h2 split format (h2.hpp): one thread per
// (pixel, 8-channel group) reads 32 B and writes the same 32 B (hi[8], lo[8]), so x == y is safe.
__global__ __launch_bounds__(256) void k_gn_apply_tab_h2(const float* x, char* y, int HW, int C,
                                                         const float* __restrict__ tsc, const float* __restrict__ tsh,
                                                         int silu, int ppb, unsigned* ovf, int bf) {
    extern __shared__ __attribute__((aligned(16))) float lsm[];
    float* sc = lsm;
    float* sh = lsm + ((C + 3) & ~3);
    const int b = blockIdx.y;
    for (int c = threadIdx.x; c < C; c += 256) {
        sc[c] = tsc[(size_t)b * C + c];
        sh[c] = tsh[(size_t)b * C + c];
    }
    __syncthreads();
    const int p0 = blockIdx.x * ppb;
    const int p1 = min(HW, p0 + ppb);
    const size_t base = ((size_t)b * HW + p0) * C;
    const int C8 = C / 8;
    const int n8 = (p1 - p0) * C8;
    bool bad = false;
    // In place (x == y): the compiler must assume each store may alias the next loads, so the
    // loads of GU groups are issued explicitly before any of their stores (each thread's groups
    // are distinct elements) — one group in flight per thread measured 4.85 TB/s.  Software-pipelined:
    // the NEXT batch's loads are issued before this batch's stores, since vmcnt orders loads and
    // stores together (a load issued behind a store cannot be waited for without that store's
    // acknowledgement, which serialised the batches).
    constexpr int GU = 4;
    int i = threadIdx.x;
    float4 n0[GU], n1[GU];
    auto issue = [&](int at) {
#pragma unroll
        for (int k = 0; k < GU; ++k) {
            const float* src = x + base + (size_t)(at + 256 * k) * 8;
            n0[k] = *reinterpret_cast<const float4*>(src);
            n1[k] = *reinterpret_cast<const float4*>(src + 4);
        }
    };
    if (i + (GU - 1) * 256 < n8) issue(i);
    for (; i + (GU - 1) * 256 < n8; i += GU * 256) {
        float4 u0[GU], u1[GU];
#pragma unroll
        for (int k = 0; k < GU; ++k) {
            u0[k] = n0[k];
            u1[k] = n1[k];
        }
        if (i + GU * 256 + (GU - 1) * 256 < n8) issue(i + GU * 256);
#pragma unroll
        for (int k = 0; k < GU; ++k) {
            const int c0 = ((i + 256 * k) % C8) * 8;
            float4 v0 = u0[k], v1 = u1[k];
            v0.x = fmaf(v0.x, sc[c0], sh[c0]); v0.y = fmaf(v0.y, sc[c0 + 1], sh[c0 + 1]);
            v0.z = fmaf(v0.z, sc[c0 + 2], sh[c0 + 2]); v0.w = fmaf(v0.w, sc[c0 + 3], sh[c0 + 3]);
            v1.x = fmaf(v1.x, sc[c0 + 4], sh[c0 + 4]); v1.y = fmaf(v1.y, sc[c0 + 5], sh[c0 + 5]);
            v1.z = fmaf(v1.z, sc[c0 + 6], sh[c0 + 6]); v1.w = fmaf(v1.w, sc[c0 + 7], sh[c0 + 7]);
            if (silu) {
                v0.x = silu_hw(v0.x); v0.y = silu_hw(v0.y); v0.z = silu_hw(v0.z); v0.w = silu_hw(v0.w);
                v1.x = silu_hw(v1.x); v1.y = silu_hw(v1.y); v1.z = silu_hw(v1.z); v1.w = silu_hw(v1.w);
            }
            uint2 h0, l0, h1, l1;
            split4x(v0, h0, l0, bf != 0);
            split4x(v1, h1, l1, bf != 0);
            char* g = y + (base + (size_t)(i + 256 * k) * 8) * 4;
            *reinterpret_cast<uint4*>(g) = make_uint4(h0.x, h0.y, h1.x, h1.y);
            *reinterpret_cast<uint4*>(g + 16) = make_uint4(l0.x, l0.y, l1.x, l1.y);
            bad = bad || h2_bad(v0.x) || h2_bad(v0.y) || h2_bad(v0.z) || h2_bad(v0.w) || h2_bad(v1.x) ||
                  h2_bad(v1.y) || h2_bad(v1.z) || h2_bad(v1.w);
        }
    }
    for (; i < n8; i += 256) {
        const int c0 = (i % C8) * 8;
        const float* src = x + base + (size_t)i * 8;
        float4 v0 = *reinterpret_cast<const float4*>(src);
        float4 v1 = *reinterpret_cast<const float4*>(src + 4);
        v0.x = fmaf(v0.x, sc[c0], sh[c0]); v0.y = fmaf(v0.y, sc[c0 + 1], sh[c0 + 1]);
        v0.z = fmaf(v0.z, sc[c0 + 2], sh[c0 + 2]); v0.w = fmaf(v0.w, sc[c0 + 3], sh[c0 + 3]);
        v1.x = fmaf(v1.x, sc[c0 + 4], sh[c0 + 4]); v1.y = fmaf(v1.y, sc[c0 + 5], sh[c0 + 5]);
        v1.z = fmaf(v1.z, sc[c0 + 6], sh[c0 + 6]); v1.w = fmaf(v1.w, sc[c0 + 7], sh[c0 + 7]);
        if (silu) {
            v0.x = silu_hw(v0.x); v0.y = silu_hw(v0.y); v0.z = silu_hw(v0.z); v0.w = silu_hw(v0.w);
            v1.x = silu_hw(v1.x); v1.y = silu_hw(v1.y); v1.z = silu_hw(v1.z); v1.w = silu_hw(v1.w);
        }
        uint2 h0, l0, h1, l1;
        split4x(v0, h0, l0, bf != 0);
        split4x(v1, h1, l1, bf != 0);
        char* g = y + (base + (size_t)i * 8) * 4;
        *reinterpret_cast<uint4*>(g) = make_uint4(h0.x, h0.y, h1.x, h1.y);
        *reinterpret_cast<uint4*>(g + 16) = make_uint4(l0.x, l0.y, l1.x, l1.y);
        bad = bad || h2_bad(v0.x) || h2_bad(v0.y) || h2_bad(v0.z) || h2_bad(v0.w) || h2_bad(v1.x) || h2_bad(v1.y) ||
              h2_bad(v1.z) || h2_bad(v1.w);
    }
    h2_flag(ovf, bad && !bf);
}

// GroupNorm + SiLU apply from tables into CHUNK-MAJOR h2 records (round 5): y = [C/8][Bt * HW][32 B], one
// plane of records per 8 channels, for the skip tensors h1 / h2 (read by the 4x4/s2 downsample as source 1
// and by the up-path concat conv as source 2: ConvParams::cm1 / cm2).  A pixel-major record source makes the
// downsample's halo DMA fetch 32 B at a stride of C * 4 B (its LDS staging re-fetches every line; DESIGN
// §3l); a plane is contiguous.  Out of place: one workgroup per CM_NR * 256 records (1536 / (C / 8) pixels
// of one image) reads pixel-major (coalesced), transposes the records through LDS and stores each plane's
// run of pixels contiguously.
constexpr int CM_NR = 6;  // records per thread

__global__ __launch_bounds__(256) void k_gn_apply_cm(const float* __restrict__ x, char* __restrict__ y, int HW,
                                                     int C, const float* __restrict__ tsc,
                                                     const float* __restrict__ tsh, unsigned* ovf) {
    extern __shared__ __attribute__((aligned(16))) float lsm[];
    const int C8 = C / 8;
    const int tpx = 256 * CM_NR / C8;  // pixels per workgroup
    const int rs = tpx * 32 + 16;      // LDS bytes per plane row (+16: consecutive planes on other banks)
    float* sc = lsm;
    float* sh = lsm + C;
    char* rec = reinterpret_cast<char*>(lsm + 2 * C);
    const int b = blockIdx.y, tid = threadIdx.x;
    for (int c = tid; c < C; c += 256) {
        sc[c] = tsc[(size_t)b * C + c];
        sh[c] = tsh[(size_t)b * C + c];
    }
    const size_t pix0 = (size_t)b * HW + (size_t)blockIdx.x * tpx;
    const float* src = x + pix0 * C;
    float4 v0[CM_NR], v1[CM_NR];
#pragma unroll
    for (int k = 0; k < CM_NR; ++k) {
        const float* q = src + (size_t)(tid + 256 * k) * 8;
        v0[k] = *reinterpret_cast<const float4*>(q);
        v1[k] = *reinterpret_cast<const float4*>(q + 4);
    }
    __syncthreads();
    bool bad = false;
#pragma unroll
    for (int k = 0; k < CM_NR; ++k) {
        const int idx = tid + 256 * k;
        const int px = idx / C8, c8 = idx - px * C8, c0 = 8 * c8;
        float4 a = v0[k], d = v1[k];
        a.x = silu_hw(fmaf(a.x, sc[c0], sh[c0]));         a.y = silu_hw(fmaf(a.y, sc[c0 + 1], sh[c0 + 1]));
        a.z = silu_hw(fmaf(a.z, sc[c0 + 2], sh[c0 + 2])); a.w = silu_hw(fmaf(a.w, sc[c0 + 3], sh[c0 + 3]));
        d.x = silu_hw(fmaf(d.x, sc[c0 + 4], sh[c0 + 4])); d.y = silu_hw(fmaf(d.y, sc[c0 + 5], sh[c0 + 5]));
        d.z = silu_hw(fmaf(d.z, sc[c0 + 6], sh[c0 + 6])); d.w = silu_hw(fmaf(d.w, sc[c0 + 7], sh[c0 + 7]));
        // the SiLU product rounded to fp32 before the split (as k_gn_apply_tab_h2, whose silu branch keeps
        // it apart): straight-line, hipcc would contract SiLU's last multiply with split1's v - hi
        asm volatile("" : "+v"(a.x), "+v"(a.y), "+v"(a.z), "+v"(a.w), "+v"(d.x), "+v"(d.y), "+v"(d.z), "+v"(d.w));
        uint2 h0, l0, h1, l1;
        split4x(a, h0, l0, false);
        split4x(d, h1, l1, false);
        char* r = rec + c8 * rs + px * 32;
        *reinterpret_cast<uint4*>(r) = make_uint4(h0.x, h0.y, h1.x, h1.y);
        *reinterpret_cast<uint4*>(r + 16) = make_uint4(l0.x, l0.y, l1.x, l1.y);
        bad = bad || h2_bad(a.x) || h2_bad(a.y) || h2_bad(a.z) || h2_bad(a.w) || h2_bad(d.x) || h2_bad(d.y) ||
              h2_bad(d.z) || h2_bad(d.w);
    }
    __syncthreads();
    const size_t npix = (size_t)gridDim.y * HW;  // pixels per plane
#pragma unroll
    for (int k = 0; k < CM_NR; ++k) {
        const int idx = tid + 256 * k;
        const int c8 = idx / tpx, px = idx - c8 * tpx;
        const char* r = rec + c8 * rs + px * 32;
        const uint4 hi = *reinterpret_cast<const uint4*>(r), lo = *reinterpret_cast<const uint4*>(r + 16);
        char* g = y + ((size_t)c8 * npix + pix0 + px) * 32;
        *reinterpret_cast<uint4*>(g) = hi;
        *reinterpret_cast<uint4*>(g + 16) = lo;
    }
    h2_flag(ovf, bad);
}

// The attention block's input side in one pass per image (round 5; sde_score_model.py:130-157 with the
// mid block's last GroupNorm+SiLU): x = silu(GN_mid(a)) is written back in place as the fp32 residual,
// the attn.norm statistics of x are summed (fp64) while x is still in registers, the attn.norm tables
// are formed in the workgroup (gn_tables_from_csum, as tcx_gn_finalize), and GN_attn(x) is written as
// h2 / bf16 records for the qkv conv.  Replaces k_gn_apply_tab + k_gn_partials + k_gn_finalize +
// k_gn_apply_tab_h2 (4 launches, x read 3 times).  One workgroup of 1024 threads per image: thread
// (row, group) holds the 8 channels of group tid % C8 at pixels row, row + R, ... (R = 1024 / C8 rows,
// at most AP_NP pixels each).
constexpr int AP_NP = 8;
__global__ __launch_bounds__(1024) void k_attn_prep(float* __restrict__ a, char* __restrict__ y, int HW, int C,
                                                    const float* __restrict__ tsc, const float* __restrict__ tsh,
                                                    const float* __restrict__ gamma, const float* __restrict__ beta,
                                                    int groups, float eps, unsigned* ovf, int bf) {
    extern __shared__ __attribute__((aligned(16))) double ap[];  // lsum[R][C] | csum[C][2] | gstat[groups][2]
    const int C8 = C / 8, R = 1024 / C8;
    double* lsum = ap;
    double* csum = lsum + (size_t)R * C;
    double* gstat = csum + 2 * C;
    float* sc = reinterpret_cast<float*>(gstat + 2 * groups);
    float* sh = sc + C;
    const int b = blockIdx.x;
    const int tid = threadIdx.x;
    const int g8 = tid % C8, row = tid / C8;
    const bool act = row < R;
    const int c0 = 8 * g8;
    float* ab = a + (size_t)b * HW * C;
    float4 v0[AP_NP], v1[AP_NP];
#pragma unroll
    for (int k = 0; k < AP_NP; ++k) {
        const int p = row + R * k;
        if (act && p < HW) {
            v0[k] = *reinterpret_cast<const float4*>(ab + (size_t)p * C + c0);
            v1[k] = *reinterpret_cast<const float4*>(ab + (size_t)p * C + c0 + 4);
        }
    }
    double s[8], ss[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) s[e] = ss[e] = 0.0;
    if (act) {
        float scl[8], shf[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            scl[e] = tsc[(size_t)b * C + c0 + e];
            shf[e] = tsh[(size_t)b * C + c0 + e];
        }
#pragma unroll
        for (int k = 0; k < AP_NP; ++k) {
            const int p = row + R * k;
            if (p < HW) {
                float4& u = v0[k];
                float4& w = v1[k];
                u.x = silu_f(fmaf(u.x, scl[0], shf[0])); u.y = silu_f(fmaf(u.y, scl[1], shf[1]));
                u.z = silu_f(fmaf(u.z, scl[2], shf[2])); u.w = silu_f(fmaf(u.w, scl[3], shf[3]));
                w.x = silu_f(fmaf(w.x, scl[4], shf[4])); w.y = silu_f(fmaf(w.y, scl[5], shf[5]));
                w.z = silu_f(fmaf(w.z, scl[6], shf[6])); w.w = silu_f(fmaf(w.w, scl[7], shf[7]));
                *reinterpret_cast<float4*>(ab + (size_t)p * C + c0) = u;
                *reinterpret_cast<float4*>(ab + (size_t)p * C + c0 + 4) = w;
                const float e8[8] = {u.x, u.y, u.z, u.w, w.x, w.y, w.z, w.w};
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    s[e] += (double)e8[e];
                    ss[e] += (double)e8[e] * (double)e8[e];
                }
            }
        }
    }
    // channel totals: the R rows of each channel summed in row order, sums then squares
    for (int pass = 0; pass < 2; ++pass) {
        if (act) {
#pragma unroll
            for (int e = 0; e < 8; ++e) lsum[(size_t)row * C + c0 + e] = pass ? ss[e] : s[e];
        }
        __syncthreads();
        for (int c = tid; c < C; c += 1024) {
            double t = 0.0;
            for (int r = 0; r < R; ++r) t += lsum[(size_t)r * C + c];
            csum[2 * c + pass] = t;
        }
        __syncthreads();
    }
    gn_tables_from_csum(C, groups, HW, gamma, beta, eps, sc, sh, gstat, csum);
    bool bad = false;
    if (act) {
        float scl[8], shf[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            scl[e] = sc[c0 + e];
            shf[e] = sh[c0 + e];
        }
        char* yb = y + (size_t)b * HW * C * 4;
#pragma unroll
        for (int k = 0; k < AP_NP; ++k) {
            const int p = row + R * k;
            if (p < HW) {
                float4 u = v0[k], w = v1[k];
                u.x = fmaf(u.x, scl[0], shf[0]); u.y = fmaf(u.y, scl[1], shf[1]);
                u.z = fmaf(u.z, scl[2], shf[2]); u.w = fmaf(u.w, scl[3], shf[3]);
                w.x = fmaf(w.x, scl[4], shf[4]); w.y = fmaf(w.y, scl[5], shf[5]);
                w.z = fmaf(w.z, scl[6], shf[6]); w.w = fmaf(w.w, scl[7], shf[7]);
                uint2 h0, l0, h1, l1;
                split4x(u, h0, l0, bf != 0);
                split4x(w, h1, l1, bf != 0);
                char* g = yb + ((size_t)p * C + c0) * 4;
                *reinterpret_cast<uint4*>(g) = make_uint4(h0.x, h0.y, h1.x, h1.y);
                *reinterpret_cast<uint4*>(g + 16) = make_uint4(l0.x, l0.y, l1.x, l1.y);
                bad = bad || h2_bad(u.x) || h2_bad(u.y) || h2_bad(u.z) || h2_bad(u.w) || h2_bad(w.x) ||
                      h2_bad(w.y) || h2_bad(w.z) || h2_bad(w.w);
            }
        }
    }
    h2_flag(ovf, bad && !bf);
}

// |x| max as the bit pattern of a non-negative float (ordered like the value: an atomicMax on the
// bits is exact and order-independent).  For the power-of-two operand scaling of the training
// path's split convs.
__global__ __launch_bounds__(256) void k_absmax(const float* __restrict__ x, size_t n4, unsigned* __restrict__ bits) {
    __shared__ float red[4];
    float m = 0.f;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    auto take = [&](const float4 v) {
        m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
    };
    for (; i + 3 * stride < n4; i += 4 * stride) {  // four loads in flight per thread
        const float4 v0 = reinterpret_cast<const float4*>(x)[i];
        const float4 v1 = reinterpret_cast<const float4*>(x)[i + stride];
        const float4 v2 = reinterpret_cast<const float4*>(x)[i + 2 * stride];
        const float4 v3 = reinterpret_cast<const float4*>(x)[i + 3 * stride];
        take(v0); take(v1); take(v2); take(v3);
    }
    for (; i < n4; i += stride) take(reinterpret_cast<const float4*>(x)[i]);
    for (int o = 32; o; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) atomicMax(bits, __float_as_uint(fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]))));
}

// the exact power of two s with max|x| * s in [2^13, 2^14) (s = 1 for an all-zero tensor)
__device__ __forceinline__ float pow2_scale(unsigned bits) {
    const float m = __uint_as_float(bits);
    if (!(m > 0.f) || !(m < 3.0e38f)) return 1.f;
    int e;
    frexpf(m, &e);  // m = f * 2^e, f in [0.5, 1)
    return ldexpf(1.f, min(14 - e, 100));
}

// h2(x * s), s from the absmax bits; comb (optional) = *wscale / s: the conv epilogue's factor that
// undoes both the weight scale and this operand scale (all exact powers of two).
__global__ __launch_bounds__(256) void k_f32_to_h2_scaled(const float* __restrict__ x, char* __restrict__ y, size_t n4,
                                                          const unsigned* __restrict__ bits,
                                                          const float* __restrict__ wscale, float* __restrict__ comb) {
    const float s = pow2_scale(*bits);
    if (comb && blockIdx.x == 0 && threadIdx.x == 0) *comb = *wscale / s;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
        float4 v = reinterpret_cast<const float4*>(x)[i];
        v.x *= s; v.y *= s; v.z *= s; v.w *= s;
        store4_h2(y, (i >> 1) * 32, (int)(i & 1), v);
    }
}

__global__ __launch_bounds__(256) void k_f32_to_h2(const float* __restrict__ x, char* __restrict__ y, size_t n4,
                                                   unsigned* ovf) {
    bool bad = false;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
        const float4 v = reinterpret_cast<const float4*>(x)[i];
        store4_h2(y, (i >> 1) * 32, (int)(i & 1), v);
        bad = bad || h2_bad(v.x) || h2_bad(v.y) || h2_bad(v.z) || h2_bad(v.w);
    }
    h2_flag(ovf, bad);
}

__global__ __launch_bounds__(256) void k_h2_to_f32(const char* __restrict__ x, float* __restrict__ y, size_t n4) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x)
        reinterpret_cast<float4*>(y)[i] = load4_h2(x, (i >> 1) * 32, (int)(i & 1));
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
    const int ppb = std::max(1, 65536 / C);  // ~256 KB of activations per block (partials folded once per block)
    const int chunks = cdiv(HW, ppb);
    const size_t shm = gn_fold_lds_bytes(C, groups);
    hipLaunchKernelGGL(k_gn_apply, dim3(chunks, Bt), dim3(256), shm, (hipStream_t)stream, x, y, HW, C, groups, part,
                       nsplit, gamma, beta, eps, silu, ppb);
    return check_launch("tcx_gn_apply");
}

extern "C" int tcx_gn_finalize(const double* part, int Bt, int HW, int C, int groups, int nsplit, const float* gamma,
                               const float* beta, float eps, float* scale, float* shift, void* stream) {
    TCX_REQUIRE(part && scale && shift && groups > 0 && C % groups == 0 && nsplit >= 1, "tcx_gn_finalize: bad args");
    if (Bt == 0) return TCX_OK;
    const size_t shm = gn_finalize_wide_lds_bytes(C, groups);
    hipLaunchKernelGGL(k_gn_finalize, dim3(Bt), dim3(1024), shm, (hipStream_t)stream, part, HW, C, groups, nsplit, gamma,
                       beta, eps, scale, shift);
    return check_launch("tcx_gn_finalize");
}

extern "C" int tcx_gn_apply_tab_absmax(const float* x, float* y, int Bt, int HW, int C, const float* scale,
                                       const float* shift, int silu, unsigned* amax, void* stream) {
    TCX_REQUIRE(x && y && scale && shift && C % 4 == 0 && aligned16(x) && aligned16(y), "tcx_gn_apply_tab: bad args");
    if (Bt == 0) return TCX_OK;
    const int ppb = std::max(1, 32768 / C);  // 128 KB of activations per block
    const dim3 grid(cdiv(HW, ppb), Bt);
    const size_t shm = (size_t)2 * ((C + 3) & ~3) * sizeof(float);
    hipLaunchKernelGGL(k_gn_apply_tab, grid, dim3(256), shm, (hipStream_t)stream, x, y, HW, C, scale, shift, silu, ppb,
                       amax);
    return check_launch("tcx_gn_apply_tab");
}

extern "C" int tcx_gn_apply_tab(const float* x, float* y, int Bt, int HW, int C, const float* scale, const float* shift,
                                int silu, void* stream) {
    return tcx_gn_apply_tab_absmax(x, y, Bt, HW, C, scale, shift, silu, nullptr, stream);
}

extern "C" int tcx_upsample2x(const float* x, float* y, int Bt, int H, int W, int C, const float* scale,
                              const float* shift, void* stream) {
    TCX_REQUIRE(x && y && C % 4 == 0 && aligned16(x) && aligned16(y), "tcx_upsample2x: bad args");
    TCX_REQUIRE((scale == nullptr) == (shift == nullptr), "tcx_upsample2x: scale/shift pair");
    if ((size_t)Bt * H * W * C == 0) return TCX_OK;
    const dim3 grid(Bt * 2 * H, cdiv(2 * W * (C / 4), UPK * 256));
    hipLaunchKernelGGL(k_upsample2x<false>, grid, dim3(256), 0, (hipStream_t)stream, x, y, Bt, H, W, C, scale, shift,
                       nullptr, 0);
    return check_launch("tcx_upsample2x");
}

namespace tcx {
// the banded upsample covers this source shape (its band of source rows fits the LDS)
bool upsample_band_ok(int H, int W, int C) { return H % 2 == 0 && W * C <= UB_MAXWC && C % 8 == 0; }
// source columns per segment of the column-segmented band (0: none fits): the widest power of two
// dividing W whose segment + 2 halo columns fit the LDS band
int upsample_seg_width(int H, int W, int C) {
    if (H % 2 != 0 || C % 8 != 0) return 0;
    for (int sw = 64; sw >= 8; sw /= 2)
        if (W % sw == 0 && sw < W && (sw + 2) * C <= UB_MAXWC) return sw;
    return 0;
}
// the upsample can take the GroupNorm+SiLU tables of its source (band or segmented band)
bool upsample_fused_ok(int H, int W, int C) { return upsample_band_ok(H, W, C) || upsample_seg_width(H, W, C) > 0; }

// h2 (f16x3) or bf16 (bf != 0) records out of the upsample / GroupNorm apply (unet.hip, and the C ABI below)
int upsample2x_h2(const float* x, void* y, int Bt, int H, int W, int C, const float* scale, const float* shift,
                  unsigned* ovf, int bf, hipStream_t st) {
    TCX_REQUIRE(x && y && C % 8 == 0 && aligned16(x) && aligned16(y), "tcx_upsample2x_h2: bad args");
    TCX_REQUIRE((scale == nullptr) == (shift == nullptr), "tcx_upsample2x_h2: scale/shift pair");
    if ((size_t)Bt * H * W * C == 0) return TCX_OK;
    if (upsample_band_ok(H, W, C)) {  // the banded LDS form (the 64^2 U-Net's us1 / us2)
        // 4 output rows per band: 48 KB of LDS, 3 workgroups per CU (r03_n: the 8-row bands and 4-channel
        // items were 3-28 % slower; r05_n: 2-row bands, 36 KB and 4 per CU, 4-7 % slower)
        constexpr int rows = 4;
        const size_t shm = (size_t)(rows / 2 + 2) * W * C * sizeof(float);
        const auto k = &k_upsample2x_band<4, true>;
        static bool attr = false;
        if (!attr) {
            if (hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)(4 * UB_MAXWC * sizeof(float))) != hipSuccess) {
                set_error("tcx_upsample2x_h2: cannot enable %zu B of dynamic LDS", 4 * UB_MAXWC * sizeof(float));
                return TCX_EHIP;
            }
            attr = true;
        }
        hipLaunchKernelGGL(k, dim3(Bt * (2 * H / rows)), dim3(256), shm, st, x, (char*)y, H, W, C, scale, shift, ovf, bf);
        return check_launch("tcx_upsample2x_h2(band)");
    }
    constexpr bool seg_on = true;  // the segmented band form at wide rows (faster than g8, r03; knob removed r04)
    if (const int sw = seg_on ? upsample_seg_width(H, W, C) : 0) {  // config 5's wide rows
        constexpr int rows = 4;
        const size_t shm = (size_t)(rows / 2 + 2) * (sw + 2) * C * sizeof(float);
        const auto k = &k_upsample2x_bandseg<4>;
        static bool attr = false;
        if (!attr) {
            if (hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)(4 * UB_MAXWC * sizeof(float))) != hipSuccess) {
                set_error("tcx_upsample2x_h2: cannot enable %zu B of dynamic LDS", 4 * UB_MAXWC * sizeof(float));
                return TCX_EHIP;
            }
            attr = true;
        }
        hipLaunchKernelGGL(k, dim3(Bt * (2 * H / rows) * (W / sw)), dim3(256), shm, st, x, (char*)y, H, W, C, sw, scale,
                           shift, ovf, bf);
        return check_launch("tcx_upsample2x_h2(segmented band)");
    }
    const dim3 grid(Bt * 2 * H, cdiv(2 * W * (C / 8), UPG * 256));
    hipLaunchKernelGGL(k_upsample2x_g8, grid, dim3(256), 0, st, x, (char*)y, H, W, C, scale, shift, ovf, bf);
    return check_launch("tcx_upsample2x_h2");
}

// Config 5's skip tensors chunk-major (round 6): GroupNorm + SiLU of a 2-byte bf16 (b2) pre-norm conv output
// into CHUNK-MAJOR b2 planes y = [C/8][Bt * HW][16 B] (8 channels x 2 B per pixel per plane), out of place.
// The readers are config 5's 4x4/s2 downsamples (k_conv4s2g's slim slots, source 1) and the up-path concat
// convs (k_conv3lb, source 2): from a pixel-major b2 row (C * 2 = 192 / 384 B per pixel) their halo DMA
// fetched 16 B per pixel and chunk, and the downsample re-read every line 4.6-5.8x from HBM
// (profiles/r05_t_cfg5_pmc_traffic.txt); a plane is contiguous.  One workgroup per CM_NR * 256 16-B
// records (tpx pixels of one image): coalesced pixel-major loads, the same arithmetic as k_gn_apply_b2<true>
// (so the values are bit-identical to the in-place apply), an LDS transpose, contiguous plane stores.
__global__ __launch_bounds__(256) void k_gn_apply_b2cm(const char* __restrict__ x, char* __restrict__ y, int HW,
                                                       int C, const float* __restrict__ tsc,
                                                       const float* __restrict__ tsh) {
    extern __shared__ __attribute__((aligned(16))) float lsm[];
    const int C8 = C / 8;
    const int tpx = 256 * CM_NR / C8;  // pixels per workgroup
    const int rs = tpx * 16 + 16;      // LDS bytes per plane row (+16: consecutive planes on other banks)
    float* sc = lsm;
    float* sh = lsm + C;
    char* rec = reinterpret_cast<char*>(lsm + 2 * C);
    const int b = blockIdx.y, tid = threadIdx.x;
    for (int c = tid; c < C; c += 256) {
        sc[c] = tsc[(size_t)b * C + c];
        sh[c] = tsh[(size_t)b * C + c];
    }
    const size_t pix0 = (size_t)b * HW + (size_t)blockIdx.x * tpx;
    const char* src = x + pix0 * C * 2;
    uint4 u[CM_NR];
#pragma unroll
    for (int k = 0; k < CM_NR; ++k) u[k] = *reinterpret_cast<const uint4*>(src + (size_t)(tid + 256 * k) * 16);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < CM_NR; ++k) {
        const int idx = tid + 256 * k;
        const int px = idx / C8, c8 = idx - px * C8, c0 = 8 * c8;
        const uint4 a = u[k];
        float v[8] = {bf_lo(a.x), bf_hi(a.x), bf_lo(a.y), bf_hi(a.y), bf_lo(a.z), bf_hi(a.z), bf_lo(a.w), bf_hi(a.w)};
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = silu_hw(fmaf(v[e], sc[c0 + e], sh[c0 + e]));
        *reinterpret_cast<uint4*>(rec + c8 * rs + px * 16) =
            make_uint4(pack2_bf(v[0], v[1]), pack2_bf(v[2], v[3]), pack2_bf(v[4], v[5]), pack2_bf(v[6], v[7]));
    }
    __syncthreads();
    const size_t npix = (size_t)gridDim.y * HW;  // pixels per plane
#pragma unroll
    for (int k = 0; k < CM_NR; ++k) {
        const int idx = tid + 256 * k;
        const int c8 = idx / tpx, px = idx - c8 * tpx;
        *reinterpret_cast<uint4*>(y + ((size_t)c8 * npix + pix0 + px) * 16) =
            *reinterpret_cast<const uint4*>(rec + c8 * rs + px * 16);
    }
}


bool gn_apply_cm_ok(int HW, int C) {
    if (C % 8 != 0) return false;
    const int c8 = C / 8;
    return 256 * CM_NR % c8 == 0 && HW % (256 * CM_NR / c8) == 0;
}

int gn_apply_cm(const float* x, void* y, int Bt, int HW, int C, const float* scale, const float* shift,
                unsigned* ovf, hipStream_t st) {
    TCX_REQUIRE(x && y && scale && shift && (const void*)x != y && aligned16(x) && aligned16(y) && gn_apply_cm_ok(HW, C),
                "gn_apply_cm: needs distinct 16-B aligned buffers, C %% 8 == 0 and whole workgroup tiles");
    if (Bt == 0) return TCX_OK;
    const int tpx = 256 * CM_NR / (C / 8);
    const size_t shm = (size_t)2 * C * sizeof(float) + (size_t)(C / 8) * (tpx * 32 + 16);
    hipLaunchKernelGGL(k_gn_apply_cm, dim3(HW / tpx, Bt), dim3(256), shm, st, x, (char*)y, HW, C, scale, shift, ovf);
    return check_launch("gn_apply_cm");
}

int gn_apply_b2cm(const void* x, void* y, int Bt, int HW, int C, const float* scale, const float* shift,
                  hipStream_t st) {
    TCX_REQUIRE(x && y && scale && shift && x != y && aligned16(x) && aligned16(y) && gn_apply_cm_ok(HW, C),
                "gn_apply_b2cm: needs distinct 16-B aligned buffers, C %% 8 == 0 and whole workgroup tiles");
    if (Bt == 0) return TCX_OK;
    const int tpx = 256 * CM_NR / (C / 8);
    const size_t shm = (size_t)2 * C * sizeof(float) + (size_t)(C / 8) * (tpx * 16 + 16);
    hipLaunchKernelGGL(k_gn_apply_b2cm, dim3(HW / tpx, Bt), dim3(256), shm, st, (const char*)x, (char*)y, HW, C, scale,
                       shift);
    return check_launch("gn_apply_b2cm");
}

int gn_apply_tab_h2(const float* x, void* y, int Bt, int HW, int C, const float* scale, const float* shift, int silu,
                    unsigned* ovf, int bf, hipStream_t st) {
    TCX_REQUIRE(x && y && scale && shift && C % 8 == 0 && aligned16(x) && aligned16(y), "tcx_gn_apply_tab_h2: bad args");
    // (the output is 2 B per element for bf == 2: its extent, not the source's, bounds the overlap test)
    const size_t ybytes = (size_t)Bt * HW * C * (bf == 2 ? 2 : 4);
    TCX_REQUIRE((const void*)x == y || (const char*)y + ybytes <= (const char*)x ||
                (const char*)x + (size_t)Bt * HW * C * 4 <= (const char*)y, "tcx_gn_apply_tab_h2: partial overlap");
    if (Bt == 0) return TCX_OK;
    const int ppb = std::max(1, 32768 / C);
    const dim3 grid(cdiv(HW, ppb), Bt);
    const size_t shm = (size_t)2 * ((C + 3) & ~3) * sizeof(float);
    if (bf == 2) {  // fp32 source -> 2-byte bf16 (x == y is not allowed: different sizes)
        TCX_REQUIRE((const void*)x != y, "tcx_gn_apply_tab_h2: an fp32 -> 2-byte apply cannot run in place");
        hipLaunchKernelGGL(k_gn_apply_b2<false>, grid, dim3(256), shm, st, (const char*)x, (char*)y, HW, C, scale, shift,
                           silu, ppb);
        return check_launch("tcx_gn_apply_tab_h2(b2)");
    }
    hipLaunchKernelGGL(k_gn_apply_tab_h2, grid, dim3(256), shm, st, x, (char*)y, HW, C, scale, shift, silu, ppb, ovf,
                       bf);
    return check_launch("tcx_gn_apply_tab_h2");
}

// GroupNorm (+ SiLU) of a 2-byte bf16 tensor in place (config 5: the pre-norm conv outputs are bf16)
int gn_apply_b2_inplace(void* x, int Bt, int HW, int C, const float* scale, const float* shift, int silu,
                        hipStream_t st) {
    TCX_REQUIRE(x && scale && shift && C % 8 == 0 && aligned16(x), "tcx_gn_apply_b2: bad args");
    if (Bt == 0) return TCX_OK;
    const int ppb = std::max(1, 32768 / C);
    const dim3 grid(cdiv(HW, ppb), Bt);
    const size_t shm = (size_t)2 * ((C + 3) & ~3) * sizeof(float);
    hipLaunchKernelGGL(k_gn_apply_b2<true>, grid, dim3(256), shm, st, (const char*)x, (char*)x, HW, C, scale, shift,
                       silu, ppb);
    return check_launch("tcx_gn_apply_b2");
}

// k_attn_prep covers the image: the 8-channel groups fit one 1024-thread workgroup and every thread
// holds at most AP_NP pixels (the 64^2 net's 16^2 x 192 attention input; config 5's 64^2 x 192 does not)
static size_t attn_prep_lds(int C, int groups) {
    const int R = 1024 / (C / 8);
    return ((size_t)R * C + 2 * (size_t)C + 2 * (size_t)groups) * sizeof(double) + 2 * (size_t)C * sizeof(float);
}
bool attn_prep_ok(int HW, int C, int groups, int bf) {
    return bf != 2 && C % 8 == 0 && C / 8 <= 1024 && groups > 0 && C % groups == 0 &&
           HW <= AP_NP * (1024 / (C / 8)) && attn_prep_lds(C, groups) <= 160 * 1024;
}
int attn_prep_h2(float* a, void* y, int Bt, int HW, int C, const float* sc, const float* sh, const float* gamma,
                 const float* beta, int groups, unsigned* ovf, int bf, hipStream_t st) {
    TCX_REQUIRE(a && y && sc && sh && aligned16(a) && aligned16(y) && attn_prep_ok(HW, C, groups, bf),
                "attn_prep_h2: bad args");
    if (Bt == 0) return TCX_OK;
    const size_t shm = attn_prep_lds(C, groups);
    static bool attr = false;
    if (!attr) {
        if (hipFuncSetAttribute(reinterpret_cast<const void*>(&k_attn_prep), hipFuncAttributeMaxDynamicSharedMemorySize,
                                160 * 1024) != hipSuccess) {
            set_error("attn_prep_h2: cannot enable 160 KB of dynamic LDS");
            return TCX_EHIP;
        }
        attr = true;
    }
    hipLaunchKernelGGL(k_attn_prep, dim3(Bt), dim3(1024), shm, st, a, (char*)y, HW, C, sc, sh, gamma, beta, groups,
                       1e-5f, ovf, bf);
    return check_launch("attn_prep_h2");
}
}  // namespace tcx

extern "C" int tcx_upsample2x_h2(const float* x, void* y, int Bt, int H, int W, int C, const float* scale,
                                 const float* shift, unsigned* ovf, void* stream) {
    return upsample2x_h2(x, y, Bt, H, W, C, scale, shift, ovf, 0, (hipStream_t)stream);
}

extern "C" int tcx_upsample2x_bf16(const float* x, void* y, int Bt, int H, int W, int C, const float* scale,
                                   const float* shift, void* stream) {
    return upsample2x_h2(x, y, Bt, H, W, C, scale, shift, nullptr, 1, (hipStream_t)stream);
}

extern "C" int tcx_gn_apply_tab_h2_cm(const float* x, void* y, int Bt, int HW, int C, const float* scale,
                                      const float* shift, unsigned* ovf, void* stream) {
    return gn_apply_cm(x, y, Bt, HW, C, scale, shift, ovf, (hipStream_t)stream);
}

extern "C" int tcx_gn_apply_tab_b2_cm(const void* x, void* y, int Bt, int HW, int C, const float* scale,
                                      const float* shift, void* stream) {
    return gn_apply_b2cm(x, y, Bt, HW, C, scale, shift, (hipStream_t)stream);
}

extern "C" int tcx_gn_apply_tab_h2(const float* x, void* y, int Bt, int HW, int C, const float* scale,
                                   const float* shift, int silu, unsigned* ovf, void* stream) {
    return gn_apply_tab_h2(x, y, Bt, HW, C, scale, shift, silu, ovf, 0, (hipStream_t)stream);
}

extern "C" int tcx_gn_apply_tab_bf16(const float* x, void* y, int Bt, int HW, int C, const float* scale,
                                     const float* shift, int silu, void* stream) {
    return gn_apply_tab_h2(x, y, Bt, HW, C, scale, shift, silu, nullptr, 1, (hipStream_t)stream);
}

extern "C" int tcx_gn_apply_tab_b2(const void* x, void* y, int Bt, int HW, int C, const float* scale,
                                   const float* shift, int silu, int in_b2, void* stream) {
    if (in_b2) {
        TCX_REQUIRE(x == y, "tcx_gn_apply_tab_b2: a 2-byte source is normalised in place");
        return gn_apply_b2_inplace(y, Bt, HW, C, scale, shift, silu, (hipStream_t)stream);
    }
    return gn_apply_tab_h2(static_cast<const float*>(x), y, Bt, HW, C, scale, shift, silu, nullptr, 2, (hipStream_t)stream);
}

extern "C" int tcx_upsample2x_b2(const float* x, void* y, int Bt, int H, int W, int C, const float* scale,
                                 const float* shift, void* stream) {
    return upsample2x_h2(x, y, Bt, H, W, C, scale, shift, nullptr, 2, (hipStream_t)stream);
}

extern "C" int tcx_f32_to_h2(const float* x, void* y, size_t n, unsigned* ovf, void* stream) {
    TCX_REQUIRE(x && y && n % 8 == 0 && aligned16(x) && aligned16(y), "tcx_f32_to_h2: n %% 8 and 16-B alignment");
    if (n == 0) return TCX_OK;
    const int blocks = (int)std::min<size_t>((n / 4 + 255) / 256, 8192);
    hipLaunchKernelGGL(k_f32_to_h2, dim3(blocks), dim3(256), 0, (hipStream_t)stream, x, (char*)y, n / 4, ovf);
    return check_launch("tcx_f32_to_h2");
}

extern "C" int tcx_h2_to_f32(const void* x, float* y, size_t n, void* stream) {
    TCX_REQUIRE(x && y && n % 8 == 0 && aligned16(x) && aligned16(y), "tcx_h2_to_f32: n %% 8 and 16-B alignment");
    if (n == 0) return TCX_OK;
    const int blocks = (int)std::min<size_t>((n / 4 + 255) / 256, 8192);
    hipLaunchKernelGGL(k_h2_to_f32, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const char*)x, y, n / 4);
    return check_launch("tcx_h2_to_f32");
}

namespace tcx {
int launch_layernorm_film(const float* x, float* y, int M, int Wd, const float* lw, const float* lb, const float* gb,
                          int ld_gb, const float* gt, float eps, hipStream_t st) {
    TCX_REQUIRE(x && y && lw && lb && M >= 0 && Wd > 0 && (!gt || gb), "layernorm_film: bad args");
    if (M == 0) return TCX_OK;
    hipLaunchKernelGGL(k_layernorm_film, dim3(cdiv(M, 4)), dim3(256), 0, st, x, y, M, Wd, lw, lb, gb, ld_gb, gt, eps);
    return check_launch("tcx_layernorm_film");
}
}  // namespace tcx

extern "C" int tcx_layernorm_film(const float* x, float* y, int M, int Wd, const float* ln_w, const float* ln_b,
                                  const float* gb, int ld_gb, float eps, void* stream) {
    TCX_REQUIRE(x && y && ln_w && ln_b && M >= 0 && Wd > 0, "tcx_layernorm_film: bad args");
    if (M == 0) return TCX_OK;
    return launch_layernorm_film(x, y, M, Wd, ln_w, ln_b, gb, ld_gb, nullptr, eps, (hipStream_t)stream);
}

extern "C" int tcx_absmax(const float* x, size_t n, unsigned* bits, void* stream) {
    TCX_REQUIRE(x && bits && n % 4 == 0 && aligned16(x), "tcx_absmax: n %% 4 and 16-B alignment");
    if (n == 0) return TCX_OK;
    const int blocks = (int)std::min<size_t>((n / 4 + 1023) / 1024, 2048);
    hipLaunchKernelGGL(k_absmax, dim3(blocks), dim3(256), 0, (hipStream_t)stream, x, n / 4, bits);
    return check_launch("tcx_absmax");
}

extern "C" int tcx_f32_to_h2_scaled(const float* x, void* y, size_t n, const unsigned* absmax_bits,
                                    const float* wscale, float* comb, void* stream) {
    TCX_REQUIRE(x && y && absmax_bits && n % 8 == 0 && aligned16(x) && aligned16(y) && (!comb || wscale),
                "tcx_f32_to_h2_scaled: bad args");
    if (n == 0) return TCX_OK;
    const int blocks = (int)std::min<size_t>((n / 4 + 255) / 256, 8192);
    hipLaunchKernelGGL(k_f32_to_h2_scaled, dim3(blocks), dim3(256), 0, (hipStream_t)stream, x, (char*)y, n / 4,
                       absmax_bits, wscale, comb);
    return check_launch("tcx_f32_to_h2_scaled");
}
