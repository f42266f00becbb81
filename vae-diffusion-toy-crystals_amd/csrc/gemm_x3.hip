// f16x3 GEMM for the Linear layers of the training path (gfx950, v_mfma_f32_32x32x16_f16).
//
// C = act(alpha A B^T (+ beta C) + bias[n] + resid[m][n]) for the three GEMMs of every large nn.Linear
// of the DiffusionPriorFiLM training step (/root/reference/src/toycrystals/models/diffusion_prior.py:
// 39-55, trained by /root/reference/scripts/train_diffusion_prior.py:240-277):
//   forward  y  = x W^T    A = h2 rows of x,   B = W  (fp32, k contiguous)
//   dgrad    dx = dy W     A = h2 rows of dy,  B = W  (fp32, n contiguous)
//   wgrad    dW = dy^T x   A = h2 rows of dy^T, B = h2 rows of x^T
//
// Operand formats.  "h2 rows" (h2.hpp records): [R][K/8][8 hi | 8 lo] f16, row r scaled by an exact
// power of two s_r chosen from the row's own max |v| (scaled max in [2^14, 2^15): no f16 overflow,
// 22 significant bits for every element within 2^-17 of the row max), inv[r] = 1 / s_r.  Written by
// tcx_h2_rows (x [R][K]) and tcx_h2_cols (the transpose of x [R][C]) in one pass each: the activation
// operands are small (batch rows), so they are split ONCE instead of once per output tile.  A scale per
// row of either operand factors out of the dot product: acc * inv_a[m] * inv_b[n] in the epilogue.
// The weight operand stays fp32 and is split in the LDS staging (each element once per 128-row M tile,
// i.e. once or twice per GEMM), scaled by the tensor's power of two (max |W| from tcx_absmax_multi).
//
// Products hi*lo + lo*hi + hi*hi on three MFMAs, fp32 accumulation: ~2^-22 relative per product, 16x
// the fp32-MFMA rate per instruction (5.3x per fp32-equivalent FLOP).
//
// Tile 128 x 128, 4 waves of 64 x 64 (2 x 2 MFMA tiles, 64 accumulator AGPRs), LDS images of 128 rows
// x 128 B per operand, double buffered (64 KB: two workgroups per CU), global loads X3_PF chunks ahead
// in registers.  The 16-B unit u (k group u >> 1, hi / lo u & 1) of row r sits at u ^ ((r >> 1) & 7): a
// ds_read_b128 lane group (16 rows of one k group) covers 16 distinct 16-B bank slots.  When the
// output tiles cannot fill the chip the reduction is split (grid.y) into raw partials [split][M][N],
// folded in a fixed order by k_x3_reduce with the epilogue (deterministic).
#include "common.hpp"
#include "h2.hpp"

#include <algorithm>
#include <type_traits>
#include <utility>

namespace tcx {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int XT = 128;          // tile rows of either operand
constexpr int XK = 32;           // reduction depth per chunk
constexpr int XROW = 128;        // LDS bytes per tile row: 4 k groups x (hi 16 B + lo 16 B)
constexpr int XIMG = XT * XROW;  // one operand image (16 KB)
constexpr int X3_PF = 4;         // register stages of the global-load pipeline

template <typename F, int... Is>
__device__ __forceinline__ void static_for(F&& f, std::integer_sequence<int, Is...>) {
    (f(std::integral_constant<int, Is>{}), ...);
}

struct X3Params {
    int M, N, K;
    float alpha, beta;
    const char* A;       // h2 rows [M][K]
    const float* inva;   // [M]
    const char* Bh;      // h2 rows [N][K] (LB 2)
    const float* invb;   // [N] (LB 2)
    const float* B;      // fp32 (LB 0 / 1): B(n, k) at B[n sbn + k sbk]
    long long sbk, sbn;
    const unsigned* amax_b;  // LB 0 / 1: max |B| as float bits
    float* C;
    long long ldc;
    const float* bias;   // [N]
    const float* resid;  // [M] rows of stride ldr
    long long ldr;
    int act;             // 0 none, 1 relu, 2 sigmoid, 3 silu
    float* part;         // split-K partials [nsplit][M][N] (null: epilogue in the GEMM)
    int nsplit, kcs;     // splits, chunks per split
    int nnblk;
};

// exponent of the power-of-two scale: max|v| in [2^e, 2^(e+1)) -> scaled max in [2^14, 2^15)
__device__ __forceinline__ int x3_exp_bits(unsigned bits) {
    bits &= 0x7fffffffu;
    if (bits == 0u) return 0;
    return 14 - max((int)(bits >> 23) - 127, -100);
}

__device__ __forceinline__ float x3_epi(const X3Params& p, float v, int m, int n, const float* cp) {
    v *= p.alpha;
    if (p.beta != 0.f) v += p.beta * *cp;
    if (p.bias) v += p.bias[n];
    if (p.resid) v += p.resid[(size_t)m * p.ldr + n];
    if (p.act == 1) v = fmaxf(v, 0.f);
    else if (p.act == 2) v = 1.f / (1.f + expf(-v));
    else if (p.act == 3) v = silu_f(v);
    return v;
}

__device__ __forceinline__ void split8(const float* v, float s, uint4& hi, uint4& lo) {
    unsigned w[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = split1(v[i] * s);
    hi = make_uint4((w[0] & 0xffffu) | (w[1] << 16), (w[2] & 0xffffu) | (w[3] << 16), (w[4] & 0xffffu) | (w[5] << 16),
                    (w[6] & 0xffffu) | (w[7] << 16));
    lo = make_uint4((w[0] >> 16) | (w[1] & 0xffff0000u), (w[2] >> 16) | (w[3] & 0xffff0000u),
                    (w[4] >> 16) | (w[5] & 0xffff0000u), (w[6] >> 16) | (w[7] & 0xffff0000u));
}

__device__ __forceinline__ int x3_unit(int r, int u) { return r * XROW + ((u ^ ((r >> 1) & 7)) << 4); }

// One operand tile: rows [r0, r0 + 128) x k [k0, k0 + 32), 4 x 16 B per thread.
// L = 2: h2 rows (piece P = tid + 256 i: row P >> 3, 16-B piece P & 7 of the row's 128-B chunk slice,
//        copied as is); L = 0: fp32, k contiguous (rows (tid >> 2) + 64 i, k group tid & 3); L = 1: fp32,
//        rows contiguous (rows 4 (tid & 31) .. +3, k = 4 (tid >> 5) .. +3).  Rows past R and k past K
//        load zeros.
template <int L>
struct X3Stage {
    static constexpr int NV = L == 2 ? 4 : 16;
    uint4 u[L == 2 ? 4 : 1];
    float v[L == 2 ? 1 : 16];
    __device__ __forceinline__ void load_h2(const char* X, int R, int K, int r0, int k0, int tid) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int P = tid + 256 * i, r = r0 + (P >> 3), pc = P & 7;
            const int k = k0 + 8 * (pc >> 1);
            u[i] = make_uint4(0u, 0u, 0u, 0u);
            if (r < R && k < K) u[i] = *reinterpret_cast<const uint4*>(X + ((size_t)r * K + k) * 4 + (pc & 1) * 16);
        }
    }
    __device__ __forceinline__ void load_f32(const float* X, int sr, int sk, int R, int K, int r0, int k0, int tid) {
        if constexpr (L == 0) {
            const int g = tid & 3;
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int r = r0 + (tid >> 2) + 64 * i;
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const int k = k0 + 8 * g + 4 * h;
                    float4 f = make_float4(0.f, 0.f, 0.f, 0.f);
                    if (r < R && k < K) f = *reinterpret_cast<const float4*>(X + (r * sr + k));
                    v[8 * i + 4 * h] = f.x; v[8 * i + 4 * h + 1] = f.y; v[8 * i + 4 * h + 2] = f.z;
                    v[8 * i + 4 * h + 3] = f.w;
                }
            }
        } else if constexpr (L == 1) {
            const int r = r0 + 4 * (tid & 31), kq = tid >> 5;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int k = k0 + 4 * kq + j;
                float4 f = make_float4(0.f, 0.f, 0.f, 0.f);
                if (r < R && k < K) f = *reinterpret_cast<const float4*>(X + (r + k * sk));
                v[4 * j] = f.x; v[4 * j + 1] = f.y; v[4 * j + 2] = f.z; v[4 * j + 3] = f.w;
            }
        }
    }
    __device__ __forceinline__ void store(char* img, float s, int tid) const {
        if constexpr (L == 2) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int P = tid + 256 * i;
                *reinterpret_cast<uint4*>(img + x3_unit(P >> 3, P & 7)) = u[i];
            }
        } else if constexpr (L == 0) {
            const int g = tid & 3;
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int r = (tid >> 2) + 64 * i;
                uint4 hi, lo;
                split8(v + 8 * i, s, hi, lo);
                *reinterpret_cast<uint4*>(img + x3_unit(r, 2 * g)) = hi;
                *reinterpret_cast<uint4*>(img + x3_unit(r, 2 * g + 1)) = lo;
            }
        } else {
            const int kq = tid >> 5, g = kq >> 1, half = (kq & 1) * 8;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int r = 4 * (tid & 31) + e;
                unsigned w[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) w[j] = split1(v[4 * j + e] * s);
                const uint2 hi = make_uint2((w[0] & 0xffffu) | (w[1] << 16), (w[2] & 0xffffu) | (w[3] << 16));
                const uint2 lo = make_uint2((w[0] >> 16) | (w[1] & 0xffff0000u), (w[2] >> 16) | (w[3] & 0xffff0000u));
                *reinterpret_cast<uint2*>(img + x3_unit(r, 2 * g) + half) = hi;
                *reinterpret_cast<uint2*>(img + x3_unit(r, 2 * g + 1) + half) = lo;
            }
        }
    }
};

template <int LB>
__global__ __launch_bounds__(256, 1) void k_gemm_x3(X3Params p) {
    mfma_agpr_form();
    __shared__ __attribute__((aligned(16))) char lds[2 * 2 * XIMG];  // [buf][A | B]
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, li = lane & 31, lh = lane >> 5;
    const int tile = xcd_remap(blockIdx.x, gridDim.x);
    const int mblk = tile / p.nnblk, nblk = tile - mblk * p.nnblk;
    const int m0 = mblk * XT, n0 = nblk * XT;
    const int split = blockIdx.y;
    const int nch_all = (p.K + XK - 1) / XK;
    const int c0 = split * p.kcs, c1 = min(c0 + p.kcs, nch_all);
    const int eb = LB == 2 ? 0 : x3_exp_bits(*p.amax_b);
    const float sb = __builtin_ldexpf(1.f, eb);

    // PF register stages: chunk i is loaded PF iterations before it is consumed (stage (i - c0) % PF),
    // stored to LDS buffer (i - c0) & 1 at the end of iteration i - 1; PF - 1 iterations of MFMA cover
    // each load's latency (one stage ahead left it exposed: r04_y, ~30 us per fc1-sized GEMM)
    X3Stage<2> sta[X3_PF];
    X3Stage<LB> stb[X3_PF];
    auto load = [&](int c, auto Q) {
        constexpr int q = decltype(Q)::value;
        sta[q].load_h2(p.A, p.M, p.K, m0, c * XK, tid);
        if constexpr (LB == 2) stb[q].load_h2(p.Bh, p.N, p.K, n0, c * XK, tid);
        else stb[q].load_f32(p.B, (int)p.sbn, (int)p.sbk, p.N, p.K, n0, c * XK, tid);
    };
    auto store = [&](int buf, auto Q) {
        constexpr int q = decltype(Q)::value;
        sta[q].store(lds + buf * 2 * XIMG, 1.f, tid);
        stb[q].store(lds + buf * 2 * XIMG + XIMG, sb, tid);
    };

    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = (f32x16){};
    const int wm = wv >> 1, wn = wv & 1;
    // this lane's fragment units for k step s: group 2 s + lh, hi unit 2 g, lo unit 2 g + 1, swizzled
    // by the row (rows wm / wn 64 + 32 i + li share (li >> 1) & 7)
    const int sw = (li >> 1) & 7;
    int uo[2][2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        const int g = 2 * s + lh;
        uo[s][0] = ((2 * g) ^ sw) << 4;
        uo[s][1] = ((2 * g + 1) ^ sw) << 4;
    }
    auto compute = [&](int cur) {
        const char* ia = lds + cur * 2 * XIMG;
        const char* ib = ia + XIMG;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            h8 ah[2], al[2], bh[2], bl[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int ra = (wm * 64 + 32 * i + li) * XROW, rb = (wn * 64 + 32 * i + li) * XROW;
                ah[i] = *reinterpret_cast<const h8*>(ia + ra + uo[s][0]);
                al[i] = *reinterpret_cast<const h8*>(ia + ra + uo[s][1]);
                bh[i] = *reinterpret_cast<const h8*>(ib + rb + uo[s][0]);
                bl[i] = *reinterpret_cast<const h8*>(ib + rb + uo[s][1]);
            }
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bl[j], acc[i][j], 0, 0, 0);
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[i], bh[j], acc[i][j], 0, 0, 0);
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bh[j], acc[i][j], 0, 0, 0);
        }
    };
    // raw barrier: LDS traffic drained (lgkmcnt 0), the global loads of later chunks left in flight —
    // __syncthreads() would also wait for vmcnt(0), i.e. for every prefetch issued this iteration
    auto barrier = [&]() {
        asm volatile("" ::: "memory");       // no LDS access moves across (the intrinsics are IntrNoMem)
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    };
    static_for([&](auto Q) {
        if (c0 + decltype(Q)::value < c1) load(c0 + decltype(Q)::value, Q);
    }, std::make_integer_sequence<int, X3_PF>{});
    if (c0 < c1) store(0, std::integral_constant<int, 0>{});
    barrier();
    for (int base = c0; base < c1; base += X3_PF) {
        static_for([&](auto Q) {
            constexpr int q = decltype(Q)::value;
            const int i = base + q;
            if (i < c1) {
                if (i + X3_PF < c1) load(i + X3_PF, Q);
                compute((i - c0) & 1);
                if (i + 1 < c1) store((i + 1 - c0) & 1, std::integral_constant<int, (q + 1) % X3_PF>{});
                barrier();
            }
        }, std::make_integer_sequence<int, X3_PF>{});
    }
    // Epilogue: every load (row / column scales, bias, residual, beta C) is issued before the first
    // store — vmcnt counts loads and stores in one order, so a load behind a store would wait for that
    // store's acknowledgement (the first form loaded inv_a[m] per element between the stores: ~30 us per
    // GEMM of serialised round trips, r04_za)
    const float ib_t = __builtin_ldexpf(1.f, -eb);
    float* P = p.part ? p.part + (size_t)split * p.M * p.N : nullptr;
    float sa_r[2][16], sb_c[2], bias_c[2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int m = m0 + wm * 64 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lh;
            sa_r[i][r] = p.inva[m < p.M ? m : p.M - 1];
        }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int n = min(n0 + wn * 64 + 32 * j + li, p.N - 1);
        sb_c[j] = LB == 2 ? p.invb[n] : ib_t;
        bias_c[j] = (!P && p.bias) ? p.bias[n] : 0.f;
    }
    const bool extra = !P && (p.resid || p.beta != 0.f);
    if (extra) {  // residual / beta C of all 64 outputs, into the accumulators' scaled values
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int m = min(m0 + wm * 64 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lh, p.M - 1);
                    const int n = min(n0 + wn * 64 + 32 * j + li, p.N - 1);
                    float add = 0.f;
                    if (p.resid) add = p.resid[(size_t)m * p.ldr + n];
                    if (p.beta != 0.f) add += p.beta * p.C[(size_t)m * p.ldc + n];
                    acc[i][j][r] = fmaf(p.alpha, acc[i][j][r] * sa_r[i][r] * sb_c[j], add);
                }
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int n = n0 + wn * 64 + 32 * j + li;
        if (n >= p.N) continue;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = m0 + wm * 64 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lh;
                if (m >= p.M) continue;
                if (P) {
                    P[(size_t)m * p.N + n] = acc[i][j][r] * sa_r[i][r] * sb_c[j];
                } else {
                    float v = extra ? acc[i][j][r] : p.alpha * (acc[i][j][r] * sa_r[i][r] * sb_c[j]);
                    v += bias_c[j];
                    if (p.act == 1) v = fmaxf(v, 0.f);
                    else if (p.act == 2) v = 1.f / (1.f + expf(-v));
                    else if (p.act == 3) v = silu_f(v);
                    p.C[(size_t)m * p.ldc + n] = v;
                }
            }
        }
    }
}

// C = epilogue(sum_s part[s]) in a fixed split order
__global__ __launch_bounds__(256) void k_x3_reduce(X3Params p) {
    const size_t MN = (size_t)p.M * p.N;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < MN; i += (size_t)gridDim.x * blockDim.x) {
        float v = 0.f;
        for (int s = 0; s < p.nsplit; ++s) v += p.part[(size_t)s * MN + i];
        const int m = (int)(i / p.N), n = (int)(i - (size_t)m * p.N);
        float* cp = p.C + (size_t)m * p.ldc + n;
        *cp = x3_epi(p, v, m, n, cp);
    }
}

// h2 rows of x [R][K] (row stride ldx), one wave per row: the row max, its scale, the split records
__global__ __launch_bounds__(256) void k_h2_rows(const float* __restrict__ x, int R, int K, long long ldx, char* out,
                                                 float* inv) {
    const int lane = threadIdx.x & 63;
    const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= R) return;
    const float* xr = x + (size_t)r * ldx;
    float m = 0.f;
    for (int k = 4 * lane; k < K; k += 256) m = fmaxf(m, absmax4(*reinterpret_cast<const float4*>(xr + k)));
    for (int o = 32; o; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    const int e = x3_exp_bits(__float_as_uint(m));
    const float s = __builtin_ldexpf(1.f, e);
    if (lane == 0) inv[r] = __builtin_ldexpf(1.f, -e);
    char* orow = out + (size_t)r * K * 4;
    for (int k = 8 * lane; k < K; k += 512) {
        float v[8];
        const float4 a = *reinterpret_cast<const float4*>(xr + k), b = *reinterpret_cast<const float4*>(xr + k + 4);
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
        uint4 hi, lo;
        split8(v, s, hi, lo);
        *reinterpret_cast<uint4*>(orow + (size_t)k * 4) = hi;
        *reinterpret_cast<uint4*>(orow + (size_t)k * 4 + 16) = lo;
    }
}

// h2 rows of x^T for x [R][C] (row stride ldx): output row c = column c of x (R values, R % 8 == 0),
// scaled by the column's max.  One workgroup per 16 columns (thread: column tid & 15, row group
// tid >> 4): pass 1 the column maxima, pass 2 (L2-hot) the records, 8 rows of one column per unit.
__global__ __launch_bounds__(256) void k_h2_cols(const float* __restrict__ x, int R, int C, long long ldx, char* out,
                                                 float* inv) {
    __shared__ float cm[16][17];
    const int cl = threadIdx.x & 15, q = threadIdx.x >> 4;
    const int c = blockIdx.x * 16 + cl;
    const bool cv = c < C;
    float m = 0.f;
    if (cv)
        for (int r = q; r < R; r += 16) m = fmaxf(m, fabsf(x[(size_t)r * ldx + c]));
    cm[q][cl] = m;
    __syncthreads();
    m = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) m = fmaxf(m, cm[i][cl]);
    const int e = x3_exp_bits(__float_as_uint(m));
    const float s = __builtin_ldexpf(1.f, e);
    if (!cv) return;
    if (q == 0) inv[c] = __builtin_ldexpf(1.f, -e);
    char* orow = out + (size_t)c * R * 4;
    for (int g = q; g < R / 8; g += 16) {
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = x[(size_t)(8 * g + j) * ldx + c];
        uint4 hi, lo;
        split8(v, s, hi, lo);
        *reinterpret_cast<uint4*>(orow + (size_t)g * 32) = hi;
        *reinterpret_cast<uint4*>(orow + (size_t)g * 32 + 16) = lo;
    }
}

// max |x| of up to 32 tensors in one launch: grid.y = tensor, grid.x strides over its float4s
struct AbsTable {
    const float* x[32];
    unsigned long long n4[32];
};

__global__ __launch_bounds__(256) void k_absmax_multi(AbsTable t, unsigned* bits) {
    const int w = blockIdx.y;
    const float4* x = reinterpret_cast<const float4*>(t.x[w]);
    const size_t n4 = t.n4[w];
    float m = 0.f;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    for (; i + 3 * stride < n4; i += 4 * stride) {
        const float4 v0 = x[i], v1 = x[i + stride], v2 = x[i + 2 * stride], v3 = x[i + 3 * stride];
        m = fmaxf(m, fmaxf(fmaxf(absmax4(v0), absmax4(v1)), fmaxf(absmax4(v2), absmax4(v3))));
    }
    for (; i < n4; i += stride) m = fmaxf(m, absmax4(x[i]));
    block_amax_publish(m, bits + w);
}

// split the reduction when the output tiles cannot fill the chip: ~256 workgroups, >= 4 chunks each
void x3_plan(int M, int N, int K, int* nsplit, int* kcs) {
    const int tiles = cdiv(M, XT) * cdiv(N, XT);
    const int nch = cdiv(K, XK);
    *nsplit = 1;
    *kcs = nch;
    if (tiles >= 192 || nch < 8) return;
    int s = std::min(cdiv(256, tiles), nch / 4);
    if (s < 2) return;
    *kcs = cdiv(nch, s);
    *nsplit = cdiv(nch, *kcs);
}

bool off32(double v) { return v < 2147483648.0; }

}  // namespace
}  // namespace tcx

using namespace tcx;

extern "C" int tcx_h2_rows(const float* x, int R, int K, long long ldx, void* out, float* inv, void* stream) {
    TCX_REQUIRE(x && out && inv && R >= 0 && K > 0 && K % 8 == 0 && ldx >= K && ldx % 4 == 0 && aligned16(x) &&
                    aligned16(out),
                "tcx_h2_rows: K %% 8, 16-B aligned rows");
    if (R == 0) return TCX_OK;
    hipLaunchKernelGGL(k_h2_rows, dim3(cdiv(R, 4)), dim3(256), 0, (hipStream_t)stream, x, R, K, ldx,
                       static_cast<char*>(out), inv);
    return check_launch("tcx_h2_rows");
}

extern "C" int tcx_h2_cols(const float* x, int R, int C, long long ldx, void* out, float* inv, void* stream) {
    TCX_REQUIRE(x && out && inv && R > 0 && R % 8 == 0 && C >= 0 && ldx >= C && aligned16(out),
                "tcx_h2_cols: R %% 8");
    if (C == 0) return TCX_OK;
    hipLaunchKernelGGL(k_h2_cols, dim3(cdiv(C, 16)), dim3(256), 0, (hipStream_t)stream, x, R, C, ldx,
                       static_cast<char*>(out), inv);
    return check_launch("tcx_h2_cols");
}

extern "C" int tcx_absmax_multi(const float* const* xs, const size_t* ns, int count, unsigned* bits, void* stream) {
    TCX_REQUIRE(xs && ns && bits && count >= 0 && count <= 32, "tcx_absmax_multi: at most 32 tensors");
    if (count == 0) return TCX_OK;
    hipStream_t st = (hipStream_t)stream;
    AbsTable t{};
    size_t mx = 0;
    for (int i = 0; i < count; ++i) {
        TCX_REQUIRE(xs[i] && ns[i] % 4 == 0 && aligned16(xs[i]), "tcx_absmax_multi: tensor %d: n %% 4, 16-B alignment",
                    i);
        t.x[i] = xs[i];
        t.n4[i] = ns[i] / 4;
        mx = std::max(mx, ns[i] / 4);
    }
    TCX_REQUIRE(hipMemsetAsync(bits, 0, (size_t)count * sizeof(unsigned), st) == hipSuccess, "tcx_absmax_multi: memset");
    const int gx = (int)std::max<size_t>(1, std::min<size_t>((mx + 1023) / 1024, 256));
    hipLaunchKernelGGL(k_absmax_multi, dim3(gx, count), dim3(256), 0, st, t, bits);
    return check_launch("tcx_absmax_multi");
}

extern "C" size_t tcx_gemm_x3_workspace(int M, int N, int K) {
    if (M <= 0 || N <= 0 || K <= 0) return 0;
    int ns, kcs;
    x3_plan(M, N, K, &ns, &kcs);
    return ns > 1 ? (size_t)ns * M * N * sizeof(float) : 0;
}

extern "C" int tcx_gemm_x3_ok(int M, int N, int K, const float* B, long long sb_k, long long sb_n, int b_h2) {
    if (M <= 0 || N <= 0 || K <= 0 || K % 8 != 0) return 0;
    if (!off32((double)M * N) || !off32((double)M * K) || !off32((double)N * K)) return 0;
    if (b_h2) return 1;
    if (!aligned16(B) || !off32((double)(N - 1) * sb_n + (double)(K - 1) * sb_k + 1)) return 0;
    return (sb_k == 1 && sb_n % 4 == 0) || (sb_n == 1 && N % 4 == 0 && sb_k % 4 == 0);
}

extern "C" int tcx_gemm_x3(int M, int N, int K, float alpha, const void* A, const float* inva, const void* B,
                           long long sb_k, long long sb_n, const float* invb, const unsigned* amax_b, float beta,
                           float* C, long long ldc, const float* bias, const float* resid, long long ld_resid, int act,
                           void* ws, size_t ws_bytes, void* stream) {
    TCX_REQUIRE(A && inva && B && C && aligned16(A) && aligned16(B) && ldc >= N, "tcx_gemm_x3: bad pointers");
    TCX_REQUIRE(tcx_gemm_x3_ok(M, N, K, static_cast<const float*>(B), sb_k, sb_n, invb != nullptr),
                "tcx_gemm_x3: operands not stageable (M %d N %d K %d, B strides %lld %lld)", M, N, K, sb_k, sb_n);
    TCX_REQUIRE(invb || amax_b, "tcx_gemm_x3: an fp32 B needs its max |B| word");
    TCX_REQUIRE(act >= 0 && act <= 3 && (!resid || ld_resid >= N) && off32((double)(M - 1) * ldc + N),
                "tcx_gemm_x3: bad epilogue");
    hipStream_t st = (hipStream_t)stream;
    X3Params p{};
    p.M = M; p.N = N; p.K = K; p.alpha = alpha; p.beta = beta;
    p.A = static_cast<const char*>(A); p.inva = inva;
    if (invb) {
        p.Bh = static_cast<const char*>(B); p.invb = invb;
    } else {
        p.B = static_cast<const float*>(B); p.sbk = sb_k; p.sbn = sb_n; p.amax_b = amax_b;
    }
    p.C = C; p.ldc = ldc; p.bias = bias; p.resid = resid; p.ldr = ld_resid; p.act = act;
    p.nnblk = cdiv(N, XT);
    int ns, kcs;
    x3_plan(M, N, K, &ns, &kcs);
    p.nsplit = 1;
    p.kcs = cdiv(K, XK);
    if (ns > 1) {
        TCX_REQUIRE(ws && ws_bytes >= (size_t)ns * M * N * sizeof(float), "tcx_gemm_x3: workspace %zu < %zu bytes",
                    ws_bytes, (size_t)ns * M * N * sizeof(float));
        p.part = static_cast<float*>(ws);
        p.nsplit = ns;
        p.kcs = kcs;
    }
    const dim3 grid(cdiv(M, XT) * p.nnblk, p.nsplit);
    if (invb) hipLaunchKernelGGL(k_gemm_x3<2>, grid, dim3(256), 0, st, p);
    else if (sb_k == 1) hipLaunchKernelGGL(k_gemm_x3<0>, grid, dim3(256), 0, st, p);
    else hipLaunchKernelGGL(k_gemm_x3<1>, grid, dim3(256), 0, st, p);
    TCX_TRY(check_launch("tcx_gemm_x3"));
    if (!p.part) return TCX_OK;
    const size_t n_all = (size_t)M * N;
    hipLaunchKernelGGL(k_x3_reduce, dim3((unsigned)std::min<size_t>((n_all + 255) / 256, 4096)), dim3(256), 0, st, p);
    return check_launch("tcx_gemm_x3 reduce");
}
