// fp32-MFMA GEMMs for the training path (gfx950, v_mfma_f32_32x32x2_f32).
//
// k_gemm   — batched, arbitrarily strided C = alpha * op(A) op(B) + beta * C (+ bias[n]).  Serves
//            the Linear layers forward and backward of every model (dX = dY W, dW = dY^T X) and the
//            attention products (S = Q K^T, O = P V and their backward) of SelfAttention2d
//            (/root/reference/src/toycrystals/models/sde_score_model.py:150-157).
// k_wgrad  — convolution weight gradient dW[co][ci][ky][kx] = sum_m dY[m][co] * im2col(X)[m][k]
//            (the backward of every nn.Conv2d / nn.ConvTranspose2d of sde_score_model.py and
//            models/vae.py), an implicit GEMM whose reduction runs over output pixels: split over
//            pixel ranges into [split][K][Cout] partials, then a fixed-order reduction (deterministic).
//
// Both use the conv kernel's tile scheme: 128 x 32*NT output tile, 4 waves x (32 rows x 32*NT),
// 32-deep reduction chunks staged through LDS rows padded to 36 floats, register-staged double
// buffering.  Operands whose reduction dimension is not the contiguous one are loaded as float4
// along the contiguous dimension and transposed on the LDS store.
#include "common.hpp"
#include "skinny.hpp"
#include "h2.hpp"
#include "thin.hpp"

namespace tcx {
struct Wg3hArgs {
    const char* x1;
    const char* x2;
    const char* dy;
    unsigned bx1, bx2, bdy;
    int B, H, W, C1, C2, Cin, Cout, circular;
    int RB;
    int nchunk, cps;
    int ncob;
    const float* comb;
    float* part;
};
// wgrad3h.hip: the halo-staged 3x3 weight gradient
bool wgrad3h_takes(int B, int H, int W, int C1, int C2, int Cout, int ks, int stride, int pad, size_t in1, size_t in2,
                   size_t ind);
int launch_wgrad3h(Wg3hArgs& a, int max_split, int* nsplit, hipStream_t st);
}  // namespace tcx

namespace tcx {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int GBM = 128;
constexpr int GBK = 32;
constexpr int GLD = 36;

struct GemmParams {
    int M, N, K;
    float alpha, beta;
    const float* A;
    long long sam, sak;
    const float* B;
    long long sbk, sbn;
    float* C;
    long long scm, scn;
    const float* bias;
    int bdiv;  // batch z -> (z / bdiv, z % bdiv) offsets
    long long sah, sal, sbh, sbl, sch, scl;
    int nmblk, nnblk;
    // split-K (tcx_gemm_ws): part != null -> grid.y = batch * nsplit, split s reduces chunks
    // [s*kcs, (s+1)*kcs) into part[s][z][M][N] (raw sums); k_gemm_reduce applies alpha/beta/bias
    float* part;
    int nsplit, kcs;
    // reduce-only extras (tcx_linear_ws): residual [M][N] (row stride N) and activation
    const float* resid;
    int act;
};

__device__ __forceinline__ float4 ld4g(const float* p) { return *reinterpret_cast<const float4*>(p); }

// LA / LB: 0 = float4 along the reduction dim, 1 = float4 along the row (M or N) dim, 2 = scalar
template <int NT, int LA, int LB>
__global__ __launch_bounds__(256, 2) void k_gemm(GemmParams p) {
    constexpr int BN = 32 * NT;
    __shared__ __attribute__((aligned(16))) float As[2][GBM * GLD];
    __shared__ __attribute__((aligned(16))) float Bs[2][BN * GLD];
    const int zz = blockIdx.y;
    const int z = p.part ? zz / p.nsplit : zz;
    const int sk = p.part ? zz - z * p.nsplit : 0;
    const int zh = z / p.bdiv, zl = z - zh * p.bdiv;
    const float* A = p.A + zh * p.sah + zl * p.sal;
    const float* B = p.B + zh * p.sbh + zl * p.sbl;
    float* C = p.C + zh * p.sch + zl * p.scl;
    const int tile = xcd_remap(blockIdx.x, gridDim.x);
    const int mblk = tile / p.nnblk, nblk = tile - (tile / p.nnblk) * p.nnblk;
    const int m0 = mblk * GBM, n0 = nblk * BN;
    const int tid = threadIdx.x;

    float ra[16];
    float rb[4 * NT];
    auto load = [&](int k0) {
        // A tile: 128 rows x 32 k
        if constexpr (LA == 0) {
            const int k4 = tid & 7, pr = tid >> 3;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int m = m0 + pr + 32 * i, k = k0 + 4 * k4;
                float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
                if (m < p.M && k < p.K) v = ld4g(A + m * p.sam + k);
                ra[4 * i] = v.x; ra[4 * i + 1] = v.y; ra[4 * i + 2] = v.z; ra[4 * i + 3] = v.w;
            }
        } else if constexpr (LA == 1) {
            const int kk = tid & 31, q = tid >> 5;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int m = m0 + 4 * (q + 8 * i), k = k0 + kk;
                float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
                if (m < p.M && k < p.K) v = ld4g(A + m + k * p.sak);
                ra[4 * i] = v.x; ra[4 * i + 1] = v.y; ra[4 * i + 2] = v.z; ra[4 * i + 3] = v.w;
            }
        } else {
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int e = tid + 256 * i, m = m0 + (e >> 5), k = k0 + (e & 31);
                ra[i] = (m < p.M && k < p.K) ? A[m * p.sam + k * p.sak] : 0.f;
            }
        }
        // B tile: BN rows (n) x 32 k
        if constexpr (LB == 0) {
            const int k4 = tid & 7, pr = tid >> 3;
#pragma unroll
            for (int j = 0; j < NT; ++j) {
                const int n = n0 + pr + 32 * j, k = k0 + 4 * k4;
                float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
                if (n < p.N && k < p.K) v = ld4g(B + n * p.sbn + k);
                rb[4 * j] = v.x; rb[4 * j + 1] = v.y; rb[4 * j + 2] = v.z; rb[4 * j + 3] = v.w;
            }
        } else if constexpr (LB == 1) {
            const int kk = tid & 31, q = tid >> 5;
#pragma unroll
            for (int j = 0; j < NT; ++j) {
                const int n = n0 + 4 * (q + 8 * j), k = k0 + kk;
                float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
                if (n < p.N && k < p.K) v = ld4g(B + n + k * p.sbk);
                rb[4 * j] = v.x; rb[4 * j + 1] = v.y; rb[4 * j + 2] = v.z; rb[4 * j + 3] = v.w;
            }
        } else {
#pragma unroll
            for (int j = 0; j < 4 * NT; ++j) {
                const int e = tid + 256 * j, n = n0 + (e >> 5), k = k0 + (e & 31);
                rb[j] = (n < p.N && k < p.K) ? B[n * p.sbn + k * p.sbk] : 0.f;
            }
        }
    };
    auto store = [&](int buf) {
        if constexpr (LA == 0) {
            const int k4 = tid & 7, pr = tid >> 3;
#pragma unroll
            for (int i = 0; i < 4; ++i)
                *reinterpret_cast<float4*>(&As[buf][(pr + 32 * i) * GLD + 4 * k4]) =
                    make_float4(ra[4 * i], ra[4 * i + 1], ra[4 * i + 2], ra[4 * i + 3]);
        } else if constexpr (LA == 1) {
            const int kk = tid & 31, q = tid >> 5;
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int e = 0; e < 4; ++e) As[buf][(4 * (q + 8 * i) + e) * GLD + kk] = ra[4 * i + e];
        } else {
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int e = tid + 256 * i;
                As[buf][(e >> 5) * GLD + (e & 31)] = ra[i];
            }
        }
        if constexpr (LB == 0) {
            const int k4 = tid & 7, pr = tid >> 3;
#pragma unroll
            for (int j = 0; j < NT; ++j)
                *reinterpret_cast<float4*>(&Bs[buf][(pr + 32 * j) * GLD + 4 * k4]) =
                    make_float4(rb[4 * j], rb[4 * j + 1], rb[4 * j + 2], rb[4 * j + 3]);
        } else if constexpr (LB == 1) {
            const int kk = tid & 31, q = tid >> 5;
#pragma unroll
            for (int j = 0; j < NT; ++j)
#pragma unroll
                for (int e = 0; e < 4; ++e) Bs[buf][(4 * (q + 8 * j) + e) * GLD + kk] = rb[4 * j + e];
        } else {
#pragma unroll
            for (int j = 0; j < 4 * NT; ++j) {
                const int e = tid + 256 * j;
                Bs[buf][(e >> 5) * GLD + (e & 31)] = rb[j];
            }
        }
    };

    f32x16 acc[NT];
#pragma unroll
    for (int n = 0; n < NT; ++n) acc[n] = (f32x16){};
    const int lane = tid & 63, wv = tid >> 6, li = lane & 31, lh = lane >> 5;
    const int nch_all = (p.K + GBK - 1) / GBK;
    const int cb = p.part ? sk * p.kcs : 0;
    const int nch = p.part ? min(p.kcs, nch_all - cb) : nch_all;
    // raw barrier per chunk: LDS drained (lgkmcnt 0) but the next chunk's global loads left in flight
    // (__syncthreads() also waits for vmcnt(0): the prefetch was then exposed every chunk)
    auto barrier = [&]() {
        asm volatile("" ::: "memory");       // no LDS access moves across (the intrinsics are IntrNoMem)
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    };
    load(cb * GBK);
    store(0);
    barrier();
    for (int c = 0; c < nch; ++c) {
        const int cur = c & 1;
        if (c + 1 < nch) load((cb + c + 1) * GBK);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const float4 fa = *reinterpret_cast<const float4*>(&As[cur][(wv * 32 + li) * GLD + lh * 16 + g * 4]);
            float4 fb[NT];
#pragma unroll
            for (int n = 0; n < NT; ++n)
                fb[n] = *reinterpret_cast<const float4*>(&Bs[cur][(n * 32 + li) * GLD + lh * 16 + g * 4]);
#pragma unroll
            for (int n = 0; n < NT; ++n) acc[n] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa.x, fb[n].x, acc[n], 0, 0, 0);
#pragma unroll
            for (int n = 0; n < NT; ++n) acc[n] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa.y, fb[n].y, acc[n], 0, 0, 0);
#pragma unroll
            for (int n = 0; n < NT; ++n) acc[n] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa.z, fb[n].z, acc[n], 0, 0, 0);
#pragma unroll
            for (int n = 0; n < NT; ++n) acc[n] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa.w, fb[n].w, acc[n], 0, 0, 0);
        }
        if (c + 1 < nch) store(cur ^ 1);
        barrier();
    }
    if (p.part) {  // raw partial sums of this K split, dense [M][N]
        float* P = p.part + ((size_t)sk * gridDim.y / p.nsplit + z) * (size_t)p.M * p.N;
#pragma unroll
        for (int n = 0; n < NT; ++n) {
            const int col = n0 + n * 32 + li;
            if (col >= p.N) continue;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = m0 + wv * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
                if (row < p.M) P[(size_t)row * p.N + col] = acc[n][r];
            }
        }
        return;
    }
    // every load (bias, beta C) before the first store: vmcnt orders loads and stores together, so a load
    // behind a store waits for the store's acknowledgement (the old per-element C read between the
    // stores serialised the epilogue of the beta = 1 residual linears)
    float bv[NT];
#pragma unroll
    for (int n = 0; n < NT; ++n) {
        const int col = min(n0 + n * 32 + li, p.N - 1);
        bv[n] = p.bias ? p.bias[col] : 0.f;
    }
    if (p.beta != 0.f) {
#pragma unroll
        for (int n = 0; n < NT; ++n) {
            const int col = min(n0 + n * 32 + li, p.N - 1);
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = min(m0 + wv * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh, p.M - 1);
                acc[n][r] = p.alpha * acc[n][r] + p.beta * C[row * p.scm + col * p.scn];
            }
        }
    } else {
#pragma unroll
        for (int n = 0; n < NT; ++n)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[n][r] = p.alpha * acc[n][r];
    }
#pragma unroll
    for (int n = 0; n < NT; ++n) {
        const int col = n0 + n * 32 + li;
        if (col >= p.N) continue;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int row = m0 + wv * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
            if (row < p.M) C[row * p.scm + col * p.scn] = acc[n][r] + bv[n];
        }
    }
}

// C[z][m][n] = alpha * sum_s part[s][z][m][n] (fixed order) + beta * C + bias[n]
__global__ __launch_bounds__(256) void k_gemm_reduce(GemmParams p, int batch) {
    const size_t MN = (size_t)p.M * p.N;
    const size_t n_all = MN * batch;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n_all; i += (size_t)gridDim.x * blockDim.x) {
        const int z = (int)(i / MN);
        const size_t e = i - (size_t)z * MN;
        const int row = (int)(e / p.N), col = (int)(e - (size_t)row * p.N);
        float v = 0.f;
        for (int s = 0; s < p.nsplit; ++s) v += p.part[((size_t)s * batch + z) * MN + e];
        const int zh = z / p.bdiv, zl = z - zh * p.bdiv;
        float* cp = p.C + zh * p.sch + zl * p.scl + row * p.scm + col * p.scn;
        float o = p.alpha * v;
        if (p.beta != 0.f) o += p.beta * *cp;
        o += p.bias ? p.bias[col] : 0.f;
        if (p.resid) o += p.resid[(size_t)row * p.N + col];
        if (p.act == 1) o = fmaxf(o, 0.f);
        else if (p.act == 2) o = 1.f / (1.f + expf(-o));
        else if (p.act == 3) o = silu_f(o);
        *cp = o;
    }
}

template <int NT>
int launch_gemm_nt(const GemmParams& p, int la, int lb, int batch, hipStream_t st) {
    const dim3 grid(p.nmblk * p.nnblk, batch * (p.part ? p.nsplit : 1));
#define TCX_G(A_, B_) hipLaunchKernelGGL((k_gemm<NT, A_, B_>), grid, dim3(256), 0, st, p)
    if (la == 0 && lb == 0) TCX_G(0, 0);
    else if (la == 0 && lb == 1) TCX_G(0, 1);
    else if (la == 0) TCX_G(0, 2);
    else if (la == 1 && lb == 0) TCX_G(1, 0);
    else if (la == 1 && lb == 1) TCX_G(1, 1);
    else if (la == 1) TCX_G(1, 2);
    else if (lb == 0) TCX_G(2, 0);
    else if (lb == 1) TCX_G(2, 1);
    else TCX_G(2, 2);
#undef TCX_G
    return check_launch("tcx_gemm");
}

// ---------------------------------------------------------------- conv weight gradient
struct WgParams {
    const float *x1, *x2;
    int C1, C2, Cin, H, W, Ho, Wo, HoWo, M;
    int ks, stride, pad, circular;
    const float* dy;
    int Cout, K;
    float* part;  // [nsplit][K][Cout]
    int nsplit, cps;  // splits, 32-pixel chunks per split
    int nkblk, ncblk;
    const float* comb;  // k_wgrad_h2: 1 / (s_x s_dy), the operands' power-of-two scales
    unsigned bx1, bx2, bdy;  // k_wgrad_h2: byte extents of x1, x2, dy (raw-buffer loads, zero past the end)
};

// ASC: scalar im2col gather (Cin % 4 != 0); BSC: scalar dY loads (Cout % 4 != 0)
template <int NT, bool ASC, bool BSC>
__global__ __launch_bounds__(256, 2) void k_wgrad(WgParams p) {
    constexpr int BN = 32 * NT;
    __shared__ __attribute__((aligned(16))) float As[2][GBM * GLD];  // [k row][pixel]
    __shared__ __attribute__((aligned(16))) float Bs[2][BN * GLD];   // [co row][pixel]
    const int split = blockIdx.y;
    const int tile = xcd_remap(blockIdx.x, gridDim.x);
    const int kblk = tile / p.ncblk, cblk = tile - (tile / p.ncblk) * p.ncblk;
    const int k0 = kblk * GBM, c0 = cblk * BN;
    const int tid = threadIdx.x;
    const int px = tid & 31, q = tid >> 5;  // pixel column, quad row group
    const int chunk0 = split * p.cps;
    const int nch_all = (p.M + 31) / 32;
    const int chunk1 = min(chunk0 + p.cps, nch_all);

    // per-thread im2col rows: 4 quads of 4 k each (k = k0 + 4 (q + 8 i) + e)
    int tdy[16], tdx[16], tci[16];
    bool tsrc1[16], tkv[16];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int k = k0 + 4 * (q + 8 * i) + e;
            const int kk = k < p.K ? k : 0;
            const int tap = kk / p.Cin, ci = kk - (kk / p.Cin) * p.Cin;
            tdy[4 * i + e] = tap / p.ks;
            tdx[4 * i + e] = tap - (tap / p.ks) * p.ks;
            tsrc1[4 * i + e] = ci < p.C1;
            tci[4 * i + e] = ci < p.C1 ? ci : ci - p.C1;
            tkv[4 * i + e] = k < p.K;
        }
    float ra[16];
    float rb[4 * NT];
    auto load = [&](int c) {
        const int m = c * 32 + px;
        const bool mv = m < p.M;
        const int mm = mv ? m : 0;
        const int b = mm / p.HoWo, r = mm - (mm / p.HoWo) * p.HoWo;
        const int oy = r / p.Wo, ox = r - (r / p.Wo) * p.Wo;
        const int iy0 = oy * p.stride - p.pad, ix0 = ox * p.stride - p.pad;
        auto addr = [&](int j, bool& ok) -> const float* {
            int yy = iy0 + tdy[j], xx = ix0 + tdx[j];
            ok = mv && tkv[j];
            if (p.circular) {
                yy = wrap_idx(yy, p.H);
                xx = wrap_idx(xx, p.W);
            } else {
                ok = ok && yy >= 0 && yy < p.H && xx >= 0 && xx < p.W;
            }
            const size_t pix = ((size_t)b * p.H + (ok ? yy : 0)) * p.W + (ok ? xx : 0);
            return tsrc1[j] ? p.x1 + pix * p.C1 + tci[j] : p.x2 + pix * p.C2 + tci[j];
        };
        if constexpr (!ASC) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                bool ok;
                const float* a = addr(4 * i, ok);
                float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
                if (ok) v = ld4g(a);
                ra[4 * i] = v.x; ra[4 * i + 1] = v.y; ra[4 * i + 2] = v.z; ra[4 * i + 3] = v.w;
            }
        } else {
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                bool ok;
                const float* a = addr(j, ok);
                ra[j] = ok ? *a : 0.f;
            }
        }
#pragma unroll
        for (int j = 0; j < NT; ++j) {
            const int co = c0 + 4 * (q + 8 * j);
            if constexpr (!BSC) {
                float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
                if (mv && co < p.Cout) v = ld4g(p.dy + (size_t)m * p.Cout + co);
                rb[4 * j] = v.x; rb[4 * j + 1] = v.y; rb[4 * j + 2] = v.z; rb[4 * j + 3] = v.w;
            } else {
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    rb[4 * j + e] = (mv && co + e < p.Cout) ? p.dy[(size_t)m * p.Cout + co + e] : 0.f;
            }
        }
    };
    auto store = [&](int buf) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int e = 0; e < 4; ++e) As[buf][(4 * (q + 8 * i) + e) * GLD + px] = ra[4 * i + e];
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) Bs[buf][(4 * (q + 8 * j) + e) * GLD + px] = rb[4 * j + e];
    };

    f32x16 acc[NT];
#pragma unroll
    for (int n = 0; n < NT; ++n) acc[n] = (f32x16){};
    const int lane = tid & 63, wv = tid >> 6, li = lane & 31, lh = lane >> 5;
    if (chunk0 < chunk1) {
        load(chunk0);
        store(0);
    }
    __syncthreads();
    for (int c = chunk0; c < chunk1; ++c) {
        const int cur = (c - chunk0) & 1;
        if (c + 1 < chunk1) load(c + 1);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const float4 fa = *reinterpret_cast<const float4*>(&As[cur][(wv * 32 + li) * GLD + lh * 16 + g * 4]);
            float4 fb[NT];
#pragma unroll
            for (int n = 0; n < NT; ++n)
                fb[n] = *reinterpret_cast<const float4*>(&Bs[cur][(n * 32 + li) * GLD + lh * 16 + g * 4]);
#pragma unroll
            for (int n = 0; n < NT; ++n) acc[n] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa.x, fb[n].x, acc[n], 0, 0, 0);
#pragma unroll
            for (int n = 0; n < NT; ++n) acc[n] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa.y, fb[n].y, acc[n], 0, 0, 0);
#pragma unroll
            for (int n = 0; n < NT; ++n) acc[n] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa.z, fb[n].z, acc[n], 0, 0, 0);
#pragma unroll
            for (int n = 0; n < NT; ++n) acc[n] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa.w, fb[n].w, acc[n], 0, 0, 0);
        }
        if (c + 1 < chunk1) store(cur ^ 1);
        __syncthreads();
    }
    float* dst = p.part + (size_t)split * p.K * p.Cout;
#pragma unroll
    for (int n = 0; n < NT; ++n) {
        const int co = c0 + n * 32 + li;
        if (co >= p.Cout) continue;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int k = k0 + wv * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
            if (k < p.K) dst[(size_t)k * p.Cout + co] = acc[n][r];
        }
    }
}

// f16x3 weight gradient: the im2col source x and dY arrive as h2 records (h2.hpp) scaled by exact
// powers of two (functional.py: tcx_absmax + tcx_f32_to_h2_scaled); both are transposed through LDS
// as f16 hi / lo planes [row][32 pixels] and each 16-pixel step is three v_mfma_f32_32x32x16_f16
// (hi*lo, lo*hi, hi*hi) instead of eight fp32 ones.  Same tiling, split plan and fixed-order reduce as
// k_wgrad; the partials are acc * comb.  Needs C1, C2, Cout % 8 == 0 (whole 4-channel quads of a record).
template <int NT>
__global__ __launch_bounds__(256, 2) void k_wgrad_h2_r2(WgParams p) {
    constexpr int BN = 32 * NT;
    constexpr int RS = 40;  // halves per LDS row: 32 pixels + 8 pad (80 B)
    __shared__ __attribute__((aligned(16))) _Float16 Ah[2][GBM * RS];
    __shared__ __attribute__((aligned(16))) _Float16 Al[2][GBM * RS];
    __shared__ __attribute__((aligned(16))) _Float16 Bh[2][BN * RS];
    __shared__ __attribute__((aligned(16))) _Float16 Bl[2][BN * RS];
    const int split = blockIdx.y;
    const int tile = xcd_remap(blockIdx.x, gridDim.x);
    const int kblk = tile / p.ncblk, cblk = tile - (tile / p.ncblk) * p.ncblk;
    const int k0 = kblk * GBM, c0 = cblk * BN;
    const int tid = threadIdx.x;
    const int px = tid & 31, q = tid >> 5;
    const int chunk0 = split * p.cps;
    const int nch_all = (p.M + 31) / 32;
    const int chunk1 = min(chunk0 + p.cps, nch_all);
    const char* x1 = reinterpret_cast<const char*>(p.x1);
    const char* x2 = reinterpret_cast<const char*>(p.x2);
    const char* dyb = reinterpret_cast<const char*>(p.dy);
    // per-thread im2col quads: k = k0 + 4 (q + 8 i) .. +3 share one tap and source (C1, C2 % 8 == 0)
    int tdy[4], tdx[4], toff[4];
    bool tsrc1[4], tkv[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int k = k0 + 4 * (q + 8 * i);
        const int kk = k < p.K ? k : 0;
        const int tap = kk / p.Cin, ci = kk - (kk / p.Cin) * p.Cin;
        tdy[i] = tap / p.ks;
        tdx[i] = tap - (tap / p.ks) * p.ks;
        tsrc1[i] = ci < p.C1;
        const int c = ci < p.C1 ? ci : ci - p.C1;
        toff[i] = (c >> 3) * 32 + (c & 4) * 2;  // byte offset of the quad's hi half in the pixel record
        tkv[i] = k < p.K;
    }
    uint2 ah[4], al[4], bh[NT], bl[NT];
    auto load = [&](int c) {
        const int m = c * 32 + px;
        const bool mv = m < p.M;
        const int mm = mv ? m : 0;
        const int b = mm / p.HoWo, r = mm - (mm / p.HoWo) * p.HoWo;
        const int oy = r / p.Wo, ox = r - (r / p.Wo) * p.Wo;
        const int iy0 = oy * p.stride - p.pad, ix0 = ox * p.stride - p.pad;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            int yy = iy0 + tdy[i], xx = ix0 + tdx[i];
            bool ok = mv && tkv[i];
            if (p.circular) {
                yy = wrap_idx(yy, p.H);
                xx = wrap_idx(xx, p.W);
            } else {
                ok = ok && yy >= 0 && yy < p.H && xx >= 0 && xx < p.W;
            }
            const size_t pix = ((size_t)b * p.H + (ok ? yy : 0)) * p.W + (ok ? xx : 0);
            const char* a = tsrc1[i] ? x1 + pix * p.C1 * 4 + toff[i] : x2 + pix * p.C2 * 4 + toff[i];
            ah[i] = ok ? *reinterpret_cast<const uint2*>(a) : make_uint2(0u, 0u);
            al[i] = ok ? *reinterpret_cast<const uint2*>(a + 16) : make_uint2(0u, 0u);
        }
#pragma unroll
        for (int j = 0; j < NT; ++j) {
            const int co = c0 + 4 * (q + 8 * j);
            const bool ok = mv && co < p.Cout;
            const char* d = dyb + ((size_t)mm * p.Cout + (co >> 3) * 8) * 4 + (co & 4) * 2;
            bh[j] = ok ? *reinterpret_cast<const uint2*>(d) : make_uint2(0u, 0u);
            bl[j] = ok ? *reinterpret_cast<const uint2*>(d + 16) : make_uint2(0u, 0u);
        }
    };
    auto put4 = [&](_Float16* plane, int row0, const uint2 v) {  // 4 consecutive rows, this pixel
        plane[(row0 + 0) * RS + px] = __builtin_bit_cast(_Float16, (unsigned short)(v.x & 0xffffu));
        plane[(row0 + 1) * RS + px] = __builtin_bit_cast(_Float16, (unsigned short)(v.x >> 16));
        plane[(row0 + 2) * RS + px] = __builtin_bit_cast(_Float16, (unsigned short)(v.y & 0xffffu));
        plane[(row0 + 3) * RS + px] = __builtin_bit_cast(_Float16, (unsigned short)(v.y >> 16));
    };
    auto store = [&](int buf) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            put4(Ah[buf], 4 * (q + 8 * i), ah[i]);
            put4(Al[buf], 4 * (q + 8 * i), al[i]);
        }
#pragma unroll
        for (int j = 0; j < NT; ++j) {
            put4(Bh[buf], 4 * (q + 8 * j), bh[j]);
            put4(Bl[buf], 4 * (q + 8 * j), bl[j]);
        }
    };
    f32x16 acc[NT];
#pragma unroll
    for (int n = 0; n < NT; ++n) acc[n] = (f32x16){};
    const int lane = tid & 63, wv = tid >> 6, li = lane & 31, lh = lane >> 5;
    if (chunk0 < chunk1) {
        load(chunk0);
        store(0);
    }
    __syncthreads();
    for (int c = chunk0; c < chunk1; ++c) {
        const int cur = (c - chunk0) & 1;
        if (c + 1 < chunk1) load(c + 1);
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            const int off = 16 * s + 8 * lh;
            const h8 fah = *reinterpret_cast<const h8*>(&Ah[cur][(wv * 32 + li) * RS + off]);
            const h8 fal = *reinterpret_cast<const h8*>(&Al[cur][(wv * 32 + li) * RS + off]);
            h8 fbh[NT], fbl[NT];
#pragma unroll
            for (int n = 0; n < NT; ++n) {
                fbh[n] = *reinterpret_cast<const h8*>(&Bh[cur][(n * 32 + li) * RS + off]);
                fbl[n] = *reinterpret_cast<const h8*>(&Bl[cur][(n * 32 + li) * RS + off]);
            }
#pragma unroll
            for (int n = 0; n < NT; ++n) acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fah, fbl[n], acc[n], 0, 0, 0);
#pragma unroll
            for (int n = 0; n < NT; ++n) acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fal, fbh[n], acc[n], 0, 0, 0);
#pragma unroll
            for (int n = 0; n < NT; ++n) acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fah, fbh[n], acc[n], 0, 0, 0);
        }
        if (c + 1 < chunk1) store(cur ^ 1);
        __syncthreads();
    }
    const float sc = *p.comb;
    float* dst = p.part + (size_t)split * p.K * p.Cout;
#pragma unroll
    for (int n = 0; n < NT; ++n) {
        const int co = c0 + n * 32 + li;
        if (co >= p.Cout) continue;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int k = k0 + wv * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
            if (k < p.K) dst[(size_t)k * p.Cout + co] = acc[n][r] * sc;
        }
    }
}

// f16x3 weight gradient, round 3: same tiles, split plan, partials and fixed-order reduce as
// k_wgrad_h2_r2 above, with the operands staged as whole 16-B record pieces and transposed by the LDS
// read instead of the store.  PMC of the round-2 kernel on the score step (profiles/r03_aa_*): TD
// (vector-memory return path) busy 88 %, MFMA busy 14 %, 315 M L1 accesses per launch — its 8-byte
// quad loads touch one cache line per lane — and 56 2-byte LDS stores per thread per chunk.
// Here a thread loads 16-B pieces (the hi or lo half of one 8-channel group of one pixel's record:
// 32 consecutive lanes read 512 contiguous bytes), stores each with ONE ds_write_b128 into a
// [pixel][hi plane 16 pieces | lo plane 16 pieces] image (512-B rows, piece o of row r at o ^ 4 (r & 3)),
// and the MFMA operands (k or co on the lane, 8 consecutive pixels) come from ds_read_b64_tr_b16:
// lane 4q + p of a 16-lane group addresses pixel row q, columns 4p .. 4p + 3 and receives one column
// of the 4 rows.  A 32-lane half reads 4 rows x 4 pieces of one plane; the swizzle puts those 16
// pieces on 16 distinct 16-B bank groups (row stride 512 B = 0 mod 256).
template <int NT>
__global__ __launch_bounds__(256, 2) void k_wgrad_h2(WgParams p) {
    constexpr int BN = 32 * NT;
    constexpr int ROWB = 512;                 // bytes per pixel row of either image
    constexpr int AB = 32 * ROWB;             // A image: 32 pixels x 128 k (hi | lo planes)
    constexpr int BB = 32 * ROWB;             // B image: 32 pixels x BN co (4 NT of 16 pieces used)
    constexpr int STG = AB + BB;
    constexpr int OB = 4 * NT;                // co octets per plane
    extern __shared__ __attribute__((aligned(16))) char wsm[];
    const int split = blockIdx.y;
    const int tile = xcd_remap(blockIdx.x, gridDim.x);
    const int kblk = tile / p.ncblk, cblk = tile - (tile / p.ncblk) * p.ncblk;
    const int k0 = kblk * GBM, c0 = cblk * BN;
    const int tid = threadIdx.x;
    const int chunk0 = split * p.cps;
    const int nch_all = (p.M + 31) / 32;
    const int chunk1 = min(chunk0 + p.cps, nch_all);
    const __amdgpu_buffer_rsrc_t r1 = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.x1), 0, (int)p.bx1, 0x00020000);
    const __amdgpu_buffer_rsrc_t r2 =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.x2 ? p.x2 : p.x1), 0, (int)(p.x2 ? p.bx2 : p.bx1), 0x00020000);
    const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.dy), 0, (int)p.bdy, 0x00020000);
    constexpr int OOB = (int)0x80000000u;

    // A pieces of this thread: idx = tid + 256 i -> pixel row tid / 32 + 8 i, logical piece lp = tid % 32
    // (plane lp / 16, octet lp % 16: k = k0 + 8 octet, one tap and one source per octet)
    const int lp = tid & 31, apl = lp >> 4, aoc = lp & 15;
    const int ak = k0 + 8 * aoc;
    const bool akv = ak < p.K;
    const int akk = akv ? ak : 0;
    const int atap = akk / p.Cin, aci = akk - (akk / p.Cin) * p.Cin;
    const int ady = atap / p.ks, adx = atap - (atap / p.ks) * p.ks;
    const bool asrc1 = aci < p.C1;
    const int aC = asrc1 ? p.C1 : p.C2;
    const int aoff = (asrc1 ? aci : aci - p.C1) * 4 + 16 * apl;  // byte offset within the pixel record
    float4 ra[4], rb[NT];
    auto load = [&](int c) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int row = (tid >> 5) + 8 * i;
            const int m = c * 32 + row;
            const bool mv = m < p.M;
            const int mm = mv ? m : 0;
            const int b = mm / p.HoWo, r = mm - (mm / p.HoWo) * p.HoWo;
            const int oy = r / p.Wo, ox = r - (r / p.Wo) * p.Wo;
            int yy = oy * p.stride - p.pad + ady, xx = ox * p.stride - p.pad + adx;
            bool ok = mv && akv;
            if (p.circular) {
                yy = wrap_idx(yy, p.H);
                xx = wrap_idx(xx, p.W);
            } else {
                ok = ok && yy >= 0 && yy < p.H && xx >= 0 && xx < p.W;
            }
            const int off = ok ? ((b * p.H + yy) * p.W + xx) * aC * 4 + aoff : OOB;
            ra[i] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(asrc1 ? r1 : r2, off, 0, 0));
        }
#pragma unroll
        for (int i = 0; i < NT; ++i) {  // B pieces: idx = tid + 256 i -> row idx / (2 OB), piece idx % (2 OB)
            const int idx = tid + 256 * i;
            const int row = idx / (2 * OB), q = idx - row * (2 * OB);
            const int pl = q / OB, oc = q - pl * OB;
            const int m = c * 32 + row;
            const int co = c0 + 8 * oc;
            const bool ok = m < p.M && co < p.Cout;
            const int off = ok ? (m * p.Cout + co) * 4 + 16 * pl : OOB;
            rb[i] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rd, off, 0, 0));
        }
    };
    auto store = [&](int buf) {
        char* A = wsm + buf * STG;
        char* B = A + AB;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int row = (tid >> 5) + 8 * i;
            *reinterpret_cast<float4*>(A + row * ROWB + 16 * (16 * apl + (aoc ^ (4 * (row & 3))))) = ra[i];
        }
#pragma unroll
        for (int i = 0; i < NT; ++i) {
            const int idx = tid + 256 * i;
            const int row = idx / (2 * OB), q = idx - row * (2 * OB);
            const int pl = q / OB, oc = q - pl * OB;
            *reinterpret_cast<float4*>(B + row * ROWB + 16 * (16 * pl + (oc ^ (4 * (row & 3))))) = rb[i];
        }
    };
    f32x16 acc[NT];
#pragma unroll
    for (int n = 0; n < NT; ++n) acc[n] = (f32x16){};
    const int lane = tid & 63, wv = tid >> 6, li = lane & 31, lh = lane >> 5;
    // tr-read address of this lane: group g = lane / 16, q = (lane / 4) % 4, pp = lane % 4; operand
    // rows (pixels) 16 s + 8 (g >> 1) + 4 r + q, columns 16 (g & 1) + 4 pp of the 32-column tile
    const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
    const int trow = 8 * (g >> 1) + q;                // + 16 s + 4 r (both keep row & 3 == q)
    const int tpc = 2 * (g & 1) + (pp >> 1);           // piece within the tile's 4-piece group
    const int tb = trow * ROWB + 8 * (pp & 1);
    const int apc = 16 * ((4 * wv + tpc) ^ (4 * q));   // A: octet 4 wv + tpc of the hi plane
    typedef short v4s __attribute__((ext_vector_type(4)));
    auto tr = [&](const char* base) {
        return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(base));
    };
    auto frag8 = [&](const char* img, int pc, int s, int plane) -> h8 {
        const char* b0 = img + tb + 16 * s * ROWB + pc + 256 * plane;
        const v4s u0 = tr(b0), u1 = tr(b0 + 4 * ROWB);
        typedef short v8s __attribute__((ext_vector_type(8)));
        const v8s u = __builtin_shufflevector(u0, u1, 0, 1, 2, 3, 4, 5, 6, 7);
        return __builtin_bit_cast(h8, u);
    };
    if (chunk0 < chunk1) {
        load(chunk0);
        store(0);
    }
    __syncthreads();
    for (int c = chunk0; c < chunk1; ++c) {
        const int cur = (c - chunk0) & 1;
        if (c + 1 < chunk1) load(c + 1);
        const char* A = wsm + cur * STG;
        const char* B = A + AB;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            const h8 fah = frag8(A, apc, s, 0);
            const h8 fal = frag8(A, apc, s, 1);
            h8 fbh[NT], fbl[NT];
#pragma unroll
            for (int n = 0; n < NT; ++n) {
                const int bpc = 16 * ((4 * n + tpc) ^ (4 * q));
                fbh[n] = frag8(B, bpc, s, 0);
                fbl[n] = frag8(B, bpc, s, 1);
            }
#pragma unroll
            for (int n = 0; n < NT; ++n) acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fah, fbl[n], acc[n], 0, 0, 0);
#pragma unroll
            for (int n = 0; n < NT; ++n) acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fal, fbh[n], acc[n], 0, 0, 0);
#pragma unroll
            for (int n = 0; n < NT; ++n) acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fah, fbh[n], acc[n], 0, 0, 0);
        }
        if (c + 1 < chunk1) store(cur ^ 1);
        __syncthreads();
    }
    const float sc = *p.comb;
    float* dst = p.part + (size_t)split * p.K * p.Cout;
#pragma unroll
    for (int n = 0; n < NT; ++n) {
        const int co = c0 + n * 32 + li;
        if (co >= p.Cout) continue;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int k = k0 + wv * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
            if (k < p.K) dst[(size_t)k * p.Cout + co] = acc[n][r] * sc;
        }
    }
}
constexpr size_t wgrad_h2_lds_bytes() { return 2 * (size_t)(32 * 512 + 32 * 512); }

// dw[co][ci][ky][kx] = beta * dw + sum_s part[s][k][co], k = (ky*ks + kx)*Cin + ci (fixed order)
__global__ void k_wgrad_reduce(const float* __restrict__ part, int nsplit, int K, int Cout, int Cin, int ks,
                               float beta, float* __restrict__ dw) {
    const size_t n = (size_t)K * Cout;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const int k = (int)(i / Cout), co = (int)(i - (size_t)k * Cout);
        float s = 0.f;
#pragma unroll 8
        for (int sp = 0; sp < nsplit; ++sp) s += part[(size_t)sp * n + i];
        const int tap = k / Cin, ci = k - tap * Cin;
        const size_t o = ((size_t)co * Cin + ci) * ks * ks + tap;
        dw[o] = beta != 0.f ? beta * dw[o] + s : s;
    }
}

void wgrad_plan(int M, int K, int Cout, int* nt, int* nsplit, int* cps, int* nkblk, int* ncblk) {
    *nt = Cout <= 32 ? 1 : (Cout <= 64 ? 2 : 3);
    *nkblk = cdiv(K, GBM);
    *ncblk = cdiv(Cout, 32 * *nt);
    const int tiles = *nkblk * *ncblk;
    const int nch = cdiv(std::max(M, 1), 32);
    int ns = std::max(1, cdiv(2048, tiles));
    ns = std::min(ns, std::max(1, nch / 8));  // >= 8 chunks per split
    ns = std::min(ns, 256);                   // the reduction folds ns partials per weight
    *cps = cdiv(nch, ns);
    *nsplit = cdiv(nch, *cps);
}

}  // namespace
}  // namespace tcx

using namespace tcx;

namespace tcx {
namespace {

// split-K plan: when the output tiles cannot fill the chip (fewer than 256) and K is long, split
// the reduction so that ~512 workgroups run; each split covers >= 4 chunks of 32
void gemm_split_plan(int M, int N, int K, int batch, int* nsplit, int* kcs) {
    const int nt = N <= 32 ? 1 : (N <= 64 ? 2 : 3);
    const long long tiles = (long long)cdiv(M, GBM) * cdiv(N, 32 * nt) * batch;
    const int nch = (K + GBK - 1) / GBK;
    *nsplit = 1;
    *kcs = nch;
    if (tiles >= 256 || nch < 8) return;
    int s = (int)std::min<long long>((512 + tiles - 1) / tiles, 16);
    s = std::min(s, nch / 4);
    if (s < 2) return;
    *kcs = (nch + s - 1) / s;
    *nsplit = (nch + *kcs - 1) / *kcs;
}

int gemm_impl(int M, int N, int K, float alpha, const float* A, long long sa_m, long long sa_k, const float* B,
              long long sb_k, long long sb_n, float beta, float* C, long long sc_m, long long sc_n, const float* bias,
              int batch, int bdiv, long long sa_hi, long long sa_lo, long long sb_hi, long long sb_lo,
              long long sc_hi, long long sc_lo, void* ws, size_t ws_bytes, hipStream_t st) {
    TCX_REQUIRE(M >= 0 && N >= 0 && K >= 0 && batch >= 0 && bdiv >= 1, "tcx_gemm: bad sizes");
    TCX_REQUIRE(C && (K == 0 || (A && B)), "tcx_gemm: null pointer");
    if (M == 0 || N == 0 || batch == 0) return TCX_OK;
    GemmParams p{};
    p.M = M; p.N = N; p.K = K; p.alpha = alpha; p.beta = beta;
    p.A = A; p.sam = sa_m; p.sak = sa_k; p.B = B; p.sbk = sb_k; p.sbn = sb_n;
    p.C = C; p.scm = sc_m; p.scn = sc_n; p.bias = bias;
    p.bdiv = bdiv; p.sah = sa_hi; p.sal = sa_lo; p.sbh = sb_hi; p.sbl = sb_lo; p.sch = sc_hi; p.scl = sc_lo;
    auto mul4 = [](long long v) { return v % 4 == 0; };
    const bool zA = mul4(sa_hi) && mul4(sa_lo) && aligned16(A);
    const bool zB = mul4(sb_hi) && mul4(sb_lo) && aligned16(B);
    int la = 2, lb = 2;
    if (K > 0) {
        if (sa_k == 1 && K % 4 == 0 && mul4(sa_m) && zA) la = 0;
        else if (sa_m == 1 && M % 4 == 0 && mul4(sa_k) && zA) la = 1;
        if (sb_k == 1 && K % 4 == 0 && mul4(sb_n) && zB) lb = 0;
        else if (sb_n == 1 && N % 4 == 0 && mul4(sb_k) && zB) lb = 1;
    }
    const int nt = N <= 32 ? 1 : (N <= 64 ? 2 : 3);
    p.nmblk = cdiv(M, GBM);
    p.nnblk = cdiv(N, 32 * nt);
    if (K == 0) {  // C = beta * C + bias: run the kernel with an empty reduction
        la = 2; lb = 2;
    }
    int ns = 1, kcs = 0;
    if (ws && K > 0) gemm_split_plan(M, N, K, batch, &ns, &kcs);
    if (ns > 1 && ws_bytes >= (size_t)ns * batch * M * N * sizeof(float)) {
        p.part = static_cast<float*>(ws);
        p.nsplit = ns;
        p.kcs = kcs;
    }
    int rc;
    if (nt == 3) rc = launch_gemm_nt<3>(p, la, lb, batch, st);
    else if (nt == 2) rc = launch_gemm_nt<2>(p, la, lb, batch, st);
    else rc = launch_gemm_nt<1>(p, la, lb, batch, st);
    if (rc != TCX_OK || !p.part) return rc;
    const size_t n_all = (size_t)batch * M * N;
    const int blocks = (int)std::min<size_t>((n_all + 255) / 256, 4096);
    hipLaunchKernelGGL(k_gemm_reduce, dim3(blocks), dim3(256), 0, st, p, batch);
    return check_launch("tcx_gemm(split-K reduce)");
}

}  // namespace
}  // namespace tcx

extern "C" int tcx_gemm(int M, int N, int K, float alpha, const float* A, long long sa_m, long long sa_k,
                        const float* B, long long sb_k, long long sb_n, float beta, float* C, long long sc_m,
                        long long sc_n, const float* bias, int batch, int bdiv, long long sa_hi, long long sa_lo,
                        long long sb_hi, long long sb_lo, long long sc_hi, long long sc_lo, void* stream) {
    return gemm_impl(M, N, K, alpha, A, sa_m, sa_k, B, sb_k, sb_n, beta, C, sc_m, sc_n, bias, batch, bdiv, sa_hi,
                     sa_lo, sb_hi, sb_lo, sc_hi, sc_lo, nullptr, 0, (hipStream_t)stream);
}

extern "C" size_t tcx_gemm_workspace(int M, int N, int K, int batch) {
    if (M <= 0 || N <= 0 || K <= 0 || batch <= 0) return 0;
    int ns, kcs;
    gemm_split_plan(M, N, K, batch, &ns, &kcs);
    return ns > 1 ? (size_t)ns * batch * M * N * sizeof(float) : 0;
}

extern "C" int tcx_gemm_ws(int M, int N, int K, float alpha, const float* A, long long sa_m, long long sa_k,
                           const float* B, long long sb_k, long long sb_n, float beta, float* C, long long sc_m,
                           long long sc_n, const float* bias, int batch, int bdiv, long long sa_hi, long long sa_lo,
                           long long sb_hi, long long sb_lo, long long sc_hi, long long sc_lo, void* ws,
                           size_t ws_bytes, void* stream) {
    return gemm_impl(M, N, K, alpha, A, sa_m, sa_k, B, sb_k, sb_n, beta, C, sc_m, sc_n, bias, batch, bdiv, sa_hi,
                     sa_lo, sb_hi, sb_lo, sc_hi, sc_lo, ws, ws_bytes, (hipStream_t)stream);
}

// ---------------------------------------------------------------- linears (split-K / skinny)
namespace tcx {
namespace {

// y[M][N] = act(x1 W1^T + x2 W2^T + b + resid) with W = wpk [npad][kpad] (k < K1 from x1, then x2):
// each source is a split-K GEMM writing raw partials (splits >= 2 chunks of 32), one fixed-order
// reduce applies bias / residual / activation.  Plan: the splits of both sources together.
struct LinPlan {
    int s1, k1cs, s2, k2cs;
};

LinPlan linear_plan(int M, int N, int K1, int K2) {
    const long long tiles = (long long)cdiv(M, GBM) * cdiv(N, 96);
    auto one = [&](int K, int& s, int& kcs) {
        const int nch = (K + GBK - 1) / GBK;
        s = (int)std::min<long long>((512 + tiles - 1) / tiles, 16);
        s = std::max(1, std::min(s, nch / 2));
        kcs = (nch + s - 1) / s;
        s = (nch + kcs - 1) / kcs;
    };
    LinPlan lp{};
    one(K1, lp.s1, lp.k1cs);
    if (K2 > 0) one(K2, lp.s2, lp.k2cs);
    return lp;
}

bool linear_wants_split(int M, int N, int K1, int K2, const float* x1, const float* x2) {
    const long long tiles = (long long)cdiv(M, GBM) * cdiv(N, 96);
    return tiles < 128 && K1 % 4 == 0 && K2 % 4 == 0 && K1 + K2 >= 256 && aligned16(x1) && (!x2 || aligned16(x2));
}

}  // namespace
}  // namespace tcx

extern "C" size_t tcx_linear_workspace(int M, int N, int K1, int K2) {
    if (M <= 0 || N <= 0 || K1 <= 0 || K2 < 0) return 0;
    if (skinny_ok(M, N, K1, K2)) return skinny_part_floats(skinny_plan(K1, K2), M, N) * sizeof(float);
    if (!linear_wants_split(M, N, K1, K2, nullptr, nullptr)) return 0;
    const LinPlan lp = linear_plan(M, N, K1, K2);
    return (size_t)(lp.s1 + lp.s2) * M * N * sizeof(float);
}

extern "C" int tcx_linear_ws(const float* x1, int K1, const float* x2, int K2, const float* wpk, const float* b,
                             const float* resid, float* y, int M, int N, int npad, int kpad, int act, void* ws,
                             size_t ws_bytes, void* stream) {
    hipStream_t st = (hipStream_t)stream;
    const size_t need = tcx_linear_workspace(M, N, K1, K2);
    if (need > 0 && ws && ws_bytes >= need && skinny_ok(M, N, K1, K2) && aligned16(wpk) && aligned16(x1) &&
        (!x2 || aligned16(x2)) && kpad % 4 == 0 && npad >= 16 * cdiv(N, 16)) {
        // M <= 64: each weight streamed once, fixed-order reduce with the epilogue (skinny.hip)
        TCX_REQUIRE(x1 && y && N > 0 && (K2 == 0) == (x2 == nullptr) && kpad >= K1 + K2 && act >= 0 && act <= 3,
                    "tcx_linear_ws: bad args");
        SkEpi e;
        e.b = b; e.resid = resid; e.act = act; e.y = y;
        return skinny_linear(x1, K1, K1, x2, K2, K2, wpk, kpad, M, N, static_cast<float*>(ws), e, st);
    }
    if (need == 0 || !ws || ws_bytes < need || !linear_wants_split(M, N, K1, K2, x1, x2) || !aligned16(wpk))
        return tcx_linear(x1, K1, x2, K2, wpk, b, resid, y, M, N, npad, kpad, act, stream);
    TCX_REQUIRE(x1 && wpk && y && M >= 0 && N > 0 && K1 > 0 && K2 >= 0 && (K2 == 0) == (x2 == nullptr),
                "tcx_linear_ws: bad args");
    TCX_REQUIRE(npad >= N && kpad >= K1 + K2 && kpad % 4 == 0 && act >= 0 && act <= 3, "tcx_linear_ws: bad padding");
    const LinPlan lp = linear_plan(M, N, K1, K2);
    float* part = static_cast<float*>(ws);
    auto src = [&](const float* x, int K, int koff, int s, int kcs, float* pbase) -> int {
        GemmParams p{};
        p.M = M; p.N = N; p.K = K; p.alpha = 1.f; p.beta = 0.f;
        p.A = x; p.sam = K; p.sak = 1;
        p.B = wpk + koff; p.sbk = 1; p.sbn = kpad;
        p.C = y; p.scm = N; p.scn = 1; p.bdiv = 1;
        p.nmblk = cdiv(M, GBM);
        p.nnblk = cdiv(N, 96);
        p.part = pbase; p.nsplit = s; p.kcs = kcs;
        return launch_gemm_nt<3>(p, 0, 0, 1, st);
    };
    TCX_TRY(src(x1, K1, 0, lp.s1, lp.k1cs, part));
    if (K2 > 0) TCX_TRY(src(x2, K2, K1, lp.s2, lp.k2cs, part + (size_t)lp.s1 * M * N));
    GemmParams r{};
    r.M = M; r.N = N; r.alpha = 1.f; r.beta = 0.f; r.C = y; r.scm = N; r.scn = 1; r.bdiv = 1;
    r.bias = b; r.part = part; r.nsplit = lp.s1 + lp.s2; r.resid = resid; r.act = act;
    const size_t n_all = (size_t)M * N;
    hipLaunchKernelGGL(k_gemm_reduce, dim3((unsigned)std::min<size_t>((n_all + 255) / 256, 4096)), dim3(256), 0, st,
                       r, 1);
    return check_launch("tcx_linear_ws reduce");
}

extern "C" size_t tcx_conv_wgrad_workspace(int Bt, int Ho, int Wo, int Cin, int Cout, int ks) {
    int nt, ns, cps, nk, nc;
    const int K = ks * ks * Cin;
    wgrad_plan(Bt * Ho * Wo, K, Cout, &nt, &ns, &cps, &nk, &nc);
    return (size_t)ns * K * Cout * sizeof(float) + 256;
}

extern "C" int tcx_conv_wgrad(const float* x1, const float* x2, int Bt, int H, int W, int C1, int C2,
                              const float* dy, int Cout, int ks, int stride, int pad, int circular, float beta,
                              float* dw, void* ws, size_t ws_bytes, void* stream) {
    TCX_REQUIRE(x1 && dy && dw && ws, "tcx_conv_wgrad: null pointer");
    TCX_REQUIRE((C2 == 0) == (x2 == nullptr) && C1 > 0 && C2 >= 0 && Cout > 0 && Bt >= 0, "tcx_conv_wgrad: bad shape");
    TCX_REQUIRE(ks >= 1 && stride >= 1 && pad >= 0, "tcx_conv_wgrad: bad geometry");
    WgParams p{};
    p.x1 = x1; p.x2 = x2; p.C1 = C1; p.C2 = C2; p.Cin = C1 + C2; p.H = H; p.W = W;
    p.Ho = (H + 2 * pad - ks) / stride + 1;
    p.Wo = (W + 2 * pad - ks) / stride + 1;
    TCX_REQUIRE(p.Ho > 0 && p.Wo > 0, "tcx_conv_wgrad: empty output");
    p.HoWo = p.Ho * p.Wo; p.M = Bt * p.HoWo;
    p.ks = ks; p.stride = stride; p.pad = pad; p.circular = circular;
    p.dy = dy; p.Cout = Cout; p.K = ks * ks * p.Cin;
    int nt;
    wgrad_plan(p.M, p.K, Cout, &nt, &p.nsplit, &p.cps, &p.nkblk, &p.ncblk);
    const size_t need = (size_t)p.nsplit * p.K * Cout * sizeof(float);
    char* base = reinterpret_cast<char*>(align_up(reinterpret_cast<uintptr_t>(ws), 256));
    TCX_REQUIRE(need + (base - (char*)ws) <= ws_bytes, "tcx_conv_wgrad: workspace too small (%zu < %zu)", ws_bytes,
                need + 256);
    p.part = reinterpret_cast<float*>(base);
    if (C2 == 0 && pad == 1 && aligned16(x1) && aligned16(dy) && aligned16(p.part)) {
        // one-channel side (the score net's first / out convs): VALU reduction planes, thin.hip
        ThinWgrad a{};
        const size_t plane = (size_t)p.K * Cout * sizeof(float);
        const size_t room = (ws_bytes - (size_t)(base - (char*)ws)) / plane;
        const int ns = thin_wgrad_plan(Bt, H, W, C1, Cout, ks, stride, (int)std::min<size_t>(room, 256), &a);
        if (ns > 0 && p.Ho == H && p.Wo == W) {
            const bool cout1 = Cout == 1;
            a.wide = cout1 ? x1 : dy;
            a.thin = cout1 ? dy : x1;
            a.pad = pad; a.circular = circular; a.sign = cout1 ? -1 : 1; a.part = p.part;
            TCX_TRY(launch_thin_wgrad(a, ns, (hipStream_t)stream));
            const size_t n = (size_t)p.K * Cout;
            hipLaunchKernelGGL(k_wgrad_reduce, dim3((int)std::min<size_t>((n + 255) / 256, 4096)), dim3(256), 0,
                               (hipStream_t)stream, p.part, ns, p.K, Cout, p.Cin, ks, beta, dw);
            return check_launch("tcx_conv_wgrad reduce");
        }
    }
    const bool asc = (C1 % 4 != 0) || (C2 % 4 != 0) || !aligned16(x1) || (x2 && !aligned16(x2));
    const bool bsc = (Cout % 4 != 0) || !aligned16(dy);
    hipStream_t st = (hipStream_t)stream;
    const dim3 grid(p.nkblk * p.ncblk, p.nsplit);
#define TCX_W(NT_)                                                                                     \
    do {                                                                                               \
        if (!asc && !bsc) hipLaunchKernelGGL((k_wgrad<NT_, false, false>), grid, dim3(256), 0, st, p); \
        else if (!asc) hipLaunchKernelGGL((k_wgrad<NT_, false, true>), grid, dim3(256), 0, st, p);     \
        else if (!bsc) hipLaunchKernelGGL((k_wgrad<NT_, true, false>), grid, dim3(256), 0, st, p);     \
        else hipLaunchKernelGGL((k_wgrad<NT_, true, true>), grid, dim3(256), 0, st, p);                \
    } while (0)
    if (nt == 3) TCX_W(3);
    else if (nt == 2) TCX_W(2);
    else TCX_W(1);
#undef TCX_W
    TCX_TRY(check_launch("tcx_conv_wgrad"));
    const size_t n = (size_t)p.K * Cout;
    const int blocks = (int)std::min<size_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(k_wgrad_reduce, dim3(blocks), dim3(256), 0, st, p.part, p.nsplit, p.K, Cout, p.Cin, ks, beta,
                       dw);
    return check_launch("tcx_conv_wgrad reduce");
}

extern "C" int tcx_conv_wgrad_h2(const void* x1, const void* x2, int Bt, int H, int W, int C1, int C2, const void* dy,
                                 int Cout, int ks, int stride, int pad, int circular, float beta, const float* comb,
                                 float* dw, void* ws, size_t ws_bytes, void* stream) {
    TCX_REQUIRE(x1 && dy && dw && ws && comb, "tcx_conv_wgrad_h2: null pointer");
    TCX_REQUIRE((C2 == 0) == (x2 == nullptr) && C1 > 0 && C1 % 8 == 0 && C2 % 8 == 0 && Cout % 8 == 0 && Bt >= 0,
                "tcx_conv_wgrad_h2: needs C1, C2, Cout %% 8 == 0 (h2 records)");
    TCX_REQUIRE(ks >= 1 && stride >= 1 && pad >= 0, "tcx_conv_wgrad_h2: bad geometry");
    TCX_REQUIRE(aligned16(x1) && (!x2 || aligned16(x2)) && aligned16(dy), "tcx_conv_wgrad_h2: 16-B alignment");
    WgParams p{};
    p.x1 = (const float*)x1; p.x2 = (const float*)x2; p.C1 = C1; p.C2 = C2; p.Cin = C1 + C2; p.H = H; p.W = W;
    p.Ho = (H + 2 * pad - ks) / stride + 1;
    p.Wo = (W + 2 * pad - ks) / stride + 1;
    TCX_REQUIRE(p.Ho > 0 && p.Wo > 0, "tcx_conv_wgrad_h2: empty output");
    p.HoWo = p.Ho * p.Wo; p.M = Bt * p.HoWo;
    p.ks = ks; p.stride = stride; p.pad = pad; p.circular = circular;
    p.dy = (const float*)dy; p.Cout = Cout; p.K = ks * ks * p.Cin; p.comb = comb;
    int nt;
    wgrad_plan(p.M, p.K, Cout, &nt, &p.nsplit, &p.cps, &p.nkblk, &p.ncblk);
    const size_t need = (size_t)p.nsplit * p.K * Cout * sizeof(float);
    char* base = reinterpret_cast<char*>(align_up(reinterpret_cast<uintptr_t>(ws), 256));
    TCX_REQUIRE(need + (base - (char*)ws) <= ws_bytes, "tcx_conv_wgrad_h2: workspace too small (%zu < %zu)",
                ws_bytes, need + 256);
    p.part = reinterpret_cast<float*>(base);
    hipStream_t st = (hipStream_t)stream;
    {
        // 3x3 stride-1 convs: the halo-staged kernel (wgrad3h.hip), all nine taps per workgroup
        const size_t in1 = (size_t)Bt * H * W * C1 * 4, in2 = (size_t)Bt * H * W * C2 * 4, ind = (size_t)p.M * Cout * 4;
        if (wgrad3h_takes(Bt, H, W, C1, C2, Cout, ks, stride, pad, in1, in2, ind)) {
            Wg3hArgs a{};
            a.x1 = (const char*)x1; a.x2 = (const char*)x2; a.dy = (const char*)dy;
            a.bx1 = (unsigned)in1; a.bx2 = (unsigned)in2; a.bdy = (unsigned)ind;
            a.B = Bt; a.H = H; a.W = W; a.C1 = C1; a.C2 = C2; a.Cin = C1 + C2; a.Cout = Cout; a.circular = circular;
            a.comb = comb; a.part = p.part;
            const size_t room = (ws_bytes - (size_t)(base - (char*)ws)) / ((size_t)p.K * Cout * sizeof(float));
            int ns = 0;
            TCX_TRY(launch_wgrad3h(a, (int)std::min<size_t>(room, 256), &ns, st));
            const size_t n = (size_t)p.K * Cout;
            hipLaunchKernelGGL(k_wgrad_reduce, dim3((int)std::min<size_t>((n + 255) / 256, 4096)), dim3(256), 0, st,
                               p.part, ns, p.K, Cout, p.Cin, ks, beta, dw);
            return check_launch("tcx_conv_wgrad_h2 reduce");
        }
    }
    const dim3 grid(p.nkblk * p.ncblk, p.nsplit);
    // operands past 2 GiB (32-bit buffer offsets) take the round-2 quad-staged k_wgrad_h2_r2 (the knob that
    // selected it for A/B was removed in round 4: 419 vs 613 us, r03)
    const size_t in1 = (size_t)Bt * H * W * C1 * 4, in2 = (size_t)Bt * H * W * C2 * 4, ind = (size_t)p.M * Cout * 4;
    if (in1 < (1u << 31) && in2 < (1u << 31) && ind < (1u << 31)) {
        p.bx1 = (unsigned)in1; p.bx2 = (unsigned)in2; p.bdy = (unsigned)ind;
        using K = void (*)(WgParams);
        const K k = nt == 3 ? &k_wgrad_h2<3> : (nt == 2 ? &k_wgrad_h2<2> : &k_wgrad_h2<1>);
        static bool attr[3] = {};
        if (!attr[nt - 1]) {
            if (hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)wgrad_h2_lds_bytes()) != hipSuccess) {
                set_error("tcx_conv_wgrad_h2: cannot enable %zu B of dynamic LDS", wgrad_h2_lds_bytes());
                return TCX_EHIP;
            }
            attr[nt - 1] = true;
        }
        hipLaunchKernelGGL(k, grid, dim3(256), wgrad_h2_lds_bytes(), st, p);
    } else if (nt == 3) hipLaunchKernelGGL((k_wgrad_h2_r2<3>), grid, dim3(256), 0, st, p);
    else if (nt == 2) hipLaunchKernelGGL((k_wgrad_h2_r2<2>), grid, dim3(256), 0, st, p);
    else hipLaunchKernelGGL((k_wgrad_h2_r2<1>), grid, dim3(256), 0, st, p);
    TCX_TRY(check_launch("tcx_conv_wgrad_h2"));
    const size_t n = (size_t)p.K * Cout;
    const int blocks = (int)std::min<size_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(k_wgrad_reduce, dim3(blocks), dim3(256), 0, st, p.part, p.nsplit, p.K, Cout, p.Cin, ks, beta,
                       dw);
    return check_launch("tcx_conv_wgrad_h2 reduce");
}
