// Skinny-M linears: y[M][N] = epilogue(x W^T) for M <= 64 rows (the prior's DDIM over a few dozen
// latents, diffusion_prior.py:203-252, and any small-batch nn.Linear of the mirrors).
//
// At M = 36 a 128-row MFMA tile wastes 72 % of its rows and the weights (412 MB per prior forward)
// are the whole cost, so this path is built around streaming W exactly once with as many bytes in
// flight as the chip needs (~16 MB for 8 TB/s at ~2 us latency) and as few launches as possible
// (a dependent kernel boundary costs ~1.5-2 us, MI355X_MICROARCH.md "boundary"):
//
//   k_skinny<MT, NB>: a workgroup = 8 waves on ONE tile of 16 output columns; wave w takes the
//     K slice [k0 + 16 NB w, +16 NB) of the workgroup's chunk of 128 NB values.
//     * every lane issues ALL its loads up front (NB weight float4 + NB x MT activation float4:
//       8 KB of weights per wave at NB = 8, no loop-carried latency); activations are re-read by
//       every column tile from L2 (x is a few hundred KB), weights come from HBM once;
//     * v_mfma_f32_16x16x4_f32 (exact fp32 products, the reference's fp32 GEMM class): lane l holds
//       W[n0 + (l&15)][kb + 4(l>>4) .. +3] and x[16t + (l&15)][same k] as float4 and feeds 4 k-steps
//       with element j of both (a k permutation applied to both sides: dot products unchanged);
//     * the 8 waves' accumulators are summed through LDS in wave order (deterministic); a chunk
//       count S = 1 (K <= 128 NB, e.g. fc1 at K = 1024) applies the epilogue right there (bias,
//       residual, activation, or the DDIM update) - no partials, no second launch; S > 1 writes
//       part[S][M][N] for one fixed-order reduce (k_sk_reduce*, optionally fused with LayerNorm).
#include "skinny.hpp"
#include "h2.hpp"

#include <algorithm>
#include <cstdlib>

namespace tcx {
namespace {

constexpr int SK_WAVES = 8;  // waves per workgroup, each on its own K slice

__device__ __attribute__((aligned(16))) float sk_zero4[4] = {0.f, 0.f, 0.f, 0.f};

typedef float f32x4 __attribute__((ext_vector_type(4)));

struct SkArgs {
    const float* x;
    int ldx, K;
    const float* w;
    int kpad, M, N;
    float* part;   // S > 1: partial planes
    int direct;    // S == 1: apply e here
    SkEpi e;
};

__device__ __forceinline__ float sk_act(float v, int act);
__device__ __forceinline__ float ddim_z(float z, float e, float abar_t, float abar_prev, int last);

template <int MT, int NB>
__global__ __launch_bounds__(512) void k_skinny(SkArgs a) {
    constexpr int KC = 16 * NB;  // k values per wave
    mfma_agpr_form();
    __shared__ float red[SK_WAVES][16 * MT][17];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int r = lane & 15, q = lane >> 4;
    const int n0 = blockIdx.x * 16;
    const int sidx = blockIdx.y;
    // wave -> K slice rotated by the column tile: the 8 waves of the 32 CUs of an XCD then read
    // different activation lines at any moment instead of all hammering the same L2 channel
    const int slice = (wv + blockIdx.x) & (SK_WAVES - 1);
    const int kw0 = sidx * SK_WAVES * KC + slice * KC;
    const int kend = min(a.K, kw0 + KC);
    const int K = a.K;
    // all loads up front: weights (clamped address, always valid), activations (zero for k blocks
    // past this wave's range; rows past M read row M-1, their outputs are discarded)
    const float* wr = a.w + (size_t)(n0 + r) * a.kpad + 4 * q;
    float4 wf[NB], xf[NB][MT];
#pragma unroll
    for (int u = 0; u < NB; ++u) {
        const int kc = min(kw0 + 16 * u, K - 16);
        wf[u] = *reinterpret_cast<const float4*>(wr + kc);
    }
#pragma unroll
    for (int u = 0; u < NB; ++u) {
        const int kb = kw0 + 16 * u;
        const int kc = min(kb, K - 16);
        const bool live = kb < kend;
#pragma unroll
        for (int t = 0; t < MT; ++t) {
            const float* xp = a.x + (size_t)min(16 * t + r, a.M - 1) * a.ldx + kc + 4 * q;
            xf[u][t] = *reinterpret_cast<const float4*>(live ? xp : sk_zero4);
        }
    }
    // keep every load above in flight before the first MFMA (left alone, the scheduler trades
    // registers for latency and interleaves one load per MFMA group: a round trip each)
    __builtin_amdgcn_sched_barrier(0);
    f32x4 acc[MT];
#pragma unroll
    for (int t = 0; t < MT; ++t) acc[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
    {
#pragma unroll
        for (int u = 0; u < NB; ++u) {
#pragma unroll
            for (int t = 0; t < MT; ++t) {
                acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(xf[u][t].x, wf[u].x, acc[t], 0, 0, 0);
                acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(xf[u][t].y, wf[u].y, acc[t], 0, 0, 0);
                acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(xf[u][t].z, wf[u].z, acc[t], 0, 0, 0);
                acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(xf[u][t].w, wf[u].w, acc[t], 0, 0, 0);
            }
        }
    }
    // D: col = n0 + (lane & 15), row = 16 t + 4 (lane >> 4) + reg
#pragma unroll
    for (int t = 0; t < MT; ++t)
#pragma unroll
        for (int e = 0; e < 4; ++e) red[wv][16 * t + 4 * q + e][r] = acc[t][e];
    __syncthreads();
    const int M = a.M, N = a.N;
    for (int o = tid; o < M * 16; o += 64 * SK_WAVES) {
        const int m = o >> 4, c = o & 15, n = n0 + c;
        float v = red[0][m][c];
#pragma unroll
        for (int w = 1; w < SK_WAVES; ++w) v += red[w][m][c];
        if (n >= N) continue;
        const size_t i = (size_t)m * N + n;
        if (!a.direct) {
            a.part[(size_t)sidx * M * N + i] = v;
            continue;
        }
        if (a.e.b) v += a.e.b[n];
        if (a.e.resid) v += a.e.resid[i];
        v = sk_act(v, a.e.act);
        if (a.e.z) a.e.z[i] = ddim_z(a.e.z[i], v, a.e.abar_t, a.e.abar_prev, a.e.last);
        else a.e.y[i] = v;
    }
}

// ---- f16x3 skinny linear: x, W in h2 storage; one wave = 16 columns x a K slice of 32 NC values
struct SkH2Args {
    const char* x;     // [M][K/8][2][8] f16
    const char* w;     // [>= 16 ceil(N/16)][K/8][2][8] f16, rows scaled by 1 / winv
    const float* winv;
    int K, M, N;
    float* part;
    int direct;
    SkEpi e;
};

__device__ __attribute__((aligned(16))) float sk_zero8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};

template <int MT, int NC>
__global__ __launch_bounds__(512) void k_skinny_h2(SkH2Args a) {
    constexpr int KC = 32 * NC;  // k values per wave
    mfma_agpr_form();
    __shared__ float red[SK_WAVES][16 * MT][17];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int r = lane & 15, q = lane >> 4;
    const int n0 = blockIdx.x * 16;
    const int sidx = blockIdx.y;
    const int slice = (wv + blockIdx.x) & (SK_WAVES - 1);  // see k_skinny
    const int K = a.K, G = K / 8;
    const int kw0 = sidx * SK_WAVES * KC + slice * KC;
    const int kend = min(K, kw0 + KC);
    // lane (r, q) of k block c holds group 4c + q (8 k values) of its row: A[i = r][k = 8q + j] and
    // B[k = 8q + j][n = r] of v_mfma_f32_16x16x32_f16 (the same k order on both sides)
    const char* wr = a.w + ((size_t)(n0 + r) * G + q) * 32;
    const float winv = a.winv[n0 + r < a.N ? n0 + r : 0];
    uint4 wh[NC], wl[NC], xh[NC][MT], xl[NC][MT];
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        const int kc = min(kw0 + 32 * c, K - 32);
        const char* p = wr + (size_t)(kc / 8) * 32;
        wh[c] = *reinterpret_cast<const uint4*>(p);
        wl[c] = *reinterpret_cast<const uint4*>(p + 16);
    }
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        const int kb = kw0 + 32 * c;
        const int kc = min(kb, K - 32);
        const bool live = kb < kend;
#pragma unroll
        for (int t = 0; t < MT; ++t) {
            const char* p = a.x + ((size_t)min(16 * t + r, a.M - 1) * G + kc / 8 + q) * 32;
            const char* src = live ? p : reinterpret_cast<const char*>(sk_zero8);
            xh[c][t] = *reinterpret_cast<const uint4*>(src);
            xl[c][t] = *reinterpret_cast<const uint4*>(src + 16);
        }
    }
    // the h2 epilogue's bias (thread tid < 2M owns row tid/2, columns n0 + 8 (tid&1) .. +7): requested
    // with the operands so that it is not a second round trip after the barrier
    float4 bia0 = make_float4(0.f, 0.f, 0.f, 0.f), bia1 = bia0;
    if (a.direct && a.e.y_h2 && a.e.b) {
        const int nb = min(n0 + 8 * (tid & 1), max(a.N - 8, 0));
        bia0 = *reinterpret_cast<const float4*>(a.e.b + nb);
        bia1 = *reinterpret_cast<const float4*>(a.e.b + nb + 4);
    }
    __builtin_amdgcn_sched_barrier(0);  // all loads in flight first (k_skinny)
    f32x4 acc[MT];
#pragma unroll
    for (int t = 0; t < MT; ++t) acc[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        const h8 bh = __builtin_bit_cast(h8, wh[c]), bl = __builtin_bit_cast(h8, wl[c]);
#pragma unroll
        for (int t = 0; t < MT; ++t) {
            const h8 ah = __builtin_bit_cast(h8, xh[c][t]), al = __builtin_bit_cast(h8, xl[c][t]);
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl, acc[t], 0, 0, 0);
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh, acc[t], 0, 0, 0);
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, acc[t], 0, 0, 0);
        }
    }
#pragma unroll
    for (int t = 0; t < MT; ++t)
#pragma unroll
        for (int e = 0; e < 4; ++e) red[wv][16 * t + 4 * q + e][r] = acc[t][e] * winv;
    __syncthreads();
    const int M = a.M, N = a.N;
    if (a.direct && a.e.y_h2) {  // 8 consecutive columns per thread -> one h2 group record
        for (int o = tid; o < M * 2; o += 64 * SK_WAVES) {
            const int m = o >> 1, c0 = 8 * (o & 1), n = n0 + c0;
            if (n >= N) continue;
            float v[8];
            const float bj[8] = {bia0.x, bia0.y, bia0.z, bia0.w, bia1.x, bia1.y, bia1.z, bia1.w};
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                float s = red[0][m][c0 + j];
#pragma unroll
                for (int w = 1; w < SK_WAVES; ++w) s += red[w][m][c0 + j];
                if (a.e.b) s += o == tid ? bj[j] : a.e.b[n + j];
                if (a.e.resid) s += a.e.resid[(size_t)m * N + n + j];
                v[j] = sk_act(s, a.e.act);
            }
            bool bad = false;
#pragma unroll
            for (int j = 0; j < 8; ++j) bad = bad || h2_bad(v[j]);
            store4_h2(static_cast<char*>(a.e.y_h2), (size_t)m * N * 4, n >> 2, make_float4(v[0], v[1], v[2], v[3]));
            store4_h2(static_cast<char*>(a.e.y_h2), (size_t)m * N * 4, (n >> 2) + 1,
                      make_float4(v[4], v[5], v[6], v[7]));
            h2_flag(a.e.ovf, bad);
        }
        return;
    }
    for (int o = tid; o < M * 16; o += 64 * SK_WAVES) {
        const int m = o >> 4, c = o & 15, n = n0 + c;
        float v = red[0][m][c];
#pragma unroll
        for (int w = 1; w < SK_WAVES; ++w) v += red[w][m][c];
        if (n >= N) continue;
        const size_t i = (size_t)m * N + n;
        if (!a.direct) {
            a.part[(size_t)sidx * M * N + i] = v;
            continue;
        }
        if (a.e.b) v += a.e.b[n];
        if (a.e.resid) v += a.e.resid[i];
        v = sk_act(v, a.e.act);
        if (a.e.z) a.e.z[i] = ddim_z(a.e.z[i], v, a.e.abar_t, a.e.abar_prev, a.e.last);
        else a.e.y[i] = v;
    }
}

// Wide form (round 5): a workgroup is 4 waves, each on CT column tiles (16 CT columns) x its own K slice
// of 32 NC values, so the activation fragments a wave loads serve CT tiles instead of one.  What bounds a
// DDIM-sized launch is the count of load instructions reaching the CUs, not the HBM stream
// (tools/probe/skinny_probe.hip, profiles/r05_o_skinny_probe.txt: without its loads the one-tile form
// takes 2.6 of its 10.3 us, and at 36 rows the activation fragments are 3x the weights' loads), so
// sharing them across tiles is the lever.  Always writes partial planes (S = K / (128 NC) chunks: 256
// workgroups at fc2 of the w1024 prior); the reduce (k_sk_reduce_ln) adds bias, residual and LayerNorm.
// Used for partial planes only: at fc1 (K = 1,024) the extra reduce launch an h2 epilogue would need costs
// more than the form saves (r05_o: 8.2 + 5.0 us vs the one-chunk form's 10.3 with its epilogue inside).  Same per-wave MFMA order as k_skinny_h2 (k order within a wave's slice), a
// fixed wave order in the workgroup and a fixed chunk order in the reduce: deterministic.
constexpr int SKW_WAVES = 4;
constexpr int SKW_NC = 2, SKW_CT = 4;
template <int MT, int NC, int CT>
__global__ __launch_bounds__(64 * SKW_WAVES) void k_skinny_h2w(SkH2Args a) {
    __shared__ float red[SKW_WAVES][16 * MT][16 * CT + 1];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int r = lane & 15, q = lane >> 4;
    const int n0 = blockIdx.x * 16 * CT;
    const int sidx = blockIdx.y;
    const int K = a.K, G = K / 8;
    const int npad = (a.N + 15) / 16 * 16;  // packed weight rows
    const int kw0 = sidx * SKW_WAVES * 32 * NC + wv * 32 * NC;
    const int kend = min(K, kw0 + 32 * NC);
    uint4 wh[CT][NC], wl[CT][NC], xh[NC][MT], xl[NC][MT];
    float winv[CT];
#pragma unroll
    for (int j = 0; j < CT; ++j) {
        const int n = min(n0 + 16 * j + r, npad - 1);  // rows past the pack re-read its last row (discarded)
        winv[j] = a.winv[min(n, a.N - 1)];
        const char* wr = a.w + ((size_t)n * G + q) * 32;
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            const int kc = min(kw0 + 32 * c, K - 32);
            const char* p = wr + (size_t)(kc / 8) * 32;
            wh[j][c] = *reinterpret_cast<const uint4*>(p);
            wl[j][c] = *reinterpret_cast<const uint4*>(p + 16);
        }
    }
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        const int kb = kw0 + 32 * c;
        const int kc = min(kb, K - 32);
        const bool live = kb < kend;
#pragma unroll
        for (int t = 0; t < MT; ++t) {
            const char* p = a.x + ((size_t)min(16 * t + r, a.M - 1) * G + kc / 8 + q) * 32;
            const char* src = live ? p : reinterpret_cast<const char*>(sk_zero8);
            xh[c][t] = *reinterpret_cast<const uint4*>(src);
            xl[c][t] = *reinterpret_cast<const uint4*>(src + 16);
        }
    }
    __builtin_amdgcn_sched_barrier(0);  // all loads in flight first (k_skinny)
    f32x4 acc[CT][MT];
#pragma unroll
    for (int j = 0; j < CT; ++j)
#pragma unroll
        for (int t = 0; t < MT; ++t) acc[j][t] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
        for (int j = 0; j < CT; ++j) {
            const h8 bh = __builtin_bit_cast(h8, wh[j][c]), bl = __builtin_bit_cast(h8, wl[j][c]);
#pragma unroll
            for (int t = 0; t < MT; ++t) {
                const h8 ah = __builtin_bit_cast(h8, xh[c][t]), al = __builtin_bit_cast(h8, xl[c][t]);
                acc[j][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl, acc[j][t], 0, 0, 0);
                acc[j][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh, acc[j][t], 0, 0, 0);
                acc[j][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, acc[j][t], 0, 0, 0);
            }
        }
#pragma unroll
    for (int j = 0; j < CT; ++j)
#pragma unroll
        for (int t = 0; t < MT; ++t)
#pragma unroll
            for (int e = 0; e < 4; ++e) red[wv][16 * t + 4 * q + e][16 * j + r] = acc[j][t][e] * winv[j];
    __syncthreads();
    const int M = a.M, N = a.N;  // N % 8 == 0 (skinny_h2_wide)
    float* part = a.part + (size_t)sidx * M * N;
    for (int o = tid; o < M * 2 * CT; o += 64 * SKW_WAVES) {  // (row, 8 columns), two 16-B stores
        const int m = o / (2 * CT), c0 = 8 * (o - (o / (2 * CT)) * (2 * CT)), n = n0 + c0;
        if (n >= N) continue;
        float v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            float s = red[0][m][c0 + k];
#pragma unroll
            for (int w = 1; w < SKW_WAVES; ++w) s += red[w][m][c0 + k];
            v[k] = s;
        }
        *reinterpret_cast<float4*>(part + (size_t)m * N + n) = make_float4(v[0], v[1], v[2], v[3]);
        *reinterpret_cast<float4*>(part + (size_t)m * N + n + 4) = make_float4(v[4], v[5], v[6], v[7]);
    }
}

typedef void (*SkH2Kernel)(SkH2Args);

SkH2Kernel sk_h2_kernel(int mt, int nc) {
#define TCX_SKH(MT_) nc == 1 ? k_skinny_h2<MT_, 1> : nc == 2 ? k_skinny_h2<MT_, 2> : k_skinny_h2<MT_, 4>
    return mt == 1 ? TCX_SKH(1) : mt == 2 ? TCX_SKH(2) : mt == 3 ? TCX_SKH(3) : TCX_SKH(4);
#undef TCX_SKH
}

int nc_for(int K) {
    int nc = 1;
    while (nc < 4 && SK_WAVES * 32 * nc < K) nc *= 2;
    return nc;
}

// the wide form serves the prior's split-K trunk linear (fc2: N >= 1024 -> >= 16 column groups of 64,
// K / 256 chunks)
bool skinny_h2_wide(int N, int K) {
    static const bool off = getenv("TCX_SKINNY_WIDE") && getenv("TCX_SKINNY_WIDE")[0] == '0';  // A/B
    return !off && N >= 1024 && N % 8 == 0 && K % (SKW_WAVES * 32 * SKW_NC) == 0;
}

int launch_h2w(const void* xh, int K, const void* wh, const float* winv, int M, int N, float* part, hipStream_t st) {
    SkH2Args a{};
    a.x = static_cast<const char*>(xh); a.w = static_cast<const char*>(wh); a.winv = winv;
    a.K = K; a.M = M; a.N = N; a.part = part;
    const int mt = cdiv(M, 16);
    const dim3 grid(cdiv(N, 16 * SKW_CT), K / (SKW_WAVES * 32 * SKW_NC));
    auto k = mt == 1 ? k_skinny_h2w<1, SKW_NC, SKW_CT> : mt == 2 ? k_skinny_h2w<2, SKW_NC, SKW_CT>
           : mt == 3 ? k_skinny_h2w<3, SKW_NC, SKW_CT> : k_skinny_h2w<4, SKW_NC, SKW_CT>;
    hipLaunchKernelGGL(k, grid, dim3(64 * SKW_WAVES), 0, st, a);
    return check_launch("skinny linear (f16x3, wide)");
}

int launch_h2(const void* xh, int K, const void* wh, const float* winv, int M, int N, float* part, const SkEpi* direct,
              hipStream_t st) {
    SkH2Args a{};
    a.x = static_cast<const char*>(xh); a.w = static_cast<const char*>(wh); a.winv = winv;
    a.K = K; a.M = M; a.N = N; a.part = part;
    a.direct = direct != nullptr;
    if (direct) a.e = *direct;
    const int nc = nc_for(K);
    hipLaunchKernelGGL(sk_h2_kernel(cdiv(M, 16), nc), dim3(cdiv(N, 16), cdiv(K, SK_WAVES * 32 * nc)),
                       dim3(64 * SK_WAVES), 0, st, a);
    return check_launch("skinny linear (f16x3)");
}

// W [n][k] fp32 -> h2 rows [npad16][kpad32/8][2][8] scaled by 2^s (row max in [2^14, 2^15)), winv = 2^-s
__global__ __launch_bounds__(256) void k_pack_linear_h2(const float* __restrict__ w, int n, int k, int kp,
                                                        char* __restrict__ wh, float* __restrict__ winv) {
    __shared__ float red[4];
    const int row = blockIdx.x, tid = threadIdx.x;
    float mx = 0.f;
    if (row < n)
        for (int i = tid; i < k; i += 256) mx = fmaxf(mx, fabsf(w[(size_t)row * k + i]));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
    if ((tid & 63) == 0) red[tid >> 6] = mx;
    __syncthreads();
    mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    int e = 0;
    if (mx > 0.f) {
        frexpf(mx, &e);  // mx in [2^(e-1), 2^e)
        e = min(max(15 - e, -100), 100);
    }
    const float sc = ldexpf(1.f, e);
    if (tid == 0) winv[row] = ldexpf(1.f, -e);
    for (int g4 = tid; g4 < kp / 4; g4 += 256) {
        const int i = 4 * g4;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (row < n) {
            const float* src = w + (size_t)row * k;
            v.x = i < k ? src[i] * sc : 0.f;
            v.y = i + 1 < k ? src[i + 1] * sc : 0.f;
            v.z = i + 2 < k ? src[i + 2] * sc : 0.f;
            v.w = i + 3 < k ? src[i + 3] * sc : 0.f;
        }
        store4_h2(wh, (size_t)row * kp * 4, g4, v);
    }
}

typedef void (*SkKernel)(SkArgs);

SkKernel sk_kernel(int mt, int nb) {
#define TCX_SKR(MT_) nb == 2 ? k_skinny<MT_, 2> : nb == 4 ? k_skinny<MT_, 4> : k_skinny<MT_, 8>
    return mt == 1 ? TCX_SKR(1) : mt == 2 ? TCX_SKR(2) : mt == 3 ? TCX_SKR(3) : TCX_SKR(4);
#undef TCX_SKR
}

int nb_for(int K) {
    int nb = 2;
    while (nb < 8 && SK_WAVES * 16 * nb < K) nb *= 2;
    return nb;
}

int launch_src(const float* x, int ldx, int K, int nb, int s, const float* w, int kpad, int M, int N, float* part,
               const SkEpi* direct, hipStream_t st) {
    SkArgs a{};
    a.x = x; a.ldx = ldx; a.K = K; a.w = w; a.kpad = kpad; a.M = M; a.N = N; a.part = part;
    a.direct = direct != nullptr;
    if (direct) a.e = *direct;
    hipLaunchKernelGGL(sk_kernel(cdiv(M, 16), nb), dim3(cdiv(N, 16), s), dim3(64 * SK_WAVES), 0, st, a);
    return check_launch("skinny linear");
}

__device__ __forceinline__ float sk_act(float v, int act) {
    if (act == 1) return fmaxf(v, 0.f);
    if (act == 2) return 1.f / (1.f + expf(-v));
    if (act == 3) return silu_f(v);
    return v;
}

// k_ddim_step's arithmetic (train.hip) on one element
__device__ __forceinline__ float ddim_z(float z, float e, float abar_t, float abar_prev, int last) {
    const float sa = sqrtf(abar_t), s1 = sqrtf(1.0f - abar_t);
    const float sp = sqrtf(abar_prev), s1p = sqrtf(1.0f - abar_prev);
    const float z0 = (z - s1 * e) / (sa + 1e-8f);
    return last ? z0 : sp * z0 + s1p * e;
}

// one row block x 1024 columns, float4 along n (N % 4 == 0)
template <bool DDIM>
__global__ __launch_bounds__(256) void k_sk_reduce4(const float* __restrict__ part, int S, int M, int N, SkEpi e) {
    const int m = blockIdx.y;
    const int n = blockIdx.x * 1024 + threadIdx.x * 4;
    if (n >= N) return;
    const size_t MN = (size_t)M * N, i = (size_t)m * N + n;
    float4 v = *reinterpret_cast<const float4*>(part + i);
#pragma unroll 4
    for (int s = 1; s < S; ++s) {
        const float4 u = *reinterpret_cast<const float4*>(part + (size_t)s * MN + i);
        v.x += u.x; v.y += u.y; v.z += u.z; v.w += u.w;
    }
    float o[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if (e.b) o[k] += e.b[n + k];
        if (e.resid) o[k] += e.resid[i + k];
        o[k] = sk_act(o[k], e.act);
    }
    if (DDIM) {
        float4 z = *reinterpret_cast<const float4*>(e.z + i);
        z.x = ddim_z(z.x, o[0], e.abar_t, e.abar_prev, e.last);
        z.y = ddim_z(z.y, o[1], e.abar_t, e.abar_prev, e.last);
        z.z = ddim_z(z.z, o[2], e.abar_t, e.abar_prev, e.last);
        z.w = ddim_z(z.w, o[3], e.abar_t, e.abar_prev, e.last);
        *reinterpret_cast<float4*>(e.z + i) = z;
    } else {
        *reinterpret_cast<float4*>(e.y + i) = make_float4(o[0], o[1], o[2], o[3]);
    }
}

template <bool DDIM>
__global__ __launch_bounds__(256) void k_sk_reduce1(const float* __restrict__ part, int S, int M, int N, SkEpi e) {
    const int m = blockIdx.y;
    const int n = blockIdx.x * 256 + threadIdx.x;
    if (n >= N) return;
    const size_t MN = (size_t)M * N, i = (size_t)m * N + n;
    float v = part[i];
#pragma unroll 4
    for (int s = 1; s < S; ++s) v += part[(size_t)s * MN + i];
    if (e.b) v += e.b[n];
    if (e.resid) v += e.resid[i];
    v = sk_act(v, e.act);
    if (DDIM) e.z[i] = ddim_z(e.z[i], v, e.abar_t, e.abar_prev, e.last);
    else e.y[i] = v;
}

// one workgroup per row: reduce + bias + resid -> y, then LayerNorm (+FiLM) -> yn (k_layernorm_film's
// arithmetic: fp64 sum / sum of squares, var = E[x^2] - mean^2, float rstd)
template <int V>  // float4 per thread: N <= 1024 V
__global__ __launch_bounds__(256) void k_sk_reduce_ln(const float* __restrict__ part, int S, int M, int N, SkEpi e,
                                                      SkLn ln) {
    __shared__ double red[2][4];
    const int m = blockIdx.x, tid = threadIdx.x;
    const size_t MN = (size_t)M * N;
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
    // every operand of the row is requested up front (one memory round trip instead of three)
    // (round 6: the bias and residual rows too -- they were a third round trip after the partial planes)
    float4 h[V], w4[V], b4[V], g4[V], e4[V], t4[V], r4[V];
#pragma unroll
    for (int v = 0; v < V; ++v) {
        const int n = 4 * tid + 1024 * v;
        h[v] = w4[v] = b4[v] = g4[v] = e4[v] = t4[v] = r4[v] = z4;
        if (n < N) {
            const size_t i = (size_t)m * N + n;
            float4 a = *reinterpret_cast<const float4*>(part + i);
            h[v] = a;
            // unconditional loads from a valid row (a branch around a load made the compiler wait on it)
            t4[v] = *reinterpret_cast<const float4*>((e.b ? e.b : ln.lw) + n);
            r4[v] = *reinterpret_cast<const float4*>((e.resid ? e.resid : part) + i);
            w4[v] = *reinterpret_cast<const float4*>(ln.lw + n);
            b4[v] = *reinterpret_cast<const float4*>(ln.lb + n);
            if (ln.gy) {
                const float* gr = ln.gy + (size_t)m * ln.ld_gy;
                g4[v] = *reinterpret_cast<const float4*>(gr + n);
                e4[v] = *reinterpret_cast<const float4*>(gr + N + n);
                if (ln.gt) {
                    const float4 tg = *reinterpret_cast<const float4*>(ln.gt + n);
                    const float4 te = *reinterpret_cast<const float4*>(ln.gt + N + n);
                    g4[v].x += tg.x; g4[v].y += tg.y; g4[v].z += tg.z; g4[v].w += tg.w;
                    e4[v].x += te.x; e4[v].y += te.y; e4[v].z += te.z; e4[v].w += te.w;
                }
            }
        }
    }
    double s = 0, q = 0;
#pragma unroll
    for (int v = 0; v < V; ++v) {
        const int n = 4 * tid + 1024 * v;
        if (n < N) {
            const size_t i = (size_t)m * N + n;
            float4 a = h[v];
            // partial planes CH at a time, every load of a chunk issued before its adds (the same order of adds)
            constexpr int CH = V == 1 ? 8 : 2;
            for (int p0 = 1; p0 < S; p0 += CH) {
                float4 u[CH];
#pragma unroll
                for (int j = 0; j < CH; ++j)  // (past the last plane: a reload of it, never added)
                    u[j] = *reinterpret_cast<const float4*>(part + (size_t)min(p0 + j, S - 1) * MN + i);
#pragma unroll
                for (int j = 0; j < CH; ++j)
                    if (p0 + j < S) { a.x += u[j].x; a.y += u[j].y; a.z += u[j].z; a.w += u[j].w; }
            }
            if (e.b) { a.x += t4[v].x; a.y += t4[v].y; a.z += t4[v].z; a.w += t4[v].w; }
            if (e.resid) { a.x += r4[v].x; a.y += r4[v].y; a.z += r4[v].z; a.w += r4[v].w; }
            *reinterpret_cast<float4*>(e.y + i) = a;
            h[v] = a;
            const double a0 = a.x, a1 = a.y, a2 = a.z, a3 = a.w;
            s += (a0 + a1) + (a2 + a3);
            q += (a0 * a0 + a1 * a1) + (a2 * a2 + a3 * a3);
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        s += __shfl_xor(s, o);
        q += __shfl_xor(q, o);
    }
    if ((tid & 63) == 0) {
        red[0][tid >> 6] = s;
        red[1][tid >> 6] = q;
    }
    __syncthreads();
    s = (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
    q = (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
    const double mean = s / N;
    double var = q / N - mean * mean;
    var = var < 0 ? 0 : var;
    const float rstd = (float)(1.0 / sqrt(var + (double)ln.eps));
    const float mf = (float)mean;
#pragma unroll
    for (int v = 0; v < V; ++v) {
        const int n = 4 * tid + 1024 * v;
        if (n < N) {
            float o[4] = {(h[v].x - mf) * rstd * w4[v].x + b4[v].x, (h[v].y - mf) * rstd * w4[v].y + b4[v].y,
                          (h[v].z - mf) * rstd * w4[v].z + b4[v].z, (h[v].w - mf) * rstd * w4[v].w + b4[v].w};
            if (ln.gy) {
                o[0] = o[0] * (1.f + g4[v].x) + e4[v].x; o[1] = o[1] * (1.f + g4[v].y) + e4[v].y;
                o[2] = o[2] * (1.f + g4[v].z) + e4[v].z; o[3] = o[3] * (1.f + g4[v].w) + e4[v].w;
            }
            const float4 ov = make_float4(o[0], o[1], o[2], o[3]);
            if (ln.yn_h2) {
                store4_h2(static_cast<char*>(ln.yn_h2), (size_t)m * N * 4, n >> 2, ov);
                h2_flag(ln.ovf, h2_bad(o[0]) || h2_bad(o[1]) || h2_bad(o[2]) || h2_bad(o[3]));
            } else {
                *reinterpret_cast<float4*>(ln.yn + (size_t)m * N + n) = ov;
            }
        }
    }
}

}  // namespace

bool skinny_ok(int M, int N, int K1, int K2) {
    static const bool off = getenv("TCX_NO_SKINNY") != nullptr;  // A/B: the 128-row split-K path
    return !off && M >= 1 && M <= 64 && N >= 1 && K1 >= 16 && K1 % 16 == 0 && K2 >= 0 && K2 % 16 == 0;
}

SkPlan skinny_plan(int K1, int K2) {
    SkPlan p{};
    p.nb1 = nb_for(K1);
    p.s1 = cdiv(K1, SK_WAVES * 16 * p.nb1);
    if (K2 > 0) {
        p.nb2 = nb_for(K2);
        p.s2 = cdiv(K2, SK_WAVES * 16 * p.nb2);
    }
    return p;
}

int skinny_partials(const float* x1, int ldx1, int K1, const float* x2, int ldx2, int K2, const float* w, int kpad,
                    int M, int N, const SkPlan& p, float* part, hipStream_t st) {
    TCX_REQUIRE(x1 && w && part && M >= 1 && M <= 64 && N >= 1 && (K2 == 0 || x2), "skinny linear: bad args");
    TCX_REQUIRE(aligned16(x1) && (!x2 || aligned16(x2)) && aligned16(w) && ldx1 % 4 == 0 && ldx2 % 4 == 0 &&
                    kpad % 4 == 0 && kpad >= K1 + K2,
                "skinny linear: 16-B alignment of x / W rows");
    TCX_TRY(launch_src(x1, ldx1, K1, p.nb1, p.s1, w, kpad, M, N, part, nullptr, st));
    if (K2 > 0)
        TCX_TRY(launch_src(x2, ldx2, K2, p.nb2, p.s2, w + K1, kpad, M, N, part + (size_t)p.s1 * M * N, nullptr, st));
    return TCX_OK;
}

int skinny_linear(const float* x1, int ldx1, int K1, const float* x2, int ldx2, int K2, const float* w, int kpad,
                  int M, int N, float* part, const SkEpi& e, hipStream_t st) {
    const SkPlan p = skinny_plan(K1, K2);
    if (p.s1 + p.s2 == 1) {  // one chunk: the epilogue runs in the GEMM kernel
        TCX_REQUIRE(x1 && w && M >= 1 && M <= 64 && N >= 1 && aligned16(x1) && aligned16(w) && ldx1 % 4 == 0 &&
                        kpad % 4 == 0 && kpad >= K1 && (e.z || e.y),
                    "skinny linear: bad args");
        return launch_src(x1, ldx1, K1, p.nb1, 1, w, kpad, M, N, nullptr, &e, st);
    }
    TCX_TRY(skinny_partials(x1, ldx1, K1, x2, ldx2, K2, w, kpad, M, N, p, part, st));
    return skinny_reduce(part, p.s1 + p.s2, M, N, e, st);
}

int skinny_reduce(const float* part, int S, int M, int N, const SkEpi& e, hipStream_t st) {
    const bool ddim = e.z != nullptr;
    TCX_REQUIRE(part && S >= 1 && (ddim || e.y), "skinny reduce: bad args");
    const bool vec = N % 4 == 0 && aligned16(part) && (!e.resid || aligned16(e.resid)) && (!e.y || aligned16(e.y)) &&
                     (!e.z || aligned16(e.z));
    if (vec) {
        const dim3 grid(cdiv(N, 1024), M);
        if (ddim) hipLaunchKernelGGL(k_sk_reduce4<true>, grid, dim3(256), 0, st, part, S, M, N, e);
        else hipLaunchKernelGGL(k_sk_reduce4<false>, grid, dim3(256), 0, st, part, S, M, N, e);
    } else {
        const dim3 grid(cdiv(N, 256), M);
        if (ddim) hipLaunchKernelGGL(k_sk_reduce1<true>, grid, dim3(256), 0, st, part, S, M, N, e);
        else hipLaunchKernelGGL(k_sk_reduce1<false>, grid, dim3(256), 0, st, part, S, M, N, e);
    }
    return check_launch("skinny reduce");
}

bool skinny_h2_ok(int M, int N, int K) {
    static const bool off = getenv("TCX_NO_SKINNY") != nullptr;
    return !off && M >= 1 && M <= 64 && N >= 1 && K >= 32 && K % 32 == 0;
}

// partial planes of skinny_h2_partials (the wide form where it applies) / of skinny_h2_linear's split-K
int skinny_h2_chunks(int N, int K) {
    return skinny_h2_wide(N, K) ? K / (SKW_WAVES * 32 * SKW_NC) : cdiv(K, SK_WAVES * 32 * nc_for(K));
}
int skinny_h2_chunks_linear(int K) { return cdiv(K, SK_WAVES * 32 * nc_for(K)); }

size_t skinny_h2_part_floats(int M, int N, int K) {
    return (size_t)std::max(skinny_h2_chunks(N, K), skinny_h2_chunks_linear(K)) * M * N;
}

int skinny_h2_partials(const void* xh, int K, const void* wh, const float* winv, int M, int N, float* part,
                       hipStream_t st) {
    TCX_REQUIRE(xh && wh && winv && part && skinny_h2_ok(M, N, K) && aligned16(xh) && aligned16(wh),
                "skinny linear (f16x3): bad args");
    if (skinny_h2_wide(N, K)) return launch_h2w(xh, K, wh, winv, M, N, part, st);
    return launch_h2(xh, K, wh, winv, M, N, part, nullptr, st);
}

int skinny_h2_linear(const void* xh, int K, const void* wh, const float* winv, int M, int N, float* part,
                     const SkEpi& e, hipStream_t st) {
    TCX_REQUIRE(xh && wh && winv && skinny_h2_ok(M, N, K) && aligned16(xh) && aligned16(wh) &&
                    (e.y || e.z || e.y_h2) && (!e.y_h2 || (N % 8 == 0 && aligned16(e.y_h2) && (!e.b || aligned16(e.b)))),
                "skinny linear (f16x3): bad args");
    if (skinny_h2_chunks_linear(K) == 1) return launch_h2(xh, K, wh, winv, M, N, nullptr, &e, st);
    TCX_REQUIRE(part && !e.y_h2, "skinny linear (f16x3): split-K needs scratch and an fp32 output");
    TCX_TRY(launch_h2(xh, K, wh, winv, M, N, part, nullptr, st));
    return skinny_reduce(part, skinny_h2_chunks_linear(K), M, N, e, st);
}

bool skinny_ln_ok(int N) { return N % 4 == 0 && N <= 4096; }

int skinny_reduce_ln(const float* part, int S, int M, int N, const SkEpi& e, const SkLn& ln, hipStream_t st) {
    TCX_REQUIRE(part && S >= 1 && e.y && (ln.yn || ln.yn_h2) && ln.lw && ln.lb && skinny_ln_ok(N) && e.act == 0 &&
                    (!ln.yn_h2 || (N % 8 == 0 && aligned16(ln.yn_h2))),
                "skinny reduce+LayerNorm: bad args");
    TCX_REQUIRE(aligned16(part) && aligned16(e.y) && aligned16(ln.lw) && aligned16(ln.lb) &&
                    (!e.b || aligned16(e.b)) && (!e.resid || aligned16(e.resid)) &&
                    (!ln.gy || (aligned16(ln.gy) && ln.ld_gy % 4 == 0)) && (!ln.gt || aligned16(ln.gt)) &&
                    (!ln.yn || aligned16(ln.yn)),
                "skinny reduce+LayerNorm: 16-B alignment");
    if (N <= 1024) hipLaunchKernelGGL(k_sk_reduce_ln<1>, dim3(M), dim3(256), 0, st, part, S, M, N, e, ln);
    else hipLaunchKernelGGL(k_sk_reduce_ln<4>, dim3(M), dim3(256), 0, st, part, S, M, N, e, ln);
    return check_launch("skinny reduce+LayerNorm");
}

}  // namespace tcx

extern "C" size_t tcx_linear_h2_bytes(int n, int k) {
    if (n <= 0 || k <= 0) return 0;
    return (size_t)tcx::cdiv(n, 16) * 16 * (size_t)tcx::cdiv(k, 32) * 32 * 4;
}

extern "C" int tcx_pack_linear_h2(const float* w, int n, int k, void* wh, float* winv, void* stream) {
    TCX_REQUIRE(w && wh && winv && n > 0 && k > 0 && tcx::aligned16(wh), "tcx_pack_linear_h2: bad args");
    const int np = tcx::cdiv(n, 16) * 16, kp = tcx::cdiv(k, 32) * 32;
    hipLaunchKernelGGL(tcx::k_pack_linear_h2, dim3(np), dim3(256), 0, (hipStream_t)stream, w, n, k, kp,
                       static_cast<char*>(wh), winv);
    return tcx::check_launch("tcx_pack_linear_h2");
}
