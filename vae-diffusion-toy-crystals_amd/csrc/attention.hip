// Bottleneck self-attention of SelfAttention2d (/root/reference/src/toycrystals/models/
// sde_score_model.py:136-167): per (batch, head) softmax(q k^T / sqrt(d)) v over N = H*W
// tokens (N = 256, d = 48 at base_ch 96).  K and V of one head fit LDS whole (2 x 48 KB), so
// one pass with an exact (non-online) softmax: 4 lanes per query row, each owning every 4th key;
// row max / sum and the output by two xor-shuffles.  The q,k,v channel split and the head-major
// channel order (view [B,heads,d,N] -> transpose) are folded into the addressing.
#include "common.hpp"
#include "h2.hpp"

namespace tcx {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

// ---------------------------------------------------------------------------------------------
// MFMA attention (fp32 v_mfma_f32_32x32x2_f32): one block per (head, batch), one wave per 32
// queries, K and V of the head staged in LDS once.
//   S^T = K Q^T : A = K rows (keys) from LDS, B = Q^T held in registers (query on the lane);
//                 the K-dim d is split by lane half: half h owns d in [h*D/2, (h+1)*D/2).
//   softmax over keys = over the 16 accumulator registers x N/32 tiles of a lane + one xor-32
//                 shuffle (both lane halves hold the same query).
//   O^T = V^T P^T: the probability accumulators ARE the B operands (key = (r&3)+8(r>>2)+4h of
//                 tile n, query on the lane), A = V^T read from LDS with the same key order.
// ---------------------------------------------------------------------------------------------
template <int D>
__global__ __launch_bounds__(512) void k_attention_mfma(const float* __restrict__ qkv, float* __restrict__ out, int N,
                                                        int C, float scale, int out_h2, unsigned* ovf) {
    constexpr int HD = D / 2;           // d per lane half
    constexpr int KS = D + 4;           // K row stride in LDS ((D+4)/4 odd: conflict-free b128)
    constexpr int DT = (D + 31) / 32;   // 32-row tiles of O^T
    constexpr int VS = DT * 32;         // V row stride (zero padded to the tile)
    constexpr int MAXT = 8;             // key tiles (N <= 256)
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float* Ks = sm;
    float* Vs = sm + (size_t)N * KS;
    const int b = blockIdx.y, h = blockIdx.x;
    const int tid = threadIdx.x, nthr = blockDim.x;
    const size_t rs = 3 * (size_t)C;
    const float* base = qkv + (size_t)b * N * rs;
    constexpr int D4 = D / 4;
    for (int i = tid; i < N * D4; i += nthr) {
        const int j = i / D4, d4 = i - (i / D4) * D4;
        const float* src = base + (size_t)j * rs + h * D + d4 * 4;
        *reinterpret_cast<float4*>(Ks + j * KS + d4 * 4) = *reinterpret_cast<const float4*>(src + C);
        *reinterpret_cast<float4*>(Vs + j * VS + d4 * 4) = *reinterpret_cast<const float4*>(src + 2 * C);
    }
    if (VS > D) {
        for (int i = tid; i < N * (VS - D); i += nthr) {
            const int j = i / (VS - D), e = i - (i / (VS - D)) * (VS - D);
            Vs[j * VS + D + e] = 0.f;
        }
    }
    __syncthreads();
    const int lane = tid & 63, w = tid >> 6;
    const int li = lane & 31, lh = lane >> 5;
    const int q = w * 32 + li;
    const int nkt = N / 32;
    // Q^T fragment: this lane's query, d in [HD*lh, HD*lh + HD)
    float qf[HD];
    {
        const float* qs = base + (size_t)q * rs + h * D + HD * lh;
#pragma unroll
        for (int s4 = 0; s4 < HD / 4; ++s4) {
            const float4 v = *reinterpret_cast<const float4*>(qs + 4 * s4);
            qf[4 * s4 + 0] = v.x; qf[4 * s4 + 1] = v.y; qf[4 * s4 + 2] = v.z; qf[4 * s4 + 3] = v.w;
        }
    }
    f32x16 sacc[MAXT];
#pragma unroll
    for (int n = 0; n < MAXT; ++n) {
        sacc[n] = (f32x16){};
        if (n < nkt) {
            const float* kr = Ks + (n * 32 + li) * KS + HD * lh;
#pragma unroll
            for (int s4 = 0; s4 < HD / 4; ++s4) {
                const float4 kv = *reinterpret_cast<const float4*>(kr + 4 * s4);
                sacc[n] = __builtin_amdgcn_mfma_f32_32x32x2f32(kv.x, qf[4 * s4 + 0], sacc[n], 0, 0, 0);
                sacc[n] = __builtin_amdgcn_mfma_f32_32x32x2f32(kv.y, qf[4 * s4 + 1], sacc[n], 0, 0, 0);
                sacc[n] = __builtin_amdgcn_mfma_f32_32x32x2f32(kv.z, qf[4 * s4 + 2], sacc[n], 0, 0, 0);
                sacc[n] = __builtin_amdgcn_mfma_f32_32x32x2f32(kv.w, qf[4 * s4 + 3], sacc[n], 0, 0, 0);
            }
        }
    }
    // softmax over the keys of query q: exp((s - max) * scale), scale = 1/sqrt(D) > 0
    float m = -INFINITY;
#pragma unroll
    for (int n = 0; n < MAXT; ++n)
        if (n < nkt) {
#pragma unroll
            for (int r = 0; r < 16; ++r) m = fmaxf(m, sacc[n][r]);
        }
    m = fmaxf(m, __shfl_xor(m, 32));
    float l = 0.f;
#pragma unroll
    for (int n = 0; n < MAXT; ++n)
        if (n < nkt) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float pv = expf((sacc[n][r] - m) * scale);
                sacc[n][r] = pv;
                l += pv;
            }
        }
    l += __shfl_xor(l, 32);
    // O^T[d][q] = sum_key V[key][d] P^T[key][q]
    f32x16 oacc[DT];
#pragma unroll
    for (int t = 0; t < DT; ++t) oacc[t] = (f32x16){};
#pragma unroll
    for (int n = 0; n < MAXT; ++n)
        if (n < nkt) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int key = n * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
                const float* vr = Vs + key * VS + li;
#pragma unroll
                for (int t = 0; t < DT; ++t)
                    oacc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(vr[t * 32], sacc[n][r], oacc[t], 0, 0, 0);
            }
        }
    const float inv = 1.f / l;
    if (out_h2) {  // h2 split record of the query's pixel (h2.hpp): 4 consecutive d per register quad
        bool bad = false;
#pragma unroll
        for (int t = 0; t < DT; ++t)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int d = t * 32 + 8 * i + 4 * lh;
                if (d < D) {
                    const float4 v = make_float4(oacc[t][4 * i] * inv, oacc[t][4 * i + 1] * inv, oacc[t][4 * i + 2] * inv,
                                                 oacc[t][4 * i + 3] * inv);
                    store4_h2(reinterpret_cast<char*>(out), ((size_t)b * N + q) * C * 4, (h * D + d) >> 2, v);
                    bad = bad || h2_bad(v.x) || h2_bad(v.y) || h2_bad(v.z) || h2_bad(v.w);
                }
            }
        h2_flag(ovf, bad);
        return;
    }
    float* dst = out + ((size_t)b * N + q) * C + h * D;
#pragma unroll
    for (int t = 0; t < DT; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int d = t * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
            if (d < D) dst[d] = oacc[t][r] * inv;
        }
}

// ---------------------------------------------------------------------------------------------
// Key-tiled (flash) form for long sequences (the 256x256 U-Net's bottleneck: N = 64*64 = 4096):
// grid (N/256 query blocks, heads, Bt), 8 waves x 32 queries; K and V staged in LDS 128 keys at a
// time; per query (on the lane) a running max m, sum l and O^T accumulators rescaled by
// exp((m_old - m_new) * scale) when a tile raises the max.  Same fp32 MFMA products as
// k_attention_mfma; exact softmax up to the rescaling roundings.
// ---------------------------------------------------------------------------------------------
template <int D>
__global__ __launch_bounds__(512) void k_attention_flash(const float* __restrict__ qkv, float* __restrict__ out, int N,
                                                         int C, float scale, int out_h2, unsigned* ovf) {
    constexpr int HD = D / 2;
    constexpr int KS = D + 4;
    constexpr int DT = (D + 31) / 32;
    constexpr int VS = DT * 32;
    constexpr int KT = 128;        // keys per staged tile
    constexpr int NST = KT / 32;   // 32-key sub-tiles
    __shared__ __attribute__((aligned(16))) float Ks[KT * KS];
    __shared__ __attribute__((aligned(16))) float Vs[KT * VS];
    const int b = blockIdx.z, h = blockIdx.y;
    const int tid = threadIdx.x;
    const size_t rs = 3 * (size_t)C;
    const float* base = qkv + (size_t)b * N * rs;
    constexpr int D4 = D / 4;
    const int lane = tid & 63, w = tid >> 6;
    const int li = lane & 31, lh = lane >> 5;
    const int q = blockIdx.x * 256 + w * 32 + li;
    float qf[HD];
    {
        const float* qs = base + (size_t)q * rs + h * D + HD * lh;
#pragma unroll
        for (int s4 = 0; s4 < HD / 4; ++s4) {
            const float4 v = *reinterpret_cast<const float4*>(qs + 4 * s4);
            qf[4 * s4 + 0] = v.x; qf[4 * s4 + 1] = v.y; qf[4 * s4 + 2] = v.z; qf[4 * s4 + 3] = v.w;
        }
    }
    if (VS > D) {
        for (int i = tid; i < KT * (VS - D); i += 512) {
            const int j = i / (VS - D), e = i - (i / (VS - D)) * (VS - D);
            Vs[j * VS + D + e] = 0.f;
        }
    }
    f32x16 oacc[DT];
#pragma unroll
    for (int t = 0; t < DT; ++t) oacc[t] = (f32x16){};
    float m = -INFINITY, l = 0.f;
    for (int k0 = 0; k0 < N; k0 += KT) {
        __syncthreads();  // previous tile fully consumed
        for (int i = tid; i < KT * D4; i += 512) {
            const int j = i / D4, d4 = i - (i / D4) * D4;
            const float* src = base + (size_t)(k0 + j) * rs + h * D + d4 * 4;
            *reinterpret_cast<float4*>(Ks + j * KS + d4 * 4) = *reinterpret_cast<const float4*>(src + C);
            *reinterpret_cast<float4*>(Vs + j * VS + d4 * 4) = *reinterpret_cast<const float4*>(src + 2 * C);
        }
        __syncthreads();
        f32x16 sacc[NST];
#pragma unroll
        for (int n = 0; n < NST; ++n) {
            sacc[n] = (f32x16){};
            const float* kr = Ks + (n * 32 + li) * KS + HD * lh;
#pragma unroll
            for (int s4 = 0; s4 < HD / 4; ++s4) {
                const float4 kv = *reinterpret_cast<const float4*>(kr + 4 * s4);
                sacc[n] = __builtin_amdgcn_mfma_f32_32x32x2f32(kv.x, qf[4 * s4 + 0], sacc[n], 0, 0, 0);
                sacc[n] = __builtin_amdgcn_mfma_f32_32x32x2f32(kv.y, qf[4 * s4 + 1], sacc[n], 0, 0, 0);
                sacc[n] = __builtin_amdgcn_mfma_f32_32x32x2f32(kv.z, qf[4 * s4 + 2], sacc[n], 0, 0, 0);
                sacc[n] = __builtin_amdgcn_mfma_f32_32x32x2f32(kv.w, qf[4 * s4 + 3], sacc[n], 0, 0, 0);
            }
        }
        float mt = -INFINITY;
#pragma unroll
        for (int n = 0; n < NST; ++n)
#pragma unroll
            for (int r = 0; r < 16; ++r) mt = fmaxf(mt, sacc[n][r]);
        mt = fmaxf(mt, __shfl_xor(mt, 32));
        const float mn = fmaxf(m, mt);
        const float alpha = expf((m - mn) * scale);  // 0 on the first tile (m = -inf)
        m = mn;
        l *= alpha;
#pragma unroll
        for (int t = 0; t < DT; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) oacc[t][r] *= alpha;
        float lt = 0.f;
#pragma unroll
        for (int n = 0; n < NST; ++n)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float pv = expf((sacc[n][r] - mn) * scale);
                sacc[n][r] = pv;
                lt += pv;
            }
        lt += __shfl_xor(lt, 32);
        l += lt;
#pragma unroll
        for (int n = 0; n < NST; ++n)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int key = n * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
                const float* vr = Vs + key * VS + li;
#pragma unroll
                for (int t = 0; t < DT; ++t)
                    oacc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(vr[t * 32], sacc[n][r], oacc[t], 0, 0, 0);
            }
    }
    const float inv = 1.f / l;
    if (out_h2) {
        bool bad = false;
#pragma unroll
        for (int t = 0; t < DT; ++t)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int d = t * 32 + 8 * i + 4 * lh;
                if (d < D) {
                    const float4 v = make_float4(oacc[t][4 * i] * inv, oacc[t][4 * i + 1] * inv, oacc[t][4 * i + 2] * inv,
                                                 oacc[t][4 * i + 3] * inv);
                    store4_h2(reinterpret_cast<char*>(out), ((size_t)b * N + q) * C * 4, (h * D + d) >> 2, v);
                    bad = bad || h2_bad(v.x) || h2_bad(v.y) || h2_bad(v.z) || h2_bad(v.w);
                }
            }
        h2_flag(ovf, bad);
        return;
    }
    float* dst = out + ((size_t)b * N + q) * C + h * D;
#pragma unroll
    for (int t = 0; t < DT; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int d = t * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
            if (d < D) dst[d] = oacc[t][r] * inv;
        }
}

template <int D>
int launch_attn_flash(const float* qkv, float* out, int Bt, int N, int C, int heads, hipStream_t st, int out_h2,
                      unsigned* ovf) {
    const float scale = (float)(1.0 / std::sqrt((double)D));
    hipLaunchKernelGGL((k_attention_flash<D>), dim3(N / 256, heads, Bt), dim3(512), 0, st, qkv, out, N, C, scale,
                       out_h2, ovf);
    return check_launch("tcx_attention(flash)");
}

template <int D>
int launch_attn_mfma(const float* qkv, float* out, int Bt, int N, int C, int heads, hipStream_t st, int out_h2 = 0,
                     unsigned* ovf = nullptr) {
    const float scale = (float)(1.0 / std::sqrt((double)D));
    constexpr int KS = D + 4, VS = ((D + 31) / 32) * 32;
    const size_t shm = (size_t)N * (KS + VS) * sizeof(float);
    static bool attr_set = false;
    if (!attr_set) {
        if (hipFuncSetAttribute(reinterpret_cast<const void*>(&k_attention_mfma<D>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) != hipSuccess) {
            set_error("tcx_attention: cannot enable 160 KB dynamic LDS");
            return TCX_EHIP;
        }
        attr_set = true;
    }
    hipLaunchKernelGGL((k_attention_mfma<D>), dim3(heads, Bt), dim3(2 * N), shm, st, qkv, out, N, C, scale, out_h2, ovf);
    return check_launch("tcx_attention(mfma)");
}

constexpr int QROWS = 64;  // query rows per block (4 lanes each) of the VALU fallback
constexpr int MAXK = 64;   // keys per lane (N <= 256)

template <int D>
__global__ __launch_bounds__(256) void k_attention(const float* __restrict__ qkv, float* __restrict__ out, int N,
                                                   int C, int heads, float scale) {
    extern __shared__ __attribute__((aligned(16))) float kv[];  // K[N][D], V[N][D]
    float* Ks = kv;
    float* Vs = kv + (size_t)N * D;
    const int b = blockIdx.z, h = blockIdx.y;
    const int tid = threadIdx.x;
    const size_t rowstride = 3 * (size_t)C;
    const float* base = qkv + (size_t)b * N * rowstride;
    // stage K, V (float4 granules)
    constexpr int D4 = D / 4;
    for (int i = tid; i < N * D4; i += 256) {
        const int j = i / D4, d4 = i - (i / D4) * D4;
        const float* src = base + (size_t)j * rowstride + h * D + d4 * 4;
        *reinterpret_cast<float4*>(Ks + j * D + d4 * 4) = *reinterpret_cast<const float4*>(src + C);
        *reinterpret_cast<float4*>(Vs + j * D + d4 * 4) = *reinterpret_cast<const float4*>(src + 2 * C);
    }
    __syncthreads();
    const int sub = tid & 3;
    const int r = blockIdx.x * QROWS + (tid >> 2);
    const bool rv = r < N;
    float q[D];
    {
        const float* qs = base + (size_t)(rv ? r : 0) * rowstride + h * D;
#pragma unroll
        for (int d4 = 0; d4 < D4; ++d4) {
            const float4 v = *reinterpret_cast<const float4*>(qs + d4 * 4);
            q[4 * d4 + 0] = v.x; q[4 * d4 + 1] = v.y; q[4 * d4 + 2] = v.z; q[4 * d4 + 3] = v.w;
        }
    }
    float s[MAXK];
    float mx = -INFINITY;
#pragma unroll
    for (int jj = 0; jj < MAXK; ++jj) {
        const int j = 4 * jj + sub;
        float a = 0.f;
        if (j < N) {
            const float* kr = Ks + j * D;
#pragma unroll
            for (int d4 = 0; d4 < D4; ++d4) {
                const float4 kk = *reinterpret_cast<const float4*>(kr + d4 * 4);
                a = fmaf(q[4 * d4 + 0], kk.x, a);
                a = fmaf(q[4 * d4 + 1], kk.y, a);
                a = fmaf(q[4 * d4 + 2], kk.z, a);
                a = fmaf(q[4 * d4 + 3], kk.w, a);
            }
            a *= scale;
            mx = fmaxf(mx, a);
        }
        s[jj] = a;
    }
    mx = fmaxf(mx, __shfl_xor(mx, 1));
    mx = fmaxf(mx, __shfl_xor(mx, 2));
    float l = 0.f;
    float o[D];
#pragma unroll
    for (int d = 0; d < D; ++d) o[d] = 0.f;
#pragma unroll
    for (int jj = 0; jj < MAXK; ++jj) {
        const int j = 4 * jj + sub;
        if (j < N) {
            const float pj = expf(s[jj] - mx);
            l += pj;
            const float* vr = Vs + j * D;
#pragma unroll
            for (int d4 = 0; d4 < D4; ++d4) {
                const float4 vv = *reinterpret_cast<const float4*>(vr + d4 * 4);
                o[4 * d4 + 0] = fmaf(pj, vv.x, o[4 * d4 + 0]);
                o[4 * d4 + 1] = fmaf(pj, vv.y, o[4 * d4 + 1]);
                o[4 * d4 + 2] = fmaf(pj, vv.z, o[4 * d4 + 2]);
                o[4 * d4 + 3] = fmaf(pj, vv.w, o[4 * d4 + 3]);
            }
        }
    }
    l += __shfl_xor(l, 1);
    l += __shfl_xor(l, 2);
#pragma unroll
    for (int d = 0; d < D; ++d) {
        o[d] += __shfl_xor(o[d], 1);
        o[d] += __shfl_xor(o[d], 2);
    }
    if (rv) {
        const float inv = 1.f / l;
        float* dst = out + ((size_t)b * N + r) * C + h * D;
        // lane `sub` stores the quads d4 = sub, sub+4, ...
#pragma unroll
        for (int d4 = 0; d4 < D4; ++d4) {
            if ((d4 & 3) == sub) {
                *reinterpret_cast<float4*>(dst + d4 * 4) =
                    make_float4(o[4 * d4] * inv, o[4 * d4 + 1] * inv, o[4 * d4 + 2] * inv, o[4 * d4 + 3] * inv);
            }
        }
    }
}

template <int D>
int launch_attn(const float* qkv, float* out, int Bt, int N, int C, int heads, hipStream_t st) {
    const float scale = (float)(1.0 / std::sqrt((double)D));
    const size_t shm = 2 * (size_t)N * D * sizeof(float);
    const dim3 grid(cdiv(N, QROWS), heads, Bt);
    static bool attr_set = false;  // > 64 KB of dynamic LDS needs the explicit opt-in
    if (!attr_set) {
        if (hipFuncSetAttribute(reinterpret_cast<const void*>(&k_attention<D>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) != hipSuccess) {
            set_error("tcx_attention: cannot enable 160 KB dynamic LDS");
            return TCX_EHIP;
        }
        attr_set = true;
    }
    hipLaunchKernelGGL((k_attention<D>), grid, dim3(256), shm, st, qkv, out, N, C, heads, scale);
    return check_launch("tcx_attention");
}

}  // namespace
}  // namespace tcx

using namespace tcx;

extern "C" int tcx_attention(const float* qkv, float* out, int Bt, int N, int C, int heads, void* stream) {
    TCX_REQUIRE(qkv && out && heads > 0 && C % heads == 0, "tcx_attention: bad args");
    TCX_REQUIRE(N > 0 && (N <= 4 * MAXK || N % 256 == 0), "tcx_attention: N must be <= 256 or a multiple of 256");
    TCX_REQUIRE(aligned16(qkv) && aligned16(out), "tcx_attention: pointers must be 16-B aligned");
    if (Bt == 0) return TCX_OK;
    const int D = C / heads;
    hipStream_t st = (hipStream_t)stream;
    if (N > 256) {  // key-tiled flash form
        switch (D) {
            case 16: return launch_attn_flash<16>(qkv, out, Bt, N, C, heads, st, 0, nullptr);
            case 32: return launch_attn_flash<32>(qkv, out, Bt, N, C, heads, st, 0, nullptr);
            case 48: return launch_attn_flash<48>(qkv, out, Bt, N, C, heads, st, 0, nullptr);
            case 64: return launch_attn_flash<64>(qkv, out, Bt, N, C, heads, st, 0, nullptr);
            default: set_error("tcx_attention: head dim %d unsupported for N > 256", D); return TCX_EUNSUP;
        }
    }
    if (N % 32 == 0) {  // MFMA path (every U-Net bottleneck: N = (H/4)*(W/4))
        switch (D) {
            case 8: return launch_attn_mfma<8>(qkv, out, Bt, N, C, heads, st);
            case 16: return launch_attn_mfma<16>(qkv, out, Bt, N, C, heads, st);
            case 24: return launch_attn_mfma<24>(qkv, out, Bt, N, C, heads, st);
            case 32: return launch_attn_mfma<32>(qkv, out, Bt, N, C, heads, st);
            case 48: return launch_attn_mfma<48>(qkv, out, Bt, N, C, heads, st);
            case 64: return launch_attn_mfma<64>(qkv, out, Bt, N, C, heads, st);
            default: break;
        }
    }
    switch (D) {
        case 8: return launch_attn<8>(qkv, out, Bt, N, C, heads, st);
        case 16: return launch_attn<16>(qkv, out, Bt, N, C, heads, st);
        case 24: return launch_attn<24>(qkv, out, Bt, N, C, heads, st);
        case 32: return launch_attn<32>(qkv, out, Bt, N, C, heads, st);
        case 48: return launch_attn<48>(qkv, out, Bt, N, C, heads, st);
        case 64: return launch_attn<64>(qkv, out, Bt, N, C, heads, st);
        default: set_error("tcx_attention: head dim %d unsupported", D); return TCX_EUNSUP;
    }
}

extern "C" int tcx_attention_h2(const float* qkv, void* out, int Bt, int N, int C, int heads, unsigned* ovf,
                                void* stream) {
    TCX_REQUIRE(qkv && out && heads > 0 && C % heads == 0 && C % 8 == 0, "tcx_attention_h2: bad args");
    TCX_REQUIRE(N > 0 && ((N <= 256 && N % 32 == 0) || N % 256 == 0),
                "tcx_attention_h2: needs N %% 32 == 0 and N <= 256, or N %% 256 == 0");
    TCX_REQUIRE(aligned16(qkv) && aligned16(out), "tcx_attention_h2: pointers must be 16-B aligned");
    if (Bt == 0) return TCX_OK;
    float* o = (float*)out;
    hipStream_t st = (hipStream_t)stream;
    if (N > 256) {
        switch (C / heads) {
            case 16: return launch_attn_flash<16>(qkv, o, Bt, N, C, heads, st, 1, ovf);
            case 32: return launch_attn_flash<32>(qkv, o, Bt, N, C, heads, st, 1, ovf);
            case 48: return launch_attn_flash<48>(qkv, o, Bt, N, C, heads, st, 1, ovf);
            case 64: return launch_attn_flash<64>(qkv, o, Bt, N, C, heads, st, 1, ovf);
            default: set_error("tcx_attention_h2: head dim %d unsupported for N > 256", C / heads); return TCX_EUNSUP;
        }
    }
    switch (C / heads) {
        case 8: return launch_attn_mfma<8>(qkv, o, Bt, N, C, heads, st, 1, ovf);
        case 16: return launch_attn_mfma<16>(qkv, o, Bt, N, C, heads, st, 1, ovf);
        case 24: return launch_attn_mfma<24>(qkv, o, Bt, N, C, heads, st, 1, ovf);
        case 32: return launch_attn_mfma<32>(qkv, o, Bt, N, C, heads, st, 1, ovf);
        case 48: return launch_attn_mfma<48>(qkv, o, Bt, N, C, heads, st, 1, ovf);
        case 64: return launch_attn_mfma<64>(qkv, o, Bt, N, C, heads, st, 1, ovf);
        default: set_error("tcx_attention_h2: head dim %d unsupported", C / heads); return TCX_EUNSUP;
    }
}
