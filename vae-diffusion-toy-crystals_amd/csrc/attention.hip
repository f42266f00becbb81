// Bottleneck self-attention of SelfAttention2d (/root/reference/src/toycrystals/models/
// sde_score_model.py:136-167): per (batch, head) softmax(q k^T / sqrt(d)) v over N = H*W
// tokens (N = 256, d = 48 at base_ch 96).  K and V of one head fit LDS whole (2 x 48 KB), so
// one pass with an exact (non-online) softmax: 4 lanes per query row, each owning every 4th key;
// row max / sum and the output by two xor-shuffles.  The q,k,v channel split and the head-major
// channel order (view [B,heads,d,N] -> transpose) are folded into the addressing.
#include "common.hpp"

namespace tcx {
namespace {

constexpr int QROWS = 64;  // query rows per block (4 lanes each)
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
    TCX_REQUIRE(N > 0 && N <= 4 * MAXK, "tcx_attention: N must be <= 256 (single-tile kernel)");
    TCX_REQUIRE(aligned16(qkv) && aligned16(out), "tcx_attention: pointers must be 16-B aligned");
    if (Bt == 0) return TCX_OK;
    const int D = C / heads;
    hipStream_t st = (hipStream_t)stream;
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
