// k_conv3p: the halo-staged 3x3 stride-1 conv over h2 (split-f16) operands with PLAIN (not
// fragment-ordered) packed weights: the fallback of the 3x3 split path when no fragment-ordered weight
// copy exists (the training convs of functional.py, zero padding, shapes k_conv3g / k_conv3l do not
// cover).  The sampler's 3x3 convs (/root/reference/src/toycrystals/models/sde_score_model.py:102,
// 105,218,222) run on k_conv3lg / k_conv3l / k_conv3g (conv3l.hip, conv3g.hip).
//
// The im2col kernel of conv.hip (k_conv SPL) gathers every im2col element from L1/L2 and writes it to
// LDS once per tap: 9 LDS writes per input element, and at the f16x3 MFMA rate those ds_write_b128
// (13 LDS cycles each), not the MFMA, set the pace.  Here a workgroup owns 128 output pixels = whole
// image rows x 96 output channels, and per 32-channel input chunk stages the (TR+2) x (W+2) halo of
// those rows ONCE in LDS (circular wrap or zero padding applied while staging); the 9 taps read their
// A fragments from the same halo at a constant (dy*(W+2) + dx)*144-byte offset, an immediate of the
// ds_read.  Per tap only the weight chunk (96 x 32 x h2) is staged.  K order: input-channel chunk
// outer, tap inner.  4 waves (two workgroups per CU), wave w = output pixels [32w, 32w+32) x NT = 3
// accumulator tiles of 32 channels; per tap and 16-deep step 3 x v_mfma_f32_32x32x16_f16 per
// accumulator (hi*lo, lo*hi, hi*hi; h2.hpp).  Epilogue shared with k_conv (conv_common.hpp).
//
// (Round 1/2 variants measured slower and removed in round 3: the unpipelined k_conv3h, 8-wave and
// 64-pixel-per-wave tiles, the wide-wave k_conv3w, s_setprio around the MFMA clusters — DESIGN.md §6.)
#include "conv_common.hpp"

#include <type_traits>

namespace tcx {
namespace {

constexpr int HROW = 36;     // floats per staged pixel: 32 (h2 of 32 channels, 128 B) + 16 B pad
constexpr int P_TP = 128;    // output pixels per workgroup tile

__host__ __device__ constexpr int halo_px(int W, int HB) { return (HB / W + 2) * (W + 2); }
// k_conv3p: k_conv3h (4 waves, 128-pixel tiles, two workgroups per CU, one halo buffer) with the
// fragment reads software-pipelined across 16-deep steps.  Per tap t the registers hold one step's
// fragments while the other step's are read: [read step 1 of tap t] [MFMAs of step 0]
// [read step 0 of tap t+1] [MFMAs of step 1], so the LDS reads of a step overlap the previous
// step's 9 MFMAs instead of stalling the wave before every tap (same 64 fragment registers as
// k_conv3h).  Step 0 of tap t+1 needs weight chunk c+1 in LDS before tap t's barrier, so the
// weight chunks rotate through THREE buffers (chunk c+2 is stored during tap c; 79.5 KB of LDS at
// W = 64).  At the last tap of an input-channel chunk the next halo is stored first (one halo
// buffer), so that tap's step-0 read of the next chunk happens after the extra barrier.
// ---------------------------------------------------------------------------------------------
constexpr size_t conv3p_lds_bytes(int NT, int W) {
    return (size_t)(halo_px(W, P_TP) + 3 * 32 * NT) * HROW * sizeof(float);
}

template <int NT, int W, bool CIRC>
__global__ __launch_bounds__(256, 2) void k_conv3p(ConvParams p) {
    constexpr int NW = 4;
    constexpr int HB = 32 * NW, NTHR = 64 * NW;
    constexpr int BN = 32 * NT;
    constexpr int W2 = W + 2;
    constexpr int NPX = halo_px(W, HB);
    constexpr int HPI = (NPX * 8 + NTHR - 1) / NTHR;
    constexpr int HBUF = NPX * HROW;
    constexpr int BBUF = BN * HROW;
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float* const Hs = sm;         // [NPX][HROW]
    float* const Bs = sm + HBUF;  // [3][BN][HROW]

    const int tid = threadIdx.x;
    const int lane = tid & 63, wv = tid >> 6, li = lane & 31, lh = lane >> 5;
    const int tile = xcd_remap(blockIdx.x, gridDim.x);
    const int mblk = tile / p.n_nblk;
    const int nblk = tile - mblk * p.n_nblk;
    const int m0 = mblk * HB, n0 = nblk * BN;
    const int b = m0 / p.HoWo;
    const int r0 = (m0 - b * p.HoWo) / W;
    const int bs = p.bmod > 0 ? b % p.bmod : b;
    const int H = p.H;
    const int cpt = p.Cin / BK;
    const int nchunks = 9 * cpt;

    const __amdgpu_buffer_rsrc_t r1 = mk_rsrc(p.x1, p.bytes1);
    const __amdgpu_buffer_rsrc_t r2 = mk_rsrc(p.x2 ? p.x2 : p.x1, p.x2 ? p.bytes2 : p.bytes1);
    const __amdgpu_buffer_rsrc_t rw = mk_rsrc(p.w, p.bytesw);

    const int rowb = p.C1 * 4;
    int hoff[HPI], hdst[HPI];
#pragma unroll
    for (int i = 0; i < HPI; ++i) {
        const int e = tid + NTHR * i;
        const int hp = e >> 3;
        hoff[i] = kOOB;
        hdst[i] = -1;
        if (hp < NPX) {
            const int hr = hp / W2, hc = hp - hr * W2;
            int y = r0 + hr - 1, x = hc - 1;
            bool ok = true;
            if (CIRC) {
                y = wrap_idx(y, H);
                x = wrap_idx(x, W);
            } else {
                ok = y >= 0 && y < H && x >= 0 && x < W;
            }
            hoff[i] = ok ? ((bs * H + y) * W + x) * rowb + (e & 7) * 16 : kOOB;
            hdst[i] = hp * HROW + (e & 7) * 4;
        }
    }
    float4 hv[HPI];
    auto halo_load = [&](int j) {
        const int ci0 = j * BK;
        const bool s1 = ci0 < p.C1;
        const int cc = (s1 ? ci0 : ci0 - p.C1) * 4;
        const __amdgpu_buffer_rsrc_t rs = s1 ? r1 : r2;
#pragma unroll
        for (int i = 0; i < HPI; ++i) hv[i] = bld4(rs, hoff[i], cc);
    };
    auto halo_store = [&]() {
#pragma unroll
        for (int i = 0; i < HPI; ++i)
            if ((i + 1) * NTHR <= NPX * 8 || hdst[i] >= 0) *reinterpret_cast<float4*>(&Hs[hdst[i]]) = hv[i];
    };
    constexpr int BPI = (BN * 8 + NTHR - 1) / NTHR;
    float4 bv[BPI];
    int boff[BPI];
#pragma unroll
    for (int i = 0; i < BPI; ++i) {
        const int e = tid + NTHR * i;
        boff[i] = ((n0 + (e >> 3)) * p.kpad) * 4 + (e & 7) * 16;
    }
    auto w_load = [&](int c) {
        const int j = c / 9, t = c - 9 * j;
        const int kb = (t * p.Cin + j * BK) * 4;
#pragma unroll
        for (int i = 0; i < BPI; ++i)
            if ((BN * 8) % NTHR == 0 || tid + NTHR * i < BN * 8) bv[i] = bld4(rw, boff[i], kb);
    };
    auto w_store = [&](int buf) {
#pragma unroll
        for (int i = 0; i < BPI; ++i) {
            const int e = tid + NTHR * i;
            if ((BN * 8) % NTHR == 0 || e < BN * 8)
                *reinterpret_cast<float4*>(&Bs[buf * BBUF + (e >> 3) * HROW + (e & 7) * 4]) = bv[i];
        }
    };

    const int mloc = wv * 32 + li;
    const int abase = ((mloc / W) * W2 + (mloc % W)) * HROW + lh * 8;
    const int bbase = li * HROW + lh * 8;
    f32x16 acc[NT];
#pragma unroll
    for (int n = 0; n < NT; ++n) acc[n] = (f32x16){};
    h8 a_h[2], a_l[2], b_h[2][NT], b_l[2][NT];
    auto rd = [&](int s, int t, int bb) {  // step s of tap t, weights from buffer bb
        const int dy = t / 3, dx = t - 3 * (t / 3);
        const float* A = &Hs[abase + (dy * W2 + dx) * HROW + 16 * s];
        a_h[s] = __builtin_bit_cast(h8, ld4(A));
        a_l[s] = __builtin_bit_cast(h8, ld4(A + 4));
        const float* B = &Bs[bb * BBUF + bbase + 16 * s];
#pragma unroll
        for (int n = 0; n < NT; ++n) {
            b_h[s][n] = __builtin_bit_cast(h8, ld4(B + n * 32 * HROW));
            b_l[s][n] = __builtin_bit_cast(h8, ld4(B + n * 32 * HROW + 4));
        }
    };
    auto mf = [&](int s) {
#pragma unroll
        for (int n = 0; n < NT; ++n) acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a_h[s], b_l[s][n], acc[n], 0, 0, 0);
#pragma unroll
        for (int n = 0; n < NT; ++n) acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a_l[s], b_h[s][n], acc[n], 0, 0, 0);
#pragma unroll
        for (int n = 0; n < NT; ++n) acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a_h[s], b_h[s][n], acc[n], 0, 0, 0);
    };

    // ---- prologue: halo 0 and weight chunks 0, 1 in LDS; chunk 2 (and halo 1) in flight
    halo_load(0);
    w_load(0);
    halo_store();
    w_store(0);
    w_load(nchunks > 1 ? 1 : 0);
    w_store(1);
    if (nchunks > 2) w_load(2);
    if (cpt > 1) halo_load(1);
    __syncthreads();
    rd(0, 0, 0);

    int wb = 0;  // buffer of chunk c (c mod 3)
    for (int j = 0; j < cpt; ++j) {
#pragma unroll
        for (int t = 0; t < 9; ++t) {
            const int c = 9 * j + t;
            const int wn = wb == 2 ? 0 : wb + 1;   // chunk c+1
            const int wn2 = wn == 2 ? 0 : wn + 1;  // chunk c+2
            // sched barriers pin the order: hipcc otherwise sinks each read group next to its
            // MFMAs (lgkmcnt(0) before each), which serialises reads and MFMAs again
            rd(1, t, wb);
            __builtin_amdgcn_sched_barrier(0);
            mf(0);
            __builtin_amdgcn_sched_barrier(0);
            if (t < 8) rd(0, t + 1, wn);
            __builtin_amdgcn_sched_barrier(0);
            mf(1);
            __builtin_amdgcn_sched_barrier(0);
            w_store(wn2);  // chunk c+2 (its buffer held chunk c-1, read before the last barrier)
            __syncthreads();
            if (c + 3 < nchunks) w_load(c + 3);
            if (t == 8) {
                // every wave is past its reads of halo j: store halo j+1 behind one extra barrier
                if (j + 1 < cpt) {
                    halo_store();
                    __syncthreads();
                    if (j + 2 < cpt) halo_load(j + 2);
                }
                rd(0, 0, wn);
            }
            wb = wn;
        }
    }
    __syncthreads();
    conv_epilogue<NT, 1, NW>(p, acc, m0, n0, wv, tid, reinterpret_cast<double*>(sm));
}

template <int NT, int W>
int launch3p(const ConvParams& p, hipStream_t st) {
    constexpr size_t shm = conv3p_lds_bytes(NT, W);
    static bool attr[2] = {false, false};
    auto kc = p.circular ? &k_conv3p<NT, W, true> : &k_conv3p<NT, W, false>;
    if (!attr[p.circular ? 1 : 0]) {
        if (hipFuncSetAttribute(reinterpret_cast<const void*>(kc), hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)shm) != hipSuccess) {
            set_error("tcx_conv2d_h2: cannot enable %zu B of dynamic LDS", shm);
            return TCX_EHIP;
        }
        attr[p.circular ? 1 : 0] = true;
    }
    const int grid = (p.M / P_TP) * p.n_nblk;
    hipLaunchKernelGGL(kc, dim3(grid), dim3(256), shm, st, p);
    return check_launch("tcx_conv2d_h2(halo, pipelined)");
}

}  // namespace

// Host dispatch (conv.hip): true when the halo kernel covers this conv.
bool conv3h_applies(const ConvParams& p, int cout_pad) {
    return p.ks == 3 && p.stride == 1 && p.pad_y == 1 && p.pad_x == 1 && p.Hi == p.H && p.Wi == p.W &&
           (p.W == 16 || p.W == 32 || p.W == 64) && p.H % (P_TP / p.W) == 0 && p.HoWo % P_TP == 0 &&
           cout_pad % 96 == 0 && p.Cin % BK == 0 && p.C1 % BK == 0 && (p.C2 == 0 || p.C2 == p.C1) &&
           p.kpad == 9 * p.Cin && p.osy == 1 && p.osx == 1;
}

int launch_conv3h(ConvParams& p, int cout_pad, hipStream_t st) {
    p.n_nblk = cout_pad / 96;
    if (p.M == 0) return TCX_OK;
    prof_begin(st);
    int rc;
    if (p.W == 64) rc = launch3p<3, 64>(p, st);
    else if (p.W == 32) rc = launch3p<3, 32>(p, st);
    else rc = launch3p<3, 16>(p, st);
    prof_end(st, 2.0 * (double)p.M * p.Cout * 9 * p.Cin);
    return rc;
}

}  // namespace tcx
