// Halo-staged 3x3 stride-1 conv over h2 (split-f16) operands: the hot layer shape of
// CondUNetTiny (every _ConvBlock conv and us*_conv, /root/reference/src/toycrystals/models/
// sde_score_model.py:102,105,218,222 — 3x3, padding 1, circular).
//
// The implicit-GEMM kernel of conv.hip (k_conv SPL) gathers every im2col element from L1/L2 and
// writes it to LDS once per tap: 9 LDS writes per input element, and at the f16x3 MFMA rate
// (18 MFMA per wave per 32-deep chunk) those ds_write_b128 (13 LDS cycles each) and the global
// loads behind them, not the MFMA, set the pace.  Here a workgroup owns 256 output pixels = whole
// image rows (TR = 256/W rows) x 96 output channels, and per 32-channel input chunk stages the
// (TR+2) x (W+2) halo of those rows ONCE in LDS (circular wrap or zero padding applied while
// staging); the 9 taps then read their A fragments from the same halo at a constant
// (dy*(W+2) + dx)*144-byte offset, an immediate of the ds_read.  Per tap only the weight chunk
// (96 x 32 x h2) is staged.  K order: input-channel chunk outer, tap inner.
//
// Tile: 8 waves (512 threads, 2 per SIMD), wave w = output pixels [32w, 32w+32) of the tile x
// NT = 3 accumulator tiles of 32 channels; per tap and 16-deep step 3 x v_mfma_f32_32x32x16_f16
// per accumulator (hi*lo, lo*hi, hi*hi; h2.hpp).  LDS: halo x2 (next chunk staged during taps
// 0-4 of the current one) + weight chunk x2 = 141.7 KB at W = 64.  Epilogue shared with k_conv
// (conv_common.hpp), GroupNorm partials per 128-pixel half so the stats layout is unchanged.
#include "conv_common.hpp"

#include <type_traits>

namespace tcx {
namespace {

constexpr int HROW = 36;     // floats per staged pixel: 32 (h2 of 32 channels, 128 B) + 16 B pad

// NW waves per workgroup, RT 32-pixel row blocks per wave: tile = 32*NW*RT output pixels = whole rows
__host__ __device__ constexpr int halo_px(int W, int HB) { return (HB / W + 2) * (W + 2); }
// halo buffers: two at one workgroup per CU (NW = 8, or RT = 2), one at NW = 4 (two per CU)
__host__ __device__ constexpr int halo_bufs(int NW, int RT) { return (NW == 8 || RT == 2) ? 2 : 1; }

constexpr size_t conv3h_lds_bytes(int NT, int W, int NW, int RT) {
    return (size_t)(halo_bufs(NW, RT) * halo_px(W, 32 * NW * RT) + 2 * 32 * NT) * HROW * sizeof(float);
}

// RT = 2: each wave owns 64 pixels (two 32-row blocks) x 32*NT channels, so every B fragment read
// from LDS feeds two MFMAs and the weight chunk staged per tap serves 256 pixels (one workgroup
// of 4 waves per CU, accumulators beyond the 256 arch VGPRs in AGPRs).
template <int NT, int W, bool CIRC, int NW, int RT = 1>
__global__ __launch_bounds__(64 * NW, RT == 1 ? 2 : 1) void k_conv3h(ConvParams p) {
    constexpr int HB = 32 * NW * RT;
    constexpr int NTHR = 64 * NW;
    constexpr int HBUFS = halo_bufs(NW, RT);
    constexpr int BN = 32 * NT;
    constexpr int W2 = W + 2;
    constexpr int NPX = halo_px(W, HB);
    constexpr int HPI = (NPX * 8 + NTHR - 1) / NTHR;  // halo pieces (16 B) per thread
    constexpr int HBUF = NPX * HROW;            // floats per halo buffer
    constexpr int BBUF = BN * HROW;
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float* const Hs = sm;                 // [HBUFS][NPX][HROW]
    float* const Bs = sm + HBUFS * HBUF;  // [2][BN][HROW]

    const int tid = threadIdx.x;
    const int lane = tid & 63, wv = tid >> 6, li = lane & 31, lh = lane >> 5;
    const int tile = xcd_remap(blockIdx.x, gridDim.x);
    const int mblk = tile / p.n_nblk;
    const int nblk = tile - mblk * p.n_nblk;
    const int m0 = mblk * HB, n0 = nblk * BN;
    const int b = m0 / p.HoWo;
    const int r0 = (m0 - b * p.HoWo) / W;  // first output row of the tile
    const int bs = p.bmod > 0 ? b % p.bmod : b;
    const int H = p.H;
    const int cpt = p.Cin / BK;  // 32-channel input chunks
    const int nchunks = 9 * cpt;

    const __amdgpu_buffer_rsrc_t r1 = mk_rsrc(p.x1, p.bytes1);
    const __amdgpu_buffer_rsrc_t r2 = mk_rsrc(p.x2 ? p.x2 : p.x1, p.x2 ? p.bytes2 : p.bytes1);
    const __amdgpu_buffer_rsrc_t rw = mk_rsrc(p.w, p.bytesw);

    // ---- halo staging plan: piece e = tid + NTHR i -> halo pixel e >> 3, 16-B piece e & 7
    const int rowb = p.C1 * 4;  // bytes per source pixel (C2 == C1 when there are two sources)
    int hoff[HPI];              // source byte offset (kOOB: zero padding -> the buffer unit reads 0)
    int hdst[HPI];              // LDS float index, -1: past the halo (no store)
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
    // One halo buffer: the whole next halo waits in registers during a chunk.  Two buffers: the
    // next halo moves in HG = 3 groups, each loaded after one barrier and stored before the barrier
    // two taps later, so only one group's registers are live at a time.
    constexpr int HG = HBUFS == 2 ? (HPI + 2) / 3 : HPI;
    float4 hv[HG];
    auto halo_load_g = [&](int j, int g) {  // input-channel chunk j (uniform), group g
        const int ci0 = j * BK;
        const bool s1 = ci0 < p.C1;
        const int cc = (s1 ? ci0 : ci0 - p.C1) * 4;
        const __amdgpu_buffer_rsrc_t rs = s1 ? r1 : r2;
#pragma unroll
        for (int i = 0; i < HG; ++i)
            if (g * HG + i < HPI) hv[i] = bld4(rs, hoff[g * HG + i], cc);
    };
    auto halo_store_g = [&](int buf, int g) {
#pragma unroll
        for (int i = 0; i < HG; ++i) {
            const int k = g * HG + i;
            if (k < HPI && ((k + 1) * NTHR <= NPX * 8 || hdst[k] >= 0))  // only the last piece can fall past the halo
                *reinterpret_cast<float4*>(&Hs[buf * HBUF + hdst[k]]) = hv[i];
        }
    };
    auto halo_load = [&](int j) { halo_load_g(j, 0); };
    auto halo_store = [&](int buf) { halo_store_g(buf, 0); };
    // ---- weight chunk staging: BN rows x 8 pieces
    constexpr int BPI = (BN * 8 + NTHR - 1) / NTHR;
    float4 bv[BPI];
    int boff[BPI];
#pragma unroll
    for (int i = 0; i < BPI; ++i) {
        const int e = tid + NTHR * i;
        boff[i] = ((n0 + (e >> 3)) * p.kpad) * 4 + (e & 7) * 16;
    }
    auto w_load = [&](int c) {  // chunk c = 9 j + t -> packed k = t * Cin + 32 j
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
            if ((BN * 8) % NTHR == 0 || e < BN * 8) *reinterpret_cast<float4*>(&Bs[buf * BBUF + (e >> 3) * HROW + (e & 7) * 4]) = bv[i];
        }
    };

    // ---- fragments
    int abase[RT];  // float index in a halo buffer of this lane's A row (tile pixel) per row block
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
        const int mloc = (wv * RT + rt) * 32 + li;
        abase[rt] = ((mloc / W) * W2 + (mloc % W)) * HROW + lh * 8;
    }
    const int bbase = li * HROW + lh * 8;
    f32x16 acc[RT][NT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int n = 0; n < NT; ++n) acc[rt][n] = (f32x16){};
    h8 a_h[RT][2], a_l[RT][2], b_h[2][NT], b_l[2][NT];
    auto rd_a = [&](int hbuf, int t) {  // tap t: both 16-deep steps
        const int dy = t / 3, dx = t - 3 * (t / 3);
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
            const float* A = &Hs[hbuf * HBUF + abase[rt] + (dy * W2 + dx) * HROW];
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                a_h[rt][s] = __builtin_bit_cast(h8, ld4(A + 16 * s));
                a_l[rt][s] = __builtin_bit_cast(h8, ld4(A + 16 * s + 4));
            }
        }
    };
    auto rd_b = [&](int bb) {
        const float* B = &Bs[bb * BBUF + bbase];
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int n = 0; n < NT; ++n) {
                b_h[s][n] = __builtin_bit_cast(h8, ld4(B + n * 32 * HROW + 16 * s));
                b_l[s][n] = __builtin_bit_cast(h8, ld4(B + n * 32 * HROW + 16 * s + 4));
            }
    };
    auto mf = [&](int s) {
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
#pragma unroll
            for (int n = 0; n < NT; ++n)
                acc[rt][n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a_h[rt][s], b_l[s][n], acc[rt][n], 0, 0, 0);
#pragma unroll
            for (int n = 0; n < NT; ++n)
                acc[rt][n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a_l[rt][s], b_h[s][n], acc[rt][n], 0, 0, 0);
#pragma unroll
            for (int n = 0; n < NT; ++n)
                acc[rt][n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a_h[rt][s], b_h[s][n], acc[rt][n], 0, 0, 0);
        }
    };

    // ---- prologue: halo 0 and weight chunk 0 in LDS; halo 1 (one buffer) and weight chunk 1 in flight
    w_load(0);
    if constexpr (HBUFS == 2) {
#pragma unroll
        for (int g = 0; g < 3; ++g) {
            halo_load_g(0, g);
            halo_store_g(0, g);
        }
        w_store(0);
    } else {
        halo_load(0);
        halo_store(0);
        w_store(0);
        if (cpt > 1) halo_load(1);
    }
    w_load(nchunks > 1 ? 1 : 0);
    __syncthreads();
    rd_a(0, 0);

    for (int j = 0; j < cpt; ++j) {
        const int hb = HBUFS == 2 ? (j & 1) : 0;
#pragma unroll
        for (int t = 0; t < 9; ++t) {
            const int c = 9 * j + t;
            const int cur = c & 1;
            rd_b(cur);
            __builtin_amdgcn_sched_barrier(0);
            mf(0);
            mf(1);
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (HBUFS == 2) {
                // halo j+1 into the other buffer (free since chunk j-1's last barrier): group g
                // loaded after the barrier of tap 2g, stored before the barrier of tap 2g+2; the
                // next tap's A fragments come from the same halo or, after tap 8, the other
                if ((t == 2 || t == 4 || t == 6) && j + 1 < cpt) halo_store_g(hb ^ 1, t / 2 - 1);
                w_store(cur ^ 1);  // weight chunk c + 1
                __syncthreads();
                if ((t == 0 || t == 2 || t == 4) && j + 1 < cpt) halo_load_g(j + 1, t / 2);
                if (c + 2 < nchunks) w_load(c + 2);
                if (t < 8) rd_a(hb, t + 1);
                else rd_a(hb ^ 1, 0);
            } else {
                // one halo buffer: after the last tap every wave is past its reads of halo j, so
                // halo j+1 (loaded during chunk j) is stored behind one extra barrier
                w_store(cur ^ 1);
                __syncthreads();
                if (c + 2 < nchunks) w_load(c + 2);
                if (t < 8) {
                    rd_a(0, t + 1);
                } else {
                    if (j + 1 < cpt) {
                        halo_store(0);
                        __syncthreads();
                        if (j + 2 < cpt) halo_load(j + 2);
                    }
                    rd_a(0, 0);
                }
            }
        }
    }
    __syncthreads();  // the halo buffers become the epilogue's reduction scratch
    if constexpr (RT == 1) {
        conv_epilogue<NT, 1, NW>(p, acc[0], m0, n0, wv, tid, reinterpret_cast<double*>(sm));
    } else {
        // two explicit calls, not a loop: a rolled loop over the (large) inlined epilogue would index
        // acc dynamically and keep the whole accumulator array in scratch, stored after every tap
        double* red = reinterpret_cast<double*>(sm);
        static_assert(RT == 2, "RT is 1 or 2");
        conv_epi_store_rt<NT, 1, RT * NW, 2>(p, reinterpret_cast<f32x16(&)[2][NT]>(acc), m0, n0, RT * wv, lane, red);
        if (p.gn) {
            __syncthreads();
            conv_epi_gn<NT, RT * NW>(p, m0, n0, tid, NTHR, red);
        }
    }
}

// ---------------------------------------------------------------------------------------------
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
constexpr size_t conv3p_lds_bytes(int NT, int W, int NW = 4) {
    return (size_t)(halo_px(W, 32 * NW) + 3 * 32 * NT) * HROW * sizeof(float);
}

// NW = 4 (default: 128-pixel tiles, two workgroups per CU) or 8 (TCX_HALO_PNW=8: 256-pixel tiles,
// one workgroup per CU, half the weight staging per FLOP)
template <int NT, int W, bool CIRC, bool PRIO = false, int NW = 4>
__global__ __launch_bounds__(64 * NW, 8 / NW) void k_conv3p(ConvParams p) {
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
            if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
            mf(0);
            if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
            __builtin_amdgcn_sched_barrier(0);
            if (t < 8) rd(0, t + 1, wn);
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
            mf(1);
            if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
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

// ---------------------------------------------------------------------------------------------
// k_conv3w: the same halo scheme with one wave per SIMD and 64 x 96 outputs per wave (two 32-row
// blocks x three 32-column blocks: 36 MFMAs per 32-deep chunk, B fragments re-used by both row
// blocks, so half the LDS fragment reads per MFMA of k_conv3h).  Tile = 256 pixels x 96 channels,
// 4 waves, one workgroup per CU (halo x2 + weight chunk x2 = 141.7 KB at W = 64).  The fragments
// of chunk c+1 are read from LDS into a second register set while chunk c's MFMAs run, so after
// each barrier the MFMAs start from registers.  Per iteration c: global loads of weight chunk c+2
// (and at tap 0 of input chunk j the halo of j+1), 36 MFMAs interleaved with the reads of chunk
// c+1's fragments, weight chunk c+2 -> LDS (and at tap 4 halo j+1 -> LDS), one barrier.
// ---------------------------------------------------------------------------------------------
template <int W, bool CIRC>
__global__ __launch_bounds__(256, 1) void k_conv3w(ConvParams p) {
    constexpr int NT = 3, BN = 96, RT = 2, NW = 4, NTHR = 256;
    constexpr int HB = 32 * RT * NW;  // 256 output pixels
    constexpr int W2 = W + 2;
    constexpr int NPX = (HB / W + 2) * W2;
    constexpr int HPI = (NPX * 8 + NTHR - 1) / NTHR;
    constexpr int HBUF = NPX * HROW, BBUF = BN * HROW;
    constexpr int BPI = BN * 8 / NTHR;  // 3
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float* const Hs = sm;             // [2][NPX][HROW]
    float* const Bs = sm + 2 * HBUF;  // [2][BN][HROW]

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
    auto halo_store = [&](int buf) {
#pragma unroll
        for (int i = 0; i < HPI; ++i)
            if ((i + 1) * NTHR <= NPX * 8 || hdst[i] >= 0)
                *reinterpret_cast<float4*>(&Hs[buf * HBUF + hdst[i]]) = hv[i];
    };
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
        for (int i = 0; i < BPI; ++i) bv[i] = bld4(rw, boff[i], kb);
    };
    auto w_store = [&](int buf) {
#pragma unroll
        for (int i = 0; i < BPI; ++i) {
            const int e = tid + NTHR * i;
            *reinterpret_cast<float4*>(&Bs[buf * BBUF + (e >> 3) * HROW + (e & 7) * 4]) = bv[i];
        }
    };

    // fragments: lane's A rows = tile pixels 64*wv + 32*rt + li
    int abase[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
        const int mloc = wv * 64 + rt * 32 + li;
        abase[rt] = ((mloc / W) * W2 + (mloc % W)) * HROW + lh * 8;
    }
    const int bbase = li * HROW + lh * 8;
    f32x16 acc[RT][NT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int n = 0; n < NT; ++n) acc[rt][n] = (f32x16){};
    // two register sets of fragments [set][rt or n][step]
    h8 ah[2][RT][2], al[2][RT][2], bh[2][NT][2], bl[2][NT][2];
    auto rd = [&](auto SET, int hbuf, int tap, int bbuf) {
        constexpr int st = decltype(SET)::value;
        const int dy = tap / 3, dx = tap - 3 * (tap / 3);
        const int toff = hbuf * HBUF + (dy * W2 + dx) * HROW;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) {
                const float* A = &Hs[toff + abase[rt] + 16 * s];
                ah[st][rt][s] = __builtin_bit_cast(h8, ld4(A));
                al[st][rt][s] = __builtin_bit_cast(h8, ld4(A + 4));
            }
            const float* B = &Bs[bbuf * BBUF + bbase + 16 * s];
#pragma unroll
            for (int n = 0; n < NT; ++n) {
                bh[st][n][s] = __builtin_bit_cast(h8, ld4(B + n * 32 * HROW));
                bl[st][n][s] = __builtin_bit_cast(h8, ld4(B + n * 32 * HROW + 4));
            }
        }
    };
    auto mf = [&](auto SET) {
        constexpr int st = decltype(SET)::value;
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int rt = 0; rt < RT; ++rt)
#pragma unroll
                for (int n = 0; n < NT; ++n) {
                    acc[rt][n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[st][rt][s], bl[st][n][s], acc[rt][n], 0, 0, 0);
                    acc[rt][n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[st][rt][s], bh[st][n][s], acc[rt][n], 0, 0, 0);
                    acc[rt][n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[st][rt][s], bh[st][n][s], acc[rt][n], 0, 0, 0);
                }
    };
    using S0 = std::integral_constant<int, 0>;
    using S1 = std::integral_constant<int, 1>;
    // one iteration: chunk c = 9 j + t computed from register set CS; chunk c+1 read into CS ^ 1
    auto iter = [&](int j, auto T, auto CS) {
        constexpr int t = decltype(T)::value;
        constexpr int cs = decltype(CS)::value;
        using NS = std::integral_constant<int, cs ^ 1>;
        const int c = 9 * j + t;
        if (c + 2 < nchunks) w_load(c + 2);
        if (t == 0 && j + 1 < cpt) halo_load(j + 1);
        mf(CS);
        if (t < 8) rd(NS{}, j & 1, t + 1, (c + 1) & 1);
        else rd(NS{}, (j + 1) & 1, 0, (c + 1) & 1);
        if (t == 4 && j + 1 < cpt) halo_store((j + 1) & 1);
        w_store(c & 1);  // weight chunk c + 2 (its slot held chunk c, read during iteration c - 1)
        __syncthreads();
    };
    auto nine = [&](int j, auto E) {  // E: register set of the even taps
        using O = std::integral_constant<int, decltype(E)::value ^ 1>;
        iter(j, std::integral_constant<int, 0>{}, E);
        iter(j, std::integral_constant<int, 1>{}, O{});
        iter(j, std::integral_constant<int, 2>{}, E);
        iter(j, std::integral_constant<int, 3>{}, O{});
        iter(j, std::integral_constant<int, 4>{}, E);
        iter(j, std::integral_constant<int, 5>{}, O{});
        iter(j, std::integral_constant<int, 6>{}, E);
        iter(j, std::integral_constant<int, 7>{}, O{});
        iter(j, std::integral_constant<int, 8>{}, E);
    };

    // prologue: halo 0, weight chunks 0 and 1 in LDS; chunk 0's fragments in set 0
    halo_load(0);
    w_load(0);
    halo_store(0);
    w_store(0);
    w_load(nchunks > 1 ? 1 : 0);
    w_store(1);
    __syncthreads();
    rd(S0{}, 0, 0, 0);
    int j = 0;
    for (; j + 1 < cpt; j += 2) {
        nine(j, S0{});
        nine(j + 1, S1{});
    }
    if (j < cpt) nine(j, S0{});

    __syncthreads();  // halo buffers -> epilogue scratch
    double* red = reinterpret_cast<double*>(sm);
    conv_epi_store_rt<NT, 1, 2 * NW, 2>(p, reinterpret_cast<f32x16(&)[2][NT]>(acc), m0, n0, 2 * wv, lane, red);
    if (p.gn) {
        __syncthreads();
        conv_epi_gn<NT, 2 * NW>(p, m0, n0, tid, NTHR, red);
    }
}

template <int W>
int launch3w(const ConvParams& p, hipStream_t st) {
    constexpr size_t shm = (size_t)(2 * ((256 / W + 2) * (W + 2)) + 2 * 96) * HROW * sizeof(float);
    static bool attr[2] = {false, false};
    auto kc = p.circular ? &k_conv3w<W, true> : &k_conv3w<W, false>;
    if (!attr[p.circular ? 1 : 0]) {
        if (hipFuncSetAttribute(reinterpret_cast<const void*>(kc), hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)shm) != hipSuccess) {
            set_error("tcx_conv2d_h2: cannot enable %zu B of dynamic LDS", shm);
            return TCX_EHIP;
        }
        attr[p.circular ? 1 : 0] = true;
    }
    const int grid = (p.M / 256) * p.n_nblk;
    hipLaunchKernelGGL(kc, dim3(grid), dim3(256), shm, st, p);
    return check_launch("tcx_conv2d_h2(halo, wide)");
}

// TCX_HALO_PNW=8: k_conv3p with 8 waves and 256-pixel tiles
bool pnw8() {
    static const bool on = [] {
        const char* e = getenv("TCX_HALO_PNW");
        return e && atoi(e) == 8;
    }();
    return on;
}

template <int NT, int W>
int launch3p(const ConvParams& p, hipStream_t st) {
    constexpr size_t shm = conv3p_lds_bytes(NT, W);
    static bool attr[2] = {false, false};
    // TCX_HALO_PRIO=1: s_setprio(1) around each MFMA cluster (A/B knob)
    static const bool prio = [] {
        const char* e = getenv("TCX_HALO_PRIO");
        return e && atoi(e) == 1;
    }();
    auto kc = p.circular ? (prio ? &k_conv3p<NT, W, true, true> : &k_conv3p<NT, W, true, false>)
                         : &k_conv3p<NT, W, false, false>;
    if (pnw8()) {
        constexpr size_t shm8 = conv3p_lds_bytes(NT, W, 8);
        auto k8 = p.circular ? &k_conv3p<NT, W, true, false, 8> : &k_conv3p<NT, W, false, false, 8>;
        static bool attr8[2] = {false, false};
        if (!attr8[p.circular ? 1 : 0]) {
            if (hipFuncSetAttribute(reinterpret_cast<const void*>(k8), hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)shm8) != hipSuccess) {
                set_error("tcx_conv2d_h2: cannot enable %zu B of dynamic LDS", shm8);
                return TCX_EHIP;
            }
            attr8[p.circular ? 1 : 0] = true;
        }
        hipLaunchKernelGGL(k8, dim3((p.M / 256) * p.n_nblk), dim3(512), shm8, st, p);
        return check_launch("tcx_conv2d_h2(halo, pipelined, 8 waves)");
    }
    if (!attr[p.circular ? 1 : 0]) {
        if (hipFuncSetAttribute(reinterpret_cast<const void*>(kc), hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)shm) != hipSuccess) {
            set_error("tcx_conv2d_h2: cannot enable %zu B of dynamic LDS", shm);
            return TCX_EHIP;
        }
        attr[p.circular ? 1 : 0] = true;
    }
    const int grid = (p.M / 128) * p.n_nblk;
    hipLaunchKernelGGL(kc, dim3(grid), dim3(256), shm, st, p);
    return check_launch("tcx_conv2d_h2(halo, pipelined)");
}

template <int NT, int W, int NW, int RT = 1>
int launch3h_w(const ConvParams& p, hipStream_t st) {
    constexpr size_t shm = conv3h_lds_bytes(NT, W, NW, RT);
    static bool attr[2] = {false, false};
    auto kc = p.circular ? &k_conv3h<NT, W, true, NW, RT> : &k_conv3h<NT, W, false, NW, RT>;
    if (!attr[p.circular ? 1 : 0]) {
        if (hipFuncSetAttribute(reinterpret_cast<const void*>(kc), hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)shm) != hipSuccess) {
            set_error("tcx_conv2d_h2: cannot enable %zu B of dynamic LDS", shm);
            return TCX_EHIP;
        }
        attr[p.circular ? 1 : 0] = true;
    }
    const int grid = (p.M / (32 * NW * RT)) * p.n_nblk;
    hipLaunchKernelGGL(kc, dim3(grid), dim3(64 * NW), shm, st, p);
    return check_launch("tcx_conv2d_h2(halo)");
}

// variant: TCX_HALO_NW=4 (default when unset: 128-pixel tiles, two workgroups per CU — k_conv3p, or
// k_conv3h with TCX_HALO_PIPE=0), 8 (k_conv3h, 256-pixel tiles of 8 waves, one workgroup per CU) or
// 0 (k_conv3w, 256-pixel tiles of 4 wide waves; slower, kept for A/B)
int halo_nw() {
    static const int nw = [] {
        const char* e = getenv("TCX_HALO_NW");
        const int v = e ? atoi(e) : 4;
        return v == 8 ? 8 : (v == 0 ? 0 : 4);
    }();
    return nw;
}
// TCX_HALO_RT=2 with TCX_HALO_NW=4: k_conv3h with two 32-pixel row blocks per wave (256-pixel tiles)
int halo_rt() {
    static const int rt = [] {
        const char* e = getenv("TCX_HALO_RT");
        return (e && atoi(e) == 2 && halo_nw() == 4) ? 2 : 1;
    }();
    return rt;
}
// k_conv3p (fragment reads pipelined across steps) serves TCX_HALO_NW=4, RT 1 (the default);
// TCX_HALO_PIPE=0 selects the unpipelined k_conv3h instead
bool halo_pipe() {
    static const bool on = [] {
        const char* e = getenv("TCX_HALO_PIPE");
        return !(e && atoi(e) == 0) && halo_nw() == 4 && halo_rt() == 1;
    }();
    return on;
}
// output pixels per workgroup tile of the selected variant
int halo_tile() { return halo_nw() ? 32 * halo_nw() * halo_rt() * (halo_pipe() && pnw8() ? 2 : 1) : 256; }

}  // namespace

// Host dispatch (conv.hip): true when the halo kernel covers this conv.
bool conv3h_applies(const ConvParams& p, int cout_pad) {
    static const bool off = getenv("TCX_NO_HALO") != nullptr;
    return !off && p.ks == 3 && p.stride == 1 && p.pad_y == 1 && p.pad_x == 1 && p.Hi == p.H && p.Wi == p.W &&
           (p.W == 16 || p.W == 32 || p.W == 64) && p.H % (halo_tile() / p.W) == 0 && p.HoWo % halo_tile() == 0 &&
           cout_pad % 96 == 0 && p.Cin % BK == 0 && p.C1 % BK == 0 && (p.C2 == 0 || p.C2 == p.C1) &&
           p.kpad == 9 * p.Cin && p.osy == 1 && p.osx == 1;
}

int launch_conv3h(ConvParams& p, int cout_pad, hipStream_t st) {
    p.n_nblk = cout_pad / 96;
    if (p.M == 0) return TCX_OK;
    prof_begin(st);
    int rc;
    if (halo_nw() == 0) {
        if (p.W == 64) rc = launch3w<64>(p, st);
        else if (p.W == 32) rc = launch3w<32>(p, st);
        else rc = launch3w<16>(p, st);
    } else if (halo_nw() == 8) {
        if (p.W == 64) rc = launch3h_w<3, 64, 8>(p, st);
        else if (p.W == 32) rc = launch3h_w<3, 32, 8>(p, st);
        else rc = launch3h_w<3, 16, 8>(p, st);
    } else if (halo_pipe()) {
        if (p.W == 64) rc = launch3p<3, 64>(p, st);
        else if (p.W == 32) rc = launch3p<3, 32>(p, st);
        else rc = launch3p<3, 16>(p, st);
    } else if (halo_rt() == 2) {
        if (p.W == 64) rc = launch3h_w<3, 64, 4, 2>(p, st);
        else if (p.W == 32) rc = launch3h_w<3, 32, 4, 2>(p, st);
        else rc = launch3h_w<3, 16, 4, 2>(p, st);
    } else {
        if (p.W == 64) rc = launch3h_w<3, 64, 4>(p, st);
        else if (p.W == 32) rc = launch3h_w<3, 32, 4>(p, st);
        else rc = launch3h_w<3, 16, 4>(p, st);
    }
    prof_end(st, 2.0 * (double)p.M * p.Cout * 9 * p.Cin);
    return rc;
}

}  // namespace tcx
