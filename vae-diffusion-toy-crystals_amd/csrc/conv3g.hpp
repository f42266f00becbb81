// conv3g.hpp — k_conv3g and its launcher, instantiated per row width in conv3g_w{16,32,64,128}.hip
// (parallel compilation); conv3g.hip holds the dispatch and the weight-fragment pack.
//
// k_conv3g: the 3x3 stride-1 circular conv of the U-Net rows W >= 32 (every _ConvBlock conv and
// us*_conv at 64^2 / 32^2, and the 128^2 rows of config 5: /root/reference/src/toycrystals/
// models/sde_score_model.py:102,105,218,222) on the f16x3 split path, with the preceding
// GroupNorm + SiLU (:103-107) applied while the input halo is staged.
//
// Why a new kernel (k_conv3p, conv3h.hip, stays for 16^2 and for callers without the fragment-
// ordered weights): k_conv3p stages every tap's weight chunk through LDS and so needs a workgroup
// barrier per tap (18 MFMAs per wave); its MFMA pipe is busy 45-48 % (PMC r01_bh, r02_f), the rest
// mostly waves parked at those barriers with both waves of a SIMD in the same phase.  Here:
//  * each wave owns 64 pixels (two 32-row blocks) x 96 channels, so a B fragment feeds two MFMAs;
//  * the input-channel chunk is 16 deep and B fragments come straight from global memory (L1/L2:
//    the 6 KB of a tap are read by every wave of the CU) in a fragment-ordered copy of the weights
//    (tcx_pack_conv_weight_h2_frag: one coalesced 1 KB dwordx4 load per wave per fragment), loaded
//    one tap ahead into the second of two register sets — no weight staging, no weight barrier;
//  * only the halo is in LDS, double-buffered: halo j+1 is staged during taps 2-5 of chunk j, so
//    a chunk of 9 taps (162 MFMAs per wave) needs 2 barriers (after taps 1 and 6) instead of 9.
// NW = 4 waves (256-pixel tiles, two workgroups per CU) for rows of 32/64 pixels, NW = 8
// (512-pixel tiles, one per CU) at 128.
//
// LDS: two halo buffers [(TR+2)*(W+2)][20 floats] (16 channels h2 = 64 B per pixel + 16 B pad: the
// 80-B pixel stride makes the ds_read_b128 of 32 consecutive pixels conflict free for every tap
// offset) and the GroupNorm tables [2][Cin] of the tile's image: 66 KB at W = 64 (two per CU),
// 128 KB at W = 128.  (W = 256 would not fit: those rows stay on the im2col kernel.)
//
// Prologue: a source may be h2 (copied) or fp32 + a per-(image, channel) GroupNorm scale/shift table
// (tcx_gn_finalize): x -> silu(x*sc + sh) is computed per 8-channel unit two taps after its load and
// split to h2 in registers right before the unit is stored.  The normalised tensor is
// never written to HBM (the k_gn_apply_tab_h2 pass it replaces read and wrote every element).
// SiLU here is x * rcp(1 + exp2(-x log2 e)) (v_exp_f32 / v_rcp_f32, ~2 ulp of fp32): the value is
// rounded to the 22-bit h2 split right after, so the difference to expf/IEEE division is below the
// split's own rounding (h2.hpp).
//
// Per tap t of chunk j (c = 9j + t; B set S = c & 1 holds B(c); A0 = row block 0 of tap t):
//   load B(c+1) -> set S^1 | read A1(t) | 9 MFMAs (row block 0) | read A0(t+1) | 9 MFMAs (row block 1)
//   [t < UPT: load halo unit t of j+1] [2 <= t < UPT+2: GN+SiLU+split, store unit t-2 into the other
//   halo buffer] [t == 1, t == 6: barrier]
// The other halo buffer held halo j-1, last read during tap 7 of chunk j-1 (the A fragments of tap
// 8 are read one tap early), before the barrier after tap 1 of chunk j; its stores end at tap 5,
// before the barrier after tap 6; its first read is A0 of tap 0 of chunk j+1, during tap 8.
#pragma once
#include "conv_common.hpp"

#include <algorithm>
#include <type_traits>

namespace tcx {
namespace {

constexpr int G_PXF = 20;   // floats per staged halo pixel: 16 channels h2 (64 B) + 16 B pad
constexpr int G_KC = 16;    // input channels per chunk
constexpr int G_NT = 3;     // 32-channel accumulator tiles per wave (96 output channels)

// NW waves of 64 pixels: tile TP = 64 NW output pixels = whole rows
__host__ __device__ constexpr int g_tp(int NW) { return 64 * NW; }
__host__ __device__ constexpr int g_npx(int W, int NW) { return (g_tp(NW) / W + 2) * (W + 2); }
__host__ __device__ constexpr int g_units(int W, int NW) { return (2 * g_npx(W, NW) + 64 * NW - 1) / (64 * NW); }
// NW = 4 (two workgroups per CU) for rows of 16/32/64 pixels and the bf16 256-px rows, NW = 8 (one
// per CU) for 128
__host__ __device__ constexpr int g_nw(int W) { return W == 128 ? 8 : 4; }
// "slim" halo (bf16 at 256-px rows, config 5): a bf16 product reads only the hi halves of the records,
// so a halo slot holds the two 16-B hi pieces of the pixel's 16-channel chunk + 16 B pad (48 B: the
// ds_read_b128 of 32 consecutive slots then lands on 3 p mod 16, distinct over every 16-lane group),
// and the halo of a 256-px row (3 x 258 slots) fits twice in 74 KB: two workgroups per CU
__host__ __device__ constexpr bool g_slim(int W, bool BF) { return BF && W == 256; }
__host__ __device__ constexpr int g_pxf(int W, bool BF) { return g_slim(W, BF) ? 12 : G_PXF; }

constexpr size_t conv3g_lds_bytes(int W, int NW, int Cin, bool BF = false) {
    return ((size_t)2 * g_npx(W, NW) * g_pxf(W, BF) + 2 * (size_t)Cin) * sizeof(float);
}

__device__ __forceinline__ float silu_split_src(float v, float sc, float sh) {
    const float y = fmaf(v, sc, sh);
    return y * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-1.4426950408889634f * y));
}

// 8 fp32 values -> h2 unit: hi halves (16 B) and lo halves (16 B); BF: bf16 halves (no range limit)
template <bool BF>
__device__ __forceinline__ void split8(const float (&v)[8], float4& hi, float4& lo, bool& bad) {
    unsigned h[4], l[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const unsigned a = BF ? split1_bf(v[2 * k]) : split1(v[2 * k]);
        const unsigned b = BF ? split1_bf(v[2 * k + 1]) : split1(v[2 * k + 1]);
        h[k] = (a & 0xffffu) | (b << 16);
        l[k] = (a >> 16) | (b & 0xffff0000u);
        if (!BF) bad = bad || h2_bad(v[2 * k]) || h2_bad(v[2 * k + 1]);
    }
    hi = make_float4(__uint_as_float(h[0]), __uint_as_float(h[1]), __uint_as_float(h[2]), __uint_as_float(h[3]));
    lo = make_float4(__uint_as_float(l[0]), __uint_as_float(l[1]), __uint_as_float(l[2]), __uint_as_float(l[3]));
}

// PRO: 0 = every source h2; 1 = every source fp32 + GroupNorm table (the transform is branch-free
// and interleaved with the MFMAs of its tap); 2 = per-source at run time (mixed concat sources).
// BF: bf16 records and weights, one v_mfma_f32_32x32x16_bf16 (hi x hi) per product.
template <int W, int NW, bool CIRC, int PRO, bool BF>
__global__ __launch_bounds__(64 * NW, 8 / NW) void k_conv3g(ConvParams p) {
    constexpr int RT = 2, NT = G_NT, BN = 32 * NT, NTHR = 64 * NW;
    constexpr int TP = g_tp(NW);
    constexpr int W2 = W + 2;
    constexpr int NPX = g_npx(W, NW);
    constexpr int NU = 2 * NPX;        // 8-channel halo units per chunk
    constexpr int UPT = g_units(W, NW);
    constexpr bool SLIM = g_slim(W, BF);
    constexpr int PXF = g_pxf(W, BF);
    constexpr int HBUF = NPX * PXF;
    // units are loaded UPL per tap at taps 0 .. NLT-1 and stored two taps later (by tap 5)
    constexpr int UPL = (UPT + 3) / 4;
    constexpr int NLT = (UPT + UPL - 1) / UPL;
    static_assert(NLT <= 4, "halo units per thread: stores must finish by tap 5");
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float* const Hs = sm;                   // [2][NPX][PXF]
    float* const Ts = sm + 2 * HBUF;        // [2][Cin]: scale, shift of this tile's image

    const int tid = threadIdx.x;
    const int lane = tid & 63, wv = tid >> 6, li = lane & 31, lh = lane >> 5;
    const int tile = xcd_remap(blockIdx.x, gridDim.x);
    const int mblk = tile / p.n_nblk;
    const int nblk = tile - mblk * p.n_nblk;
    const int m0 = mblk * TP, n0 = nblk * BN;
    const int b = m0 / p.HoWo;
    const int r0 = (m0 - b * p.HoWo) / W;
    const int bs = p.bmod > 0 ? b % p.bmod : b;
    const int H = p.H;
    const int Cin = p.Cin;
    const int cpt = Cin / G_KC;        // chunks (even: Cin % 32 == 0)
    const int nch = 9 * cpt;
    const bool gn1 = PRO == 1 || (PRO == 2 && p.sc1 != nullptr);
    const bool gn2 = PRO == 1 || (PRO == 2 && p.sc2 != nullptr);

    const __amdgpu_buffer_rsrc_t r1 = mk_rsrc(p.x1, p.bytes1);
    const __amdgpu_buffer_rsrc_t r2 = mk_rsrc(p.x2 ? p.x2 : p.x1, p.x2 ? p.bytes2 : p.bytes1);
    const __amdgpu_buffer_rsrc_t rw = mk_rsrc(reinterpret_cast<const float*>(p.wf), p.bytesw);

    // ---- GroupNorm tables of this tile's image (concatenated channel order)
    if (PRO != 0 && (gn1 || gn2)) {
        for (int c = tid; c < Cin; c += NTHR) {
            const bool s1 = c < p.C1;
            const float* sc = s1 ? p.sc1 : p.sc2;
            const float* sh = s1 ? p.sh1 : p.sh2;
            const int cc = s1 ? c : c - p.C1;
            const int Cs = s1 ? p.C1 : p.C2;
            Ts[c] = sc ? sc[(size_t)b * Cs + cc] : 1.f;
            Ts[Cin + c] = sh ? sh[(size_t)b * Cs + cc] : 0.f;
        }
    }

    // ---- halo plan: unit u = tid + NTHR i -> halo pixel u % NPX, 8-channel group u / NPX (eight
    // consecutive lanes store eight consecutive 80-B pixel slots: conflict-free ds_write_b128)
    const int rowb = p.C1 * 4;  // bytes per source pixel (C2 == C1 when there are two sources)
    int hoff[UPT];              // source byte offset of the unit (kOOB: zero padding)
#pragma unroll
    for (int i = 0; i < UPT; ++i) {
        const int u = tid + NTHR * i;
        const int hp = u < NPX ? u : u - NPX;
        hoff[i] = kOOB;
        if (u < NU) {
            const int hr = hp / W2, hc = hp - hr * W2;
            int y = r0 + hr - 1, x = hc - 1;
            bool ok = true;
            if (CIRC) {
                y = wrap_idx(y, H);
                x = wrap_idx(x, W);
            } else {
                ok = y >= 0 && y < H && x >= 0 && x < W;
            }
            hoff[i] = ok ? ((bs * H + y) * W + x) * rowb + (u < NPX ? 0 : 32) : kOOB;
        }
    }
    // Every vector-memory load is unconditional (after the last chunk the loads re-read valid bytes
    // that are never used): a load under a branch makes hipcc's wait counting fall back to
    // vmcnt(0), which would drain the halo loads in flight.
    float4 hv[UPT][2];  // unit i of the next halo (loaded at tap i, stored at tap i+2)
    auto src_of = [&](int j, __amdgpu_buffer_rsrc_t& rs, int& cc) {
        const int ci0 = j * G_KC;
        const bool s1 = ci0 < p.C1;
        cc = (s1 ? ci0 : ci0 - p.C1) * 4;
        rs = s1 ? r1 : r2;
        return s1 ? gn1 : gn2;
    };
    auto unit_load = [&](int j, int i) {
        if (i >= UPT) return;
        __amdgpu_buffer_rsrc_t rs;
        int cc;
        const bool gn = src_of(j, rs, cc);
        hv[i][0] = bld4(rs, hoff[i], cc);
        // slim: an h2/bf16 record unit is its 16-B hi piece; an fp32 prologue source is 32 B
        if (!SLIM || PRO == 1 || (PRO == 2 && gn)) hv[i][1] = bld4(rs, hoff[i], cc + 16);
    };
    // fp32 source with a GroupNorm table: silu(x*sc+sh) -> h2 in registers (zero padding stays 0)
    auto unit_transform = [&](int j, int i) {
        if constexpr (PRO == 0) return;
        if (i >= UPT) return;
        __amdgpu_buffer_rsrc_t rs;
        int cc;
        const bool gn = src_of(j, rs, cc);
        if (PRO == 2 && !gn) return;
        const int u = tid + NTHR * i;
        const int c = j * G_KC + (u < NPX ? 0 : 8);
        const float4 s0 = *reinterpret_cast<const float4*>(&Ts[c]);
        const float4 s1v = *reinterpret_cast<const float4*>(&Ts[c + 4]);
        const float4 h0 = *reinterpret_cast<const float4*>(&Ts[Cin + c]);
        const float4 h1 = *reinterpret_cast<const float4*>(&Ts[Cin + c + 4]);
        float v[8] = {silu_split_src(hv[i][0].x, s0.x, h0.x), silu_split_src(hv[i][0].y, s0.y, h0.y),
                      silu_split_src(hv[i][0].z, s0.z, h0.z), silu_split_src(hv[i][0].w, s0.w, h0.w),
                      silu_split_src(hv[i][1].x, s1v.x, h1.x), silu_split_src(hv[i][1].y, s1v.y, h1.y),
                      silu_split_src(hv[i][1].z, s1v.z, h1.z), silu_split_src(hv[i][1].w, s1v.w, h1.w)};
        if (!CIRC && hoff[i] == kOOB) {
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] = 0.f;
        }
        bool bad = false;
        split8<BF>(v, hv[i][0], hv[i][1], bad);
        if (!BF) h2_flag(p.ovf, bad);
    };
    auto unit_write = [&](int i, int buf) {
        if (i >= UPT) return;
        const int u = tid + NTHR * i;
        if (!((i + 1) * NTHR <= NU || u < NU)) return;
        if constexpr (SLIM) {  // hi piece of group g at 16 g
            float* d = &Hs[buf * HBUF + (u < NPX ? u * PXF : (u - NPX) * PXF + 4)];
            *reinterpret_cast<float4*>(d) = hv[i][0];
        } else {
            float* d = &Hs[buf * HBUF + (u < NPX ? u * PXF : (u - NPX) * PXF + 8)];
            *reinterpret_cast<float4*>(d) = hv[i][0];
            *reinterpret_cast<float4*>(d + 4) = hv[i][1];
        }
    };

    // ---- fragments.  B: fragment-ordered weights [nblk][chunk c][n][hi, lo][lane][16 B]
    int abase[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
        const int mloc = (wv * RT + rt) * 32 + li;
        abase[rt] = ((mloc / W) * W2 + (mloc % W)) * PXF + lh * (SLIM ? 4 : 8);
    }
    f32x16 acc[RT][NT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int n = 0; n < NT; ++n) acc[rt][n] = (f32x16){};
    h8 a_h[RT], a_l[RT], b_h[2][NT], b_l[2][NT];
    auto rd_a = [&](int rt, int t, int hb) {
        const int dy = t / 3, dx = t - 3 * (t / 3);
        const float* A = &Hs[hb * HBUF + abase[rt] + (dy * W2 + dx) * PXF];
        a_h[rt] = __builtin_bit_cast(h8, ld4(A));
        if constexpr (!BF) a_l[rt] = __builtin_bit_cast(h8, ld4(A + 4));
    };
    const int bl = lane * 16;
    auto ld_b = [&](int s, int c) {
        c = c < nch ? c : nch - 1;
        const int cb = ((nblk * nch + c) * NT) * 2048;  // NT fragments of [2][64][16 B]
#pragma unroll
        for (int n = 0; n < NT; ++n) {
            b_h[s][n] = __builtin_bit_cast(h8, bld4(rw, bl, cb + n * 2048));
            b_l[s][n] = __builtin_bit_cast(h8, bld4(rw, bl, cb + n * 2048 + 1024));
        }
    };
    auto mf = [&](int rt, int s) {
        if constexpr (BF) {
#pragma unroll
            for (int n = 0; n < NT; ++n)
                acc[rt][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf8, a_h[rt]),
                                                                     __builtin_bit_cast(bf8, b_h[s][n]), acc[rt][n], 0,
                                                                     0, 0);
            return;
        }
#pragma unroll
        for (int n = 0; n < NT; ++n)
            acc[rt][n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a_h[rt], b_l[s][n], acc[rt][n], 0, 0, 0);
#pragma unroll
        for (int n = 0; n < NT; ++n)
            acc[rt][n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a_l[rt], b_h[s][n], acc[rt][n], 0, 0, 0);
#pragma unroll
        for (int n = 0; n < NT; ++n)
            acc[rt][n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a_h[rt], b_h[s][n], acc[rt][n], 0, 0, 0);
    };

    // row-block-1 MFMAs of B set s with the GN+SiLU(+split) of halo unit i placed one value per gap
    auto mf1_transform = [&](int j, int i, int s) {
        if constexpr (BF) {  // one MFMA per n: the transform is not interleaved
            mf(1, s);
            unit_transform(j, i);
            return;
        }
        const int u = tid + NTHR * i;
        const int c = j * G_KC + (u < NPX ? 0 : 8);
        const float4 s0 = *reinterpret_cast<const float4*>(&Ts[c]);
        const float4 s1v = *reinterpret_cast<const float4*>(&Ts[c + 4]);
        const float4 h0 = *reinterpret_cast<const float4*>(&Ts[Cin + c]);
        const float4 h1 = *reinterpret_cast<const float4*>(&Ts[Cin + c + 4]);
        const float xs[8] = {hv[i][0].x, hv[i][0].y, hv[i][0].z, hv[i][0].w, hv[i][1].x, hv[i][1].y, hv[i][1].z,
                             hv[i][1].w};
        const float scs[8] = {s0.x, s0.y, s0.z, s0.w, s1v.x, s1v.y, s1v.z, s1v.w};
        const float shs[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
        unsigned sp[8];  // (lo << 16) | hi of each value
        bool bad = false;
        const bool zero = !CIRC && hoff[i] == kOOB;  // zero padding: the normalised ring is 0
        const h8* As[3] = {&a_h[1], &a_l[1], &a_h[1]};
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            const int g = k / 3, n = k - 3 * (k / 3);
            const h8& bb = g == 0 ? b_l[s][n] : b_h[s][n];
            acc[1][n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(*As[g], bb, acc[1][n], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
            if (k < 8) {
                float v = silu_split_src(xs[k], scs[k], shs[k]);
                v = zero ? 0.f : v;
                bad = bad || h2_bad(v);
                sp[k] = split1(v);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        unsigned h[4], l[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            h[k] = (sp[2 * k] & 0xffffu) | (sp[2 * k + 1] << 16);
            l[k] = (sp[2 * k] >> 16) | (sp[2 * k + 1] & 0xffff0000u);
        }
        hv[i][0] = make_float4(__uint_as_float(h[0]), __uint_as_float(h[1]), __uint_as_float(h[2]), __uint_as_float(h[3]));
        hv[i][1] = make_float4(__uint_as_float(l[0]), __uint_as_float(l[1]), __uint_as_float(l[2]), __uint_as_float(l[3]));
        h2_flag(p.ovf, bad);
    };
    // ---- prologue: tables, halo 0 in LDS; B(0) in registers
    if (gn1 || gn2) __syncthreads();  // Ts before the first transform
#pragma unroll
    for (int i = 0; i < UPT; ++i) unit_load(0, i);
    ld_b(0, 0);
#pragma unroll
    for (int i = 0; i < UPT; ++i) {
        unit_transform(0, i);
        unit_write(i, 0);
    }
    __syncthreads();
    rd_a(0, 0, 0);

    // one tap: T compile-time tap index, S the register set of B(c) (c & 1), HBc halo buffer of chunk j
    auto iter = [&](int j, auto T, auto S, auto HBc) {
        constexpr int t = decltype(T)::value;
        constexpr int s = decltype(S)::value;
        constexpr int hb = decltype(HBc)::value;
        const int c = 9 * j + t;
        const bool more = j + 1 < cpt;
        ld_b(s ^ 1, c + 1);
        if (t != 8) rd_a(1, t, hb);  // A1(8) was read during tap 7
        __builtin_amdgcn_sched_barrier(0);
        mf(0, s);
        __builtin_amdgcn_sched_barrier(0);
        if (c + 1 < nch) {
            if (t == 8) rd_a(0, 0, hb ^ 1);
            else rd_a(0, t + 1, hb);
        }
        __builtin_amdgcn_sched_barrier(0);
        constexpr bool st = t >= 2 && t < NLT + 2;  // this tap stores halo units UPL (t - 2) .. of chunk j+1
        if constexpr (st && PRO == 1 && UPL == 1) {
            // GN+SiLU of the unit's 8 values interleaved one per MFMA gap with the row-block-1
            // MFMAs (~10 VALU per gap, under the ~5 issue slots x 2 waves an MFMA gap hides:
            // MI355X_MICROARCH.md issue costs), the h2 split after the last one
            mf1_transform(more ? j + 1 : j, t - 2, s);
        } else {
            mf(1, s);
        }
        __builtin_amdgcn_sched_barrier(0);
        if (t == 7) rd_a(1, 8, hb);
        if constexpr (t < NLT) {  // (not stored after the last chunk)
#pragma unroll
            for (int q = 0; q < UPL; ++q) unit_load(more ? j + 1 : j, UPL * t + q);
        }
        if constexpr (st) {
            // unconditional (after the last chunk the other buffer is dead): a branch here lets hipcc
            // sink the interleaved split of mf1_transform out of the MFMA gaps into it
#pragma unroll
            for (int q = 0; q < UPL; ++q) {
                if constexpr (PRO == 2 || (PRO == 1 && UPL > 1)) unit_transform(more ? j + 1 : j, UPL * (t - 2) + q);
                unit_write(UPL * (t - 2) + q, hb ^ 1);
            }
        }
        if (t == 1 || t == 6) __syncthreads();
    };
    using S0 = std::integral_constant<int, 0>;
    using S1 = std::integral_constant<int, 1>;
    auto nine = [&](int j, auto E) {  // E: register set of tap 0 (c = 9j even <=> j even) = halo buffer
        using O = std::integral_constant<int, decltype(E)::value ^ 1>;
        iter(j, std::integral_constant<int, 0>{}, E, E);
        iter(j, std::integral_constant<int, 1>{}, O{}, E);
        iter(j, std::integral_constant<int, 2>{}, E, E);
        iter(j, std::integral_constant<int, 3>{}, O{}, E);
        iter(j, std::integral_constant<int, 4>{}, E, E);
        iter(j, std::integral_constant<int, 5>{}, O{}, E);
        iter(j, std::integral_constant<int, 6>{}, E, E);
        iter(j, std::integral_constant<int, 7>{}, O{}, E);
        iter(j, std::integral_constant<int, 8>{}, E, E);
    };
    for (int j = 0; j < cpt; j += 2) {
        nine(j, S0{});
        nine(j + 1, S1{});
    }

    __syncthreads();  // LDS -> epilogue reduction scratch
    double* red = reinterpret_cast<double*>(sm);
    conv_epi_store_rt<NT, BF ? 2 : 1, RT * NW, RT>(p, acc, m0, n0, RT * wv, lane, red);
    if (p.gn) {
        __syncthreads();
        conv_epi_gn<NT, RT * NW>(p, m0, n0, tid, NTHR, red);
    }
}

template <int W, int NW = g_nw(W)>
int launch3g(const ConvParams& p, hipStream_t st) {
    constexpr bool ONLY_BF = W == 256;  // the 256-px rows exist only in the slim bf16 form
    if (ONLY_BF && !p.bf) {
        set_error("tcx_conv2d_h2: 256-px rows on k_conv3g need bf16");
        return TCX_EINVAL;
    }
    const size_t shm = conv3g_lds_bytes(W, NW, p.Cin, p.bf);
    static bool attr[12] = {};
    const bool has1 = p.sc1 != nullptr, has2 = p.C2 > 0 && p.sc2 != nullptr;
    const int pro = !has1 && !has2 ? 0 : ((has1 && (p.C2 == 0 || has2)) ? 1 : 2);
    using K = void (*)(ConvParams);
    K ks[12] = {};
    if constexpr (!ONLY_BF) {
        const K k16[6] = {&k_conv3g<W, NW, false, 0, false>, &k_conv3g<W, NW, false, 1, false>,
                          &k_conv3g<W, NW, false, 2, false>, &k_conv3g<W, NW, true, 0, false>,
                          &k_conv3g<W, NW, true, 1, false>,  &k_conv3g<W, NW, true, 2, false>};
        for (int i = 0; i < 6; ++i) ks[i] = k16[i];
    }
    const K kb[6] = {&k_conv3g<W, NW, false, 0, true>, &k_conv3g<W, NW, false, 1, true>,
                     &k_conv3g<W, NW, false, 2, true>, &k_conv3g<W, NW, true, 0, true>,
                     &k_conv3g<W, NW, true, 1, true>,  &k_conv3g<W, NW, true, 2, true>};
    for (int i = 0; i < 6; ++i) ks[6 + i] = kb[i];
    const int ki = (p.bf ? 6 : 0) + (p.circular ? 3 : 0) + pro;
    const K kc = ks[ki];
    if (!attr[ki]) {
        const size_t mx = conv3g_lds_bytes(W, NW, 384, p.bf);
        if (hipFuncSetAttribute(reinterpret_cast<const void*>(kc), hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)mx) != hipSuccess) {
            set_error("tcx_conv2d_h2: cannot enable %zu B of dynamic LDS", mx);
            return TCX_EHIP;
        }
        attr[ki] = true;
    }
    const int grid = (p.M / g_tp(NW)) * p.n_nblk;
    hipLaunchKernelGGL(kc, dim3(grid), dim3(64 * NW), shm, st, p);
    return check_launch("tcx_conv2d_h2(halo 3g)");
}

}  // namespace
}  // namespace tcx
