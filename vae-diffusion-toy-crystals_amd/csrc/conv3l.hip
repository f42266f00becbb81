// k_conv3l: the 3x3 stride-1 circular conv of the U-Net at rows of 32 / 64 pixels (every _ConvBlock
// conv and us*_conv at 64^2 / 32^2: /root/reference/src/toycrystals/models/sde_score_model.py:102,
// 105,218,222) on the f16x3 split path, with the optional GroupNorm + SiLU prologue (:103-107) of
// k_conv3g.  Same tiles, accumulators, halo pipeline and epilogue as k_conv3g (conv3g.hip); what
// changes is where the B (weight) fragments come from.
//
// Why: k_conv3g loads every B fragment straight from global memory into each wave's registers, so
// the 4 waves of a workgroup fetch the same 6 KB per tap through the vector-memory return path.
// PMC on up1_1 (profiles/r02_ze_*): TD busy 89 %, TA busy 67 % of the kernel's cycles, MFMA pipe
// busy 48 % — the load path, not the MFMA, sets the pace.  Here each workgroup stages a tap pair's
// 12 KB of fragments ONCE (3 dwordx4 loads per wave, written with ds_write_b128 into a two-pair LDS
// ring) and every wave reads its B fragments with ds_read_b128: the load-path bytes per tap drop
// from 24 KB to 6 KB per workgroup, the LDS gets 6 extra conflict-free b128 reads per 18 MFMAs.
//
// Tap c (0 .. 9 cpt - 1, chunk j = c / 9, tap t = c % 9) of one wave:
//   ds_read B(c+1) -> register set (c+1)&1 | read A1(t) | 9 MFMAs row block 0 | read A0(t+1) |
//   9 MFMAs row block 1 (+ GN+SiLU of one halo unit) | halo unit load / store (as k_conv3g) |
//   c even: write the staged pair c/2+1 into ring slot (c/2+1)&1, load pair c/2+2, barrier.
// Pair k = taps {2k, 2k+1} is written during tap 2k-2, made visible by the barrier after it, read
// during taps 2k-1 and 2k (prefetch one tap ahead), and its slot is rewritten during tap 2k+2, after
// the barrier that ends tap 2k.  One barrier per two taps, which also orders the halo double buffer
// (halo j+1 is stored during taps 2-5 of chunk j; an even tap lies between tap 5 and tap 8).
//
// LDS (one array): halo [2][NPX][64 B] with the 16-B pieces of a pixel XOR-swizzled by (col >> 2) & 3
// (k_conv3lg at 16-px rows: (col >> 1) & 3)
// (conflict-free ds_read_b128 of 32 consecutive pixels at any tap offset, and conflict-free
// ds_write_b128 of 8 consecutive pixels), the B ring [2 pairs][2 taps][3 n][hi, lo][64 lanes][16 B]
// = 24 KB, the GroupNorm tables [2][Cin]: 78 KB at W = 64, Cin = 384 — two workgroups per CU.
#include "conv_common.hpp"

#include <algorithm>
#include <type_traits>
#include <utility>

namespace tcx {
namespace {

constexpr int L_KC = 16;     // input channels per chunk
constexpr int L_NT = 3;      // 32-channel accumulator tiles per wave (96 output channels)
constexpr int L_NW = 4;      // waves per workgroup (256-pixel tiles)
constexpr int L_TP = 64 * L_NW;
constexpr int L_PAIR = 2 * L_NT * 2 * 1024;  // bytes of B fragments per tap pair (12 KB)

__host__ __device__ constexpr int l_npx(int W) { return (L_TP / W + 2) * (W + 2); }
__host__ __device__ constexpr int l_units(int W) { return (2 * l_npx(W) + 64 * L_NW - 1) / (64 * L_NW); }
constexpr size_t conv3l_lds_bytes(int W, int Cin) {
    return (size_t)2 * l_npx(W) * 64 + 2 * (size_t)L_PAIR + 2 * (size_t)Cin * sizeof(float);
}

__device__ __forceinline__ float l_silu(float v, float sc, float sh) {
    const float y = fmaf(v, sc, sh);
    return y * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-1.4426950408889634f * y));
}

// PRO: 0 = every source h2; 1 = every source fp32 + GroupNorm table; 2 = per source at run time
// (only PRO 2, the mixed two-source prologue, is launched: k_conv3lg below serves PRO 0 and 1)
template <int W, int PRO>
__global__ __launch_bounds__(64 * L_NW, 2) void k_conv3l(ConvParams p) {
    constexpr int RT = 2, NT = L_NT, BN = 32 * NT, NTHR = 64 * L_NW;
    constexpr int W2 = W + 2;
    constexpr int NPX = l_npx(W);
    constexpr int NU = 2 * NPX;   // 8-channel halo units per chunk
    constexpr int UPT = l_units(W);
    constexpr int HB = NPX * 64;  // bytes per halo buffer
    constexpr int RING = 2 * HB;  // byte offset of the B ring
    constexpr int TAB = RING + 2 * L_PAIR;
    // row block 1 of a wave: 32 pixels further in the row (W = 64) or the next row (W = 32); the
    // swizzle term depends only on the column, so both are an immediate offset from row block 0
    constexpr int RT1 = W == 64 ? 32 * 64 : W2 * 64;
    static_assert(W == 32 || W == 64, "k_conv3l: rows of 32 or 64 pixels");
    static_assert(UPT <= 4, "halo units per thread: stores must finish by tap 5");
    extern __shared__ __attribute__((aligned(16))) float sm[];
    char* const smc = reinterpret_cast<char*>(sm);
    float* const Ts = reinterpret_cast<float*>(smc + TAB);  // [2][Cin]: scale, shift of this tile's image

    const int tid = threadIdx.x;
    const int lane = tid & 63, li = lane & 31, lh = lane >> 5;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (scalar offsets)
    const int tile = xcd_remap(blockIdx.x, gridDim.x);
    const int mblk = tile / p.n_nblk;
    const int nblk = tile - mblk * p.n_nblk;
    const int m0 = mblk * L_TP, n0 = nblk * BN;
    const int b = m0 / p.HoWo;
    const int r0 = (m0 - b * p.HoWo) / W;
    const int bs = p.bmod > 0 ? b % p.bmod : b;
    const int H = p.H;
    const int Cin = p.Cin;
    const int cpt = Cin / L_KC;  // chunks (even: Cin % 32 == 0)
    const int nch = 9 * cpt;
    const bool gn1 = PRO == 1 || (PRO == 2 && p.sc1 != nullptr);
    const bool gn2 = PRO == 1 || (PRO == 2 && p.sc2 != nullptr);

    const __amdgpu_buffer_rsrc_t r1 = mk_rsrc(p.x1, p.bytes1);
    const __amdgpu_buffer_rsrc_t r2 = mk_rsrc(p.x2 ? p.x2 : p.x1, p.x2 ? p.bytes2 : p.bytes1);
    const __amdgpu_buffer_rsrc_t rw = mk_rsrc(reinterpret_cast<const float*>(p.wf), p.bytesw);
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

    // ---- halo plan: unit u = tid + NTHR i -> halo pixel u % NPX, 8-channel group u / NPX; the
    // unit's hi piece (logical piece 2g) lands at byte 64 s + 16 ((2g) ^ sw(col)), its lo piece
    // (2g + 1) at that address ^ 16
    const int rowb = p.C1 * 4;
    int hoff[UPT];  // source byte offset of the unit
    int hdst[UPT];  // LDS byte offset of the unit's hi piece in buffer 0
#pragma unroll
    for (int i = 0; i < UPT; ++i) {
        const int u = tid + NTHR * i;
        const int hp = u < NPX ? u : u - NPX;
        const int g = u < NPX ? 0 : 1;
        const int hr = hp / W2, hc = hp - hr * W2;
        const int y = wrap_idx(r0 + hr - 1, H), x = wrap_idx(hc - 1, W);
        hoff[i] = u < NU ? ((bs * H + y) * W + x) * rowb + g * 32 : kOOB;
        hdst[i] = hp * 64 + 16 * ((2 * g) ^ ((hc >> 2) & 3));
    }
    float4 hv[UPT][2];
    auto src_of = [&](int j, __amdgpu_buffer_rsrc_t& rs, int& cc) {
        const int ci0 = j * L_KC;
        const bool s1 = ci0 < p.C1;
        cc = (s1 ? ci0 : ci0 - p.C1) * 4;
        rs = s1 ? r1 : r2;
        return s1 ? gn1 : gn2;
    };
    auto unit_load = [&](int j, int i) {
        __amdgpu_buffer_rsrc_t rs;
        int cc;
        src_of(j, rs, cc);
        hv[i][0] = bld4(rs, hoff[i], cc);
        hv[i][1] = bld4(rs, hoff[i], cc + 16);
    };
    auto unit_transform = [&](int j, int i) {
        if constexpr (PRO == 0) return;
        __amdgpu_buffer_rsrc_t rs;
        int cc;
        const bool gn = src_of(j, rs, cc);
        if (PRO == 2 && !gn) return;
        const int u = tid + NTHR * i;
        const int c = j * L_KC + (u < NPX ? 0 : 8);
        const float4 s0 = *reinterpret_cast<const float4*>(&Ts[c]);
        const float4 s1v = *reinterpret_cast<const float4*>(&Ts[c + 4]);
        const float4 h0 = *reinterpret_cast<const float4*>(&Ts[Cin + c]);
        const float4 h1 = *reinterpret_cast<const float4*>(&Ts[Cin + c + 4]);
        const float v[8] = {l_silu(hv[i][0].x, s0.x, h0.x), l_silu(hv[i][0].y, s0.y, h0.y),
                            l_silu(hv[i][0].z, s0.z, h0.z), l_silu(hv[i][0].w, s0.w, h0.w),
                            l_silu(hv[i][1].x, s1v.x, h1.x), l_silu(hv[i][1].y, s1v.y, h1.y),
                            l_silu(hv[i][1].z, s1v.z, h1.z), l_silu(hv[i][1].w, s1v.w, h1.w)};
        unsigned h[4], l[4];
        bool bad = false;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const unsigned a = split1(v[2 * k]), bb = split1(v[2 * k + 1]);
            h[k] = (a & 0xffffu) | (bb << 16);
            l[k] = (a >> 16) | (bb & 0xffff0000u);
            bad = bad || h2_bad(v[2 * k]) || h2_bad(v[2 * k + 1]);
        }
        hv[i][0] = make_float4(__uint_as_float(h[0]), __uint_as_float(h[1]), __uint_as_float(h[2]), __uint_as_float(h[3]));
        hv[i][1] = make_float4(__uint_as_float(l[0]), __uint_as_float(l[1]), __uint_as_float(l[2]), __uint_as_float(l[3]));
        h2_flag(p.ovf, bad);
    };
    auto unit_write = [&](int i, int buf) {
        const int u = tid + NTHR * i;
        if (!((i + 1) * NTHR <= NU || u < NU)) return;
        *reinterpret_cast<float4*>(smc + buf * HB + hdst[i]) = hv[i][0];
        *reinterpret_cast<float4*>(smc + buf * HB + (hdst[i] ^ 16)) = hv[i][1];
    };

    // ---- A fragment addresses: lane (li, lh) of row block 0 at tap (dy, dx) reads pixel slot
    // s = (rr + dy) W2 + cc + dx, logical pieces 2 lh (hi) and 2 lh + 1 (lo)
    int xa[3];
    {
        const int mloc = (wv * RT) * 32 + li;
        const int rr = mloc / W, cc = mloc % W;
#pragma unroll
        for (int dx = 0; dx < 3; ++dx)
            xa[dx] = (rr * W2 + cc + dx) * 64 + 16 * ((2 * lh) ^ (((cc + dx) >> 2) & 3));
    }
    f32x16 acc[RT][NT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int n = 0; n < NT; ++n) acc[rt][n] = (f32x16){};
    h8 a_h[RT], a_l[RT], b_h[2][NT], b_l[2][NT];
    auto rd_a = [&](int rt, int t, int hb) {
        const int dy = t / 3, dx = t - 3 * (t / 3);
        const int off = hb * HB + rt * RT1 + dy * W2 * 64;
        a_h[rt] = __builtin_bit_cast(h8, *reinterpret_cast<const float4*>(smc + xa[dx] + off));
        a_l[rt] = __builtin_bit_cast(h8, *reinterpret_cast<const float4*>(smc + (xa[dx] ^ 16) + off));
    };
    // B(c) from the ring: pair slot (c >> 1) & 1, tap c & 1 of the pair; fragment n hi at +2 KB n
    const int bl = lane * 16;
    auto rd_b = [&](int s, int c) {
        const char* B = smc + RING + ((c >> 1) & 1) * L_PAIR + (c & 1) * (L_PAIR / 2) + bl;
#pragma unroll
        for (int n = 0; n < NT; ++n) {
            b_h[s][n] = __builtin_bit_cast(h8, *reinterpret_cast<const float4*>(B + n * 2048));
            b_l[s][n] = __builtin_bit_cast(h8, *reinterpret_cast<const float4*>(B + n * 2048 + 1024));
        }
    };
    // staging of pair k: wave wv moves KB [3 wv, 3 wv + 3) of the pair's 12 KB
    float4 bst[3];
    const int npair = nch / 2;
    const int bsl = bl + wv * 3072;  // this wave's bytes of a pair (VGPR offset)
    auto ld_pair = [&](int k) {
        k = k < npair ? k : npair - 1;
        const int base = (nblk * nch + 2 * k) * NT * 2048;
#pragma unroll
        for (int i = 0; i < 3; ++i) bst[i] = bld4(rw, bsl, base + i * 1024);
    };
    auto wr_pair = [&](int k) {
        char* d = smc + RING + (k & 1) * L_PAIR + wv * 3072 + bl;
#pragma unroll
        for (int i = 0; i < 3; ++i) *reinterpret_cast<float4*>(d + i * 1024) = bst[i];
    };
    auto mf = [&](int rt, int s) {
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
    // row-block-1 MFMAs with the GN+SiLU(+split) of halo unit i placed one value per gap (k_conv3g)
    auto mf1_transform = [&](int j, int i, int s) {
        const int u = tid + NTHR * i;
        const int c = j * L_KC + (u < NPX ? 0 : 8);
        const float4 s0 = *reinterpret_cast<const float4*>(&Ts[c]);
        const float4 s1v = *reinterpret_cast<const float4*>(&Ts[c + 4]);
        const float4 h0 = *reinterpret_cast<const float4*>(&Ts[Cin + c]);
        const float4 h1 = *reinterpret_cast<const float4*>(&Ts[Cin + c + 4]);
        const float xs[8] = {hv[i][0].x, hv[i][0].y, hv[i][0].z, hv[i][0].w, hv[i][1].x, hv[i][1].y, hv[i][1].z,
                             hv[i][1].w};
        const float scs[8] = {s0.x, s0.y, s0.z, s0.w, s1v.x, s1v.y, s1v.z, s1v.w};
        const float shs[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
        unsigned sp[8];
        bool bad = false;
        const h8* As[3] = {&a_h[1], &a_l[1], &a_h[1]};
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            const int g = k / 3, n = k - 3 * (k / 3);
            const h8& bb = g == 0 ? b_l[s][n] : b_h[s][n];
            acc[1][n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(*As[g], bb, acc[1][n], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
            if (k < 8) {
                const float v = l_silu(xs[k], scs[k], shs[k]);
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

    // ---- prologue: tables, pair 0 in the ring, pair 1 staged, halo 0 in LDS; B(0), A0(0) in registers
    ld_pair(0);
#pragma unroll
    for (int i = 0; i < UPT; ++i) unit_load(0, i);
    if (gn1 || gn2) __syncthreads();  // Ts before the first transform
    wr_pair(0);
    ld_pair(1);
#pragma unroll
    for (int i = 0; i < UPT; ++i) {
        unit_transform(0, i);
        unit_write(i, 0);
    }
    __syncthreads();
    rd_b(0, 0);
    rd_a(0, 0, 0);

    // one tap: T compile-time tap index, S = c & 1 (register set of B(c)), HBc halo buffer of chunk j
    auto iter = [&](int j, auto T, auto S, auto HBc) {
        constexpr int t = decltype(T)::value;
        constexpr int s = decltype(S)::value;
        constexpr int hb = decltype(HBc)::value;
        const int c = 9 * j + t;
        const bool more = j + 1 < cpt;
        rd_b(s ^ 1, c + 1);
        if (t != 8) rd_a(1, t, hb);  // A1(8) was read during tap 7
        __builtin_amdgcn_sched_barrier(0);
        mf(0, s);
        __builtin_amdgcn_sched_barrier(0);
        if (t == 8) rd_a(0, 0, hb ^ 1);
        else rd_a(0, t + 1, hb);
        __builtin_amdgcn_sched_barrier(0);
        constexpr bool st = t >= 2 && t < UPT + 2;  // this tap stores halo unit t - 2 of chunk j+1
        if constexpr (st && PRO == 1) {
            mf1_transform(more ? j + 1 : j, t - 2, s);
        } else {
            mf(1, s);
        }
        __builtin_amdgcn_sched_barrier(0);
        if (t == 7) rd_a(1, 8, hb);
        if constexpr (t < UPT) unit_load(more ? j + 1 : j, t);
        if constexpr (st) {
            if constexpr (PRO == 2) unit_transform(more ? j + 1 : j, t - 2);
            unit_write(t - 2, hb ^ 1);
        }
        if constexpr (s == 0) {  // c even: pair c/2 + 1 into the ring, load pair c/2 + 2, barrier
            wr_pair((c >> 1) + 1);
            ld_pair((c >> 1) + 2);
            __syncthreads();
        }
    };
    auto nine = [&](int j, auto E) {  // E = (9 j) & 1 = j & 1: register set of tap 0 = halo buffer
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
    using S0 = std::integral_constant<int, 0>;
    using S1 = std::integral_constant<int, 1>;
    for (int j = 0; j < cpt; j += 2) {
        nine(j, S0{});
        nine(j + 1, S1{});
    }

    __syncthreads();  // LDS -> epilogue reduction scratch
    double* red = reinterpret_cast<double*>(sm);
    conv_epi_store_rt<NT, 1, RT * L_NW, RT>(p, acc, m0, n0, RT * wv, lane, red);
    if (p.gn) {
        __syncthreads();
        conv_epi_gn<NT, RT * L_NW>(p, m0, n0, tid, NTHR, red);
    }
}


// ---- k_conv3lg: the single-source forms (PRO 0: h2 source; PRO 1: fp32 source + GroupNorm+SiLU
// tables) with ALL staging by LDS-DMA and split roles.
// vmcnt is one in-order counter per wave: in k_conv3l a wait for a tap pair's weights (L2, issued
// two taps earlier) also waits for every halo load issued before it (HBM), so the halo gets at most
// ~2 taps of latency cover; ablations at up1_1 (profiles/r02_zi_*): no halo staging -9 %, no weight
// staging -6 % of the launch.  Here waves 0-1 move the weight pairs (6 x 1 KB buffer_load ... lds
// each per pair) and waves 2-3 the halo (13 / 12 x 1 KB per chunk): a wave only ever waits for its
// own kind of load.  The halo of chunk j+1 is issued at the start of taps 0-3 of chunk j and waited for
// at tap 6/7 (4-7 taps of cover), a pair at the start of tap 2k-3 and waited for at the end of 2k-2.  No VGPR staging, no
// ds_write; waits are explicit s_waitcnt before raw s_barrier (hipcc's __syncthreads would drain
// every LDS-DMA in flight).  The halo slot image is the swizzled one of k_conv3l, written lane-
// linearly: lane l of halo instruction i fills slot 16 i + l / 4, physical piece l % 4, so it reads
// logical piece (l % 4) ^ sw(col) of that pixel (the per-lane source address carries the swizzle).
// PRO 1: the halo waves DMA the raw fp32 chunk (16 channels = 64 B per pixel, the size of its h2
// record) into the same slots; it is published by the barrier of tap 4 (even chunk) / 5 (odd), and
// during the next two taps every wave rewrites its quarter of the units IN PLACE as h2 of
// silu(x sc + sh) (per unit: two ds_read_b128, eight values one per MFMA gap, two ds_write_b128).
// Waves 0-1 own the 8-channel group 0 of every slot, waves 2-3 group 1, so a wave's GroupNorm
// scale/shift for the chunk are 16 wave-uniform values (SGPRs, from the LDS copy of the image's tables).
__device__ __forceinline__ void lds_dma16(__amdgpu_buffer_rsrc_t r, char* lds, int voff, int soff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, voff, soff, 0, 0);
}
constexpr int WAIT_VM0 = 0x0F70;    // s_waitcnt vmcnt(0)
constexpr int WAIT_LGKM0 = 0xC07F;  // s_waitcnt lgkmcnt(0)

// GroupNorm-prologue transform schedules (k_conv3lg PRO 1), two task slots per MFMA gap: 0-7 value k, 8-11 channel pair k - 8, 12 the
// write-back, -1 none.  S1: one unit over both row blocks' 18 gaps; S2: one unit in one row block's 9
// gaps (the odd chunk's tap 6 carries two units)
constexpr int kTvS1[36] = {0, -1, 1, -1, 8, -1, 2, -1, 3, -1, 9, -1, -1, -1, -1, -1, -1, -1,
                           4, -1, 5, -1, 10, -1, 6, -1, 7, -1, 11, 12, -1, -1, -1, -1, -1, -1};
constexpr int kTvS2[18] = {0, -1, 1, 8, 2, -1, 3, 9, 4, -1, 5, 10, 6, -1, 7, 11, 12, -1};
template <int SCH, int G, int SLOT>
struct TvCode {
    static constexpr int value = SCH == 1 ? kTvS1[2 * G + SLOT] : kTvS2[2 * G + SLOT];
};
template <typename F, int... Is>
__device__ __forceinline__ void static_for(F&& f, std::integer_sequence<int, Is...>) {
    (f(std::integral_constant<int, Is>{}), ...);
}

// PQ (PRO 1): the raw halo's DMA is spread over taps 0 .. PQ - 1 (r03_s: 3 taps ~1 % faster than 2 on the
// prologue layers, 4 equal to 3; the wait stays at tap 4 / 5)
// PRO 1's GroupNorm tables: staged in LDS once per workgroup and read per chunk with broadcast
// ds_reads issued at tap 8 and moved to SGPRs at tap 0 (r03_t: ~1 % faster than two scalar loads +
// lgkmcnt(0) per chunk at tap 8, which also waited for every LDS read in flight)
template <int W, int PRO, int PQ = 3>
__global__ __launch_bounds__(64 * L_NW, 2) void k_conv3lg(ConvParams p) {
    constexpr int RT = 2, NT = L_NT, NTHR = 64 * L_NW;
    constexpr int W2 = W + 2;
    constexpr int NPX = l_npx(W);
    constexpr int NI = (NPX + 15) / 16;  // halo instructions per chunk (16 slots each)
    constexpr int NIH = (NI + 1) / 2;    // per halo wave (wave 2: even i, wave 3: odd i)
    constexpr int HB = NI * 16 * 64;
    constexpr int RING = 2 * HB;
    // row block 1 of a wave: 32 pixels on (W = 64), the next row (32), two rows on (16)
    constexpr int RT1 = W == 64 ? 32 * 64 : (W == 32 ? W2 * 64 : 2 * W2 * 64);
    static_assert(W == 16 || W == 32 || W == 64, "k_conv3lg: rows of 16, 32 or 64 pixels");
    // piece swizzle by column: (col >> 2) & 3 at 32/64-px rows; at 16-px rows a row block spans two
    // rows, for which (col >> 1) & 3 is the conflict-free choice (exhaustive check over taps/rows)
    auto sw = [](int col) { return W == 16 ? (col >> 1) & 3 : (col >> 2) & 3; };
    extern __shared__ __attribute__((aligned(16))) float sm[];
    char* const smc = reinterpret_cast<char*>(sm);
    // LDS-DMA destinations from a base the optimiser cannot fold to a constant: a compile-time LDS
    // address reaches instruction selection as a constant local->flat->local cast whose null check
    // hipcc cannot encode ("Operand has incorrect register class")
    int lz;
    asm volatile("s_mov_b32 %0, 0" : "=s"(lz));
    char* const smd = smc + lz;

    const int tid = threadIdx.x;
    const int lane = tid & 63, li = lane & 31, lh = lane >> 5;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int tile = xcd_remap(blockIdx.x, gridDim.x);
    const int mblk = tile / p.n_nblk;
    const int nblk = tile - mblk * p.n_nblk;
    const int m0 = mblk * L_TP, n0 = nblk * 32 * NT;
    const int b = m0 / p.HoWo;
    const int r0 = (m0 - b * p.HoWo) / W;
    const int bs = p.bmod > 0 ? b % p.bmod : b;
    const int H = p.H;
    const int cpt = p.Cin / L_KC;
    const int nch = 9 * cpt;
    const int npair = nch / 2;

    const __amdgpu_buffer_rsrc_t r1 = mk_rsrc(p.x1, p.bytes1);
    const __amdgpu_buffer_rsrc_t r2 = mk_rsrc(p.x2 ? p.x2 : p.x1, p.x2 ? p.bytes2 : p.bytes1);
    const __amdgpu_buffer_rsrc_t rw = mk_rsrc(reinterpret_cast<const float*>(p.wf), p.bytesw);

    // halo waves: the per-lane source offset of instruction i (computed at issue: keeping all 13 live
    // across the tap loop cost more registers than the ~12 VALU per instruction; the chunk's channel
    // offset rides in soffset)
    const int hw = wv & 1;
    const int rowb = p.C1 * 4;
    const int img0 = bs * H;
    // slot 16 i + ls (ls = lane / 4) of instruction i (compile-time i after unrolling) lies in halo
    // row R(i) or R(i) + 1: the row's image offset (with the circular wrap) is wave-uniform scalar
    // work, the lane only selects between the two and adds its column
    const int ls = lane >> 2;
    auto halo_voff = [&](int i) {
        const int hr0 = (16 * i) / W2;                // compile-time after unrolling
        const int th = W2 * (hr0 + 1) - 16 * i;       // lanes with ls >= th are in row hr0 + 1
        const int y0 = wrap_idx(r0 + hr0 - 1, H), y1 = wrap_idx(r0 + hr0, H);
        const int yo0 = (img0 + y0) * W * rowb, yo1 = (img0 + y1) * W * rowb;
        const bool nx = ls >= th;
        int hc = 16 * i - hr0 * W2 + ls - (nx ? W2 : 0);
        const int sl = 16 * i + ls;
        const int hcs = hc;                            // the slot's own column (its swizzle)
        if (sl >= NPX) hc = (NPX - 1) % W2;            // padding slots read a valid pixel
        const int x = hc == 0 ? W - 1 : (hc == W + 1 ? 0 : hc - 1);
        const int yo = (sl >= NPX) ? (img0 + wrap_idx(r0 + (NPX - 1) / W2 - 1, H)) * W * rowb : (nx ? yo1 : yo0);
        return yo + x * rowb + 16 * ((lane & 3) ^ sw(hcs));
    };
    auto halo_issue = [&](int j, int buf, int q0, int q1) {
        const int ci0 = j * L_KC;
        const bool s1 = ci0 < p.C1;
        const int cc = (s1 ? ci0 : ci0 - p.C1) * 4;
        const __amdgpu_buffer_rsrc_t rs = s1 ? r1 : r2;
#pragma unroll
        for (int q = 0; q < NIH; ++q) {
            if (q < q0 || q >= q1) continue;
            const int i = 2 * q + hw;
            if (i < NI) lds_dma16(rs, smd + buf * HB + i * 1024, halo_voff(i), cc);
        }
    };
    // weight waves: pair k (12 KB) -> ring slot k & 1; wave w moves KB [6 w, 6 w + 6)
    auto pair_issue = [&](int k) {
        k = k < npair ? k : npair - 1;
        const int base = (nblk * nch + 2 * k) * NT * 2048 + wv * 6144;
        char* const d = smd + RING + (k & 1) * L_PAIR + wv * 6144;
#pragma unroll
        for (int i = 0; i < 6; ++i) lds_dma16(rw, d + i * 1024, lane * 16, base + i * 1024);
    };

    int xa[3];
    {
        const int mloc = (wv * RT) * 32 + li;
        const int rr = mloc / W, cc = mloc % W;
#pragma unroll
        for (int dx = 0; dx < 3; ++dx)
            xa[dx] = (rr * W2 + cc + dx) * 64 + 16 * ((2 * lh) ^ sw(cc + dx));
    }
    f32x16 acc[RT][NT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int n = 0; n < NT; ++n) acc[rt][n] = (f32x16){};
    h8 a_h[RT], a_l[RT], b_h[2][NT], b_l[2][NT];
    auto rd_a = [&](int rt, int t, int hb) {
        const int dy = t / 3, dx = t - 3 * (t / 3);
        const int off = hb * HB + rt * RT1 + dy * W2 * 64;
        a_h[rt] = __builtin_bit_cast(h8, *reinterpret_cast<const float4*>(smc + xa[dx] + off));
        a_l[rt] = __builtin_bit_cast(h8, *reinterpret_cast<const float4*>(smc + (xa[dx] ^ 16) + off));
    };
    const int bl = lane * 16;
    auto rd_b = [&](int s, int c) {
        const char* B = smc + RING + ((c >> 1) & 1) * L_PAIR + (c & 1) * (L_PAIR / 2) + bl;
#pragma unroll
        for (int n = 0; n < NT; ++n) {
            b_h[s][n] = __builtin_bit_cast(h8, *reinterpret_cast<const float4*>(B + n * 2048));
            b_l[s][n] = __builtin_bit_cast(h8, *reinterpret_cast<const float4*>(B + n * 2048 + 1024));
        }
    };
    auto mf = [&](int rt, int s) {
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
    auto barrier = [&]() {
        __builtin_amdgcn_s_waitcnt(WAIT_LGKM0);
        __builtin_amdgcn_s_barrier();
    };

    // PRO 1: units of this wave: group g = wv >> 1, slots (wv & 1) 64 + lane + 128 i (i < 4)
    constexpr int NPXS = NPX;
    constexpr int TU = (NPX + 127) / 128;  // units per thread: 4 at 64-px rows, 3 at 32 and 16
    const int tg = wv >> 1;
    // lanes past the last slot rewrite a padding slot (no divergence around MFMAs); several lanes
    // share one, so what they read may already be another lane's h2: their range flag is masked
    int tdst[TU];
    unsigned tval = 0;
#pragma unroll
    for (int i = 0; i < TU; ++i) {
        const int hp0 = (wv & 1) * 64 + lane + 128 * i;
        const int hp = hp0 < NPXS ? hp0 : NPXS + (lane & 3);
        const int hc = hp % W2;
        tdst[i] = hp * 64 + 16 * ((2 * tg) ^ sw(hc));
        tval |= hp0 < NPXS ? 1u << i : 0u;
    }
    float tsc[8], tsh[8];  // this wave's group of the chunk being transformed (wave-uniform)
    // tables in LDS after the ring ([sc | sh][Cin]); issue = 4 broadcast ds_read_b128 into tq, commit =
    // readfirstlane into the SGPR copies
    const float* const TsL = reinterpret_cast<const float*>(smc + RING + 2 * L_PAIR);
    float4 tq[4];
    auto issue_tabs = [&](int j) {
        const float* t = TsL + j * L_KC + 8 * tg;
        tq[0] = *reinterpret_cast<const float4*>(t);
        tq[1] = *reinterpret_cast<const float4*>(t + 4);
        tq[2] = *reinterpret_cast<const float4*>(t + p.C1);
        tq[3] = *reinterpret_cast<const float4*>(t + p.C1 + 4);
    };
    auto commit_tabs = [&]() {
        const float* q = reinterpret_cast<const float*>(tq);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            tsc[k] = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, q[k])));
            tsh[k] = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, q[8 + k])));
        }
    };
    // A unit's 8 values spread over the 18 MFMA gaps of a tap (rb 0: gaps 0-8, rb 1: 9-17).
    // Per gap at most one value (fma, exp2, add, rcp, mul: 5 VALU, two of them 8-cycle transcendentals)
    // or one channel pair's h2 split (cvt_pk, 2 cvt back, 2 sub, cvt_pk); the write-back of the two
    // 16-B pieces after the last split.  Out-of-range values are caught by a running max of |v|
    // (v_max3: half an instruction per value) checked once per unit (a NaN source stays NaN in either
    // precision, so only finite overflow matters).
    typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    struct TUnit {
        float x[8], v[8];
        unsigned hi[4], lo[4];
        float m;
    };
    auto tu_load = [&](TUnit& u, int i, int buf) {
        const float4 x0 = *reinterpret_cast<const float4*>(smc + buf * HB + tdst[i]);
        const float4 x1 = *reinterpret_cast<const float4*>(smc + buf * HB + (tdst[i] ^ 16));
        u.x[0] = x0.x; u.x[1] = x0.y; u.x[2] = x0.z; u.x[3] = x0.w;
        u.x[4] = x1.x; u.x[5] = x1.y; u.x[6] = x1.z; u.x[7] = x1.w;
        u.m = 0.f;
    };
    auto tu_val = [&](TUnit& u, int k) { u.v[k] = l_silu(u.x[k], tsc[k], tsh[k]); };
    auto tu_pair = [&](TUnit& u, int q) {
        const f32x2 v = {u.v[2 * q], u.v[2 * q + 1]};
        const f16x2 h = __builtin_convertvector(v, f16x2);
        const f32x2 r = v - __builtin_convertvector(h, f32x2);
        const f16x2 l = __builtin_convertvector(r, f16x2);
        u.hi[q] = __builtin_bit_cast(unsigned, h);
        u.lo[q] = __builtin_bit_cast(unsigned, l);
        u.m = fmaxf(u.m, fmaxf(fabsf(v[0]), fabsf(v[1])));
    };
    auto tu_store = [&](TUnit& u, int i, int buf, bool live) {
        *reinterpret_cast<uint4*>(smc + buf * HB + tdst[i]) = make_uint4(u.hi[0], u.hi[1], u.hi[2], u.hi[3]);
        *reinterpret_cast<uint4*>(smc + buf * HB + (tdst[i] ^ 16)) = make_uint4(u.lo[0], u.lo[1], u.lo[2], u.lo[3]);
        h2_flag(p.ovf, !(u.m < kH2Max) && live && ((tval >> i) & 1));
    };
    // one task (compile-time code C) of a gap
    auto tu_task = [&](TUnit& u, auto C, int i, int buf, bool live) {
        constexpr int code = decltype(C)::value;
        if constexpr (code >= 0 && code < 8) tu_val(u, code);
        else if constexpr (code >= 8 && code < 12) tu_pair(u, code - 8);
        else if constexpr (code == 12) tu_store(u, i, buf, live);
    };
    // the 9 MFMAs of row block rt with the tasks of gaps [G0, G0 + 9) of schedule SCH on unit u
    auto mf_tasks = [&](int rt, int s, TUnit& u, auto SCH, auto G0, int i, int buf, bool live) {
        constexpr int sch = decltype(SCH)::value, g0 = decltype(G0)::value;
        static_for([&](auto K) {
            constexpr int k = decltype(K)::value;
            constexpr int g = k / 3, n = k - 3 * (k / 3);
            const h8& aa = g == 1 ? a_l[rt] : a_h[rt];
            const h8& bb = g == 0 ? b_l[s][n] : b_h[s][n];
            acc[rt][n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(aa, bb, acc[rt][n], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
            tu_task(u, std::integral_constant<int, TvCode<sch, g0 + k, 0>::value>{}, i, buf, live);
            tu_task(u, std::integral_constant<int, TvCode<sch, g0 + k, 1>::value>{}, i, buf, live);
            __builtin_amdgcn_sched_barrier(0);
        }, std::make_integer_sequence<int, 9>{});
    };
    // the whole chunk's transform at once (prologue)
    auto transform_all = [&](int buf) {
#pragma unroll
        for (int i = 0; i < TU; ++i) {
            char* const d = smc + buf * HB + tdst[i];
            const float4 x0 = *reinterpret_cast<const float4*>(d);
            const float4 x1 = *reinterpret_cast<const float4*>(smc + buf * HB + (tdst[i] ^ 16));
            const float xs[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
            unsigned sp[8];
            bool bad = false;
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const float v = l_silu(xs[k], tsc[k], tsh[k]);
                bad = bad || h2_bad(v);
                sp[k] = split1(v);
            }
            unsigned h[4], l[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                h[k] = (sp[2 * k] & 0xffffu) | (sp[2 * k + 1] << 16);
                l[k] = (sp[2 * k] >> 16) | (sp[2 * k + 1] & 0xffff0000u);
            }
            *reinterpret_cast<float4*>(d) =
                make_float4(__uint_as_float(h[0]), __uint_as_float(h[1]), __uint_as_float(h[2]), __uint_as_float(h[3]));
            *reinterpret_cast<float4*>(smc + buf * HB + (tdst[i] ^ 16)) =
                make_float4(__uint_as_float(l[0]), __uint_as_float(l[1]), __uint_as_float(l[2]), __uint_as_float(l[3]));
            h2_flag(p.ovf, bad && ((tval >> i) & 1));
        }
    };

    // ---- prologue: pairs 0, 1 and halo 0 in LDS (PRO 1: and the image's GroupNorm tables)
    if (wv < 2) {
        pair_issue(0);
        pair_issue(1);
    } else {
        halo_issue(0, 0, 0, NIH);
    }
    if constexpr (PRO == 1) {
        float* const Tw = reinterpret_cast<float*>(smc + RING + 2 * L_PAIR);
        for (int c = tid; c < p.C1; c += NTHR) {
            Tw[c] = p.sc1[(size_t)b * p.C1 + c];
            Tw[p.C1 + c] = p.sh1[(size_t)b * p.C1 + c];
        }
    }
    __builtin_amdgcn_s_waitcnt(WAIT_VM0);
    barrier();
    if constexpr (PRO == 1) {
        issue_tabs(0);
        commit_tabs();
        transform_all(0);
        barrier();
        if (cpt > 1) issue_tabs(1);  // committed at tap 0 of chunk 0
    }
    rd_b(0, 0);
    rd_a(0, 0, 0);

    auto iter = [&](int j, auto T, auto S, auto HBc) {
        constexpr int t = decltype(T)::value;
        constexpr int s = decltype(S)::value;
        constexpr int hb = decltype(HBc)::value;
        const int c = 9 * j + t;
        // PRO 1: raw halo j+1 published by the barrier of tap 4 (even chunk) / 5 (odd); one unit per
        // tap transformed in the row-block-0 MFMA gaps from the next tap on (even chunk: taps 5-8;
        // odd: units 0 and 1 in tap 6, then 7, 8); the h2 is published by a barrier at the end of tap
        // 8 (an extra one in an odd chunk), so A0 of the next chunk's tap 0 is read after it
        constexpr int TR = hb ? 6 : 5;  // first transform tap
        constexpr bool tr = PRO == 1 && t >= TR && (hb ? (t == 6 ? 0 : t - 5) : t - 5) < TU;  // unit u0
        constexpr int u0 = hb ? (t == 6 ? 0 : t - 5) : t - 5;
        constexpr bool tr1 = PRO == 1 && hb && t == 6;  // and unit u1 = 1 (odd chunk's tap 6)
        constexpr int u1 = 1;
        constexpr bool pre_a0 = PRO == 0;  // tap 8 prefetches A0 of the next chunk
        // (measured r03_l: moving the transform to taps 5-6 / 6-7 so that tap 8 prefetches A0 and the
        // odd chunk's extra barrier goes, two units per tap, was 0-2 % slower per layer)
        const bool more = j + 1 < cpt;
        // LDS-DMA issue first thing in the tap (right after the barrier that freed the target): a
        // pair issued at the start of odd tap 2k-3 has two taps of latency cover before its wait
        if (wv < 2) {
            if constexpr (s == 1) pair_issue((c + 3) >> 1);
        } else if constexpr (PRO == 0 ? t < 4 : t < PQ) {
            // halo of chunk j+1 into the other buffer (not after the last chunk): PRO 0 a quarter per
            // tap over taps 0-3, PRO 1 a third per tap over taps 0-2 (the raw data is waited for at tap 4/5)
            constexpr int NQ = PRO == 0 ? 4 : PQ;
            constexpr int q0 = (NIH * t) / NQ, q1 = (NIH * (t + 1)) / NQ;
            if (more) halo_issue(j + 1, hb ^ 1, q0, q1);
        }
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (!pre_a0 && t == 0) rd_a(0, 0, hb);  // published at the end of the last tap
        if constexpr (PRO == 1 && t == 0) commit_tabs();  // tables of chunk j + 1
        rd_b(s ^ 1, c + 1);
        if (t != 8) rd_a(1, t, hb);
        __builtin_amdgcn_sched_barrier(0);
        using I0 = std::integral_constant<int, 0>;
        using I1 = std::integral_constant<int, 1>;
        using I2 = std::integral_constant<int, 2>;
        using I9 = std::integral_constant<int, 9>;
        TUnit ua, ub;
        if constexpr (tr) {
            tu_load(ua, u0, hb ^ 1);
            if constexpr (tr1) tu_load(ub, u1, hb ^ 1);
        }
        if constexpr (tr1) mf_tasks(0, s, ua, I2{}, I0{}, u0, hb ^ 1, more);
        else if constexpr (tr) mf_tasks(0, s, ua, I1{}, I0{}, u0, hb ^ 1, more);
        else mf(0, s);
        __builtin_amdgcn_sched_barrier(0);
        if (t == 8) {
            if constexpr (pre_a0) rd_a(0, 0, hb ^ 1);
        } else {
            rd_a(0, t + 1, hb);
        }
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (tr1) mf_tasks(1, s, ub, I2{}, I0{}, u1, hb ^ 1, more);
        else if constexpr (tr) mf_tasks(1, s, ua, I1{}, I9{}, u0, hb ^ 1, more);
        else mf(1, s);
        __builtin_amdgcn_sched_barrier(0);
        if (t == 7) rd_a(1, 8, hb);
        if constexpr (PRO == 1 && t == 8) {
            if (j + 2 < cpt) issue_tabs(j + 2);
            if constexpr (s == 1) barrier();  // odd chunk: publish the transformed halo
        }
        if constexpr (s == 0) {  // even tap: the barrier that publishes pair c/2 + 1 (and halo j+1:
                                 // PRO 0 at tap 6 of an even chunk / 7 of an odd one; PRO 1 the raw
                                 // data at tap 4 / 5)
            constexpr bool halo_wait = PRO == 0 ? t == (hb ? 7 : 6) : t == TR - 1;
            if (wv < 2 || halo_wait) __builtin_amdgcn_s_waitcnt(WAIT_VM0);
            barrier();
        }
    };
    auto nine = [&](int j, auto E) {
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
    using S0 = std::integral_constant<int, 0>;
    using S1 = std::integral_constant<int, 1>;
    for (int j = 0; j < cpt; j += 2) {
        nine(j, S0{});
        nine(j + 1, S1{});
    }

    __builtin_amdgcn_s_waitcnt(WAIT_VM0);  // the clamped tail pairs land before LDS is reused
    __syncthreads();
    double* red = reinterpret_cast<double*>(sm);
    conv_epi_store_rt<NT, 1, RT * L_NW, RT>(p, acc, m0, n0, RT * wv, lane, red);
    if (p.gn) {
        __syncthreads();
        conv_epi_gn<NT, RT * L_NW>(p, m0, n0, tid, NTHR, red);
    }
}

template <int W>
constexpr size_t conv3lg_lds_bytes() {  // + the GroupNorm tables of PRO 1 ([2][Cin <= 384] floats)
    return (size_t)2 * ((l_npx(W) + 15) / 16) * 16 * 64 + 2 * (size_t)L_PAIR + 2 * 384 * sizeof(float);
}

template <int W>
int launch3l(const ConvParams& p, hipStream_t st) {
    const bool has1 = p.sc1 != nullptr, has2 = p.C2 > 0 && p.sc2 != nullptr;
    const int grid = (p.M / L_TP) * p.n_nblk;
    using K = void (*)(ConvParams);
    if ((!has1 && !has2) || (has1 && p.C2 == 0)) {  // PRO 0 (h2 sources) or 1 (one fp32 source): LDS-DMA form
        const int pro = has1 ? 1 : 0;
        static bool attr_g[2] = {};
        const K kg = pro ? &k_conv3lg<W, 1> : &k_conv3lg<W, 0>;
        const int ai = pro;
        if (!attr_g[ai]) {
            if (hipFuncSetAttribute(reinterpret_cast<const void*>(kg), hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)conv3lg_lds_bytes<W>()) != hipSuccess) {
                set_error("tcx_conv2d_h2: cannot enable %zu B of dynamic LDS", conv3lg_lds_bytes<W>());
                return TCX_EHIP;
            }
            attr_g[ai] = true;
        }
        hipLaunchKernelGGL(kg, dim3(grid), dim3(64 * L_NW), conv3lg_lds_bytes<W>(), st, p);
        return check_launch("tcx_conv2d_h2(halo 3lg)");
    }
    // two sources, one of them with a GroupNorm prologue: the register-staged k_conv3l
    static bool attr = false;
    const K kc = &k_conv3l<W, 2>;
    if (!attr) {
        if (hipFuncSetAttribute(reinterpret_cast<const void*>(kc), hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)conv3l_lds_bytes(W, 384)) != hipSuccess) {
            set_error("tcx_conv2d_h2: cannot enable %zu B of dynamic LDS", conv3l_lds_bytes(W, 384));
            return TCX_EHIP;
        }
        attr = true;
    }
    hipLaunchKernelGGL(kc, dim3(grid), dim3(64 * L_NW), conv3l_lds_bytes(W, p.Cin), st, p);
    return check_launch("tcx_conv2d_h2(halo 3l)");
}

}  // namespace

// TCX_CONV3L=0 keeps k_conv3g at rows of 32 / 64 pixels (A/B measurements)
bool conv3l_enabled() {
    static const bool on = [] {
        const char* e = getenv("TCX_CONV3L");
        return !(e && e[0] == '0');
    }();
    return on;
}

bool conv3m_takes(const ConvParams& p);

// called by launch_conv3g once conv3g_applies() holds (fragment-ordered weights, Cin % 32 == 0,
// Cin <= 384, cout_pad % 96 == 0, whole-row tiles)
bool conv3l_takes(const ConvParams& p) {
    if (!conv3l_enabled() || p.bf || !p.circular || p.M % L_TP != 0 || p.HoWo % L_TP != 0) return false;
    if (p.W == 32 || p.W == 64) return true;
    if (conv3m_takes(p)) return true;  // 16-px rows: the 16x16x32 forms, incl. the GroupNorm prologue
    // 16-px rows: the LDS-DMA kernel for h2 sources (mid.net.0: 2 % faster than k_conv3g); its
    // GroupNorm prologue form is 9 % slower than k_conv3g's there (profiles/r02_zt_*), so that stays
    return p.W == 16 && p.sc1 == nullptr && !(p.C2 > 0 && p.sc2 != nullptr);
}

// 16-px rows (the mid block, one 256-pixel tile per 16x16 image): only the LDS-DMA form exists
template <int PRO>
int launch3lg16(const ConvParams& p, hipStream_t st) {
    static bool attr = false;
    if (!attr) {
        if (hipFuncSetAttribute(reinterpret_cast<const void*>(&k_conv3lg<16, PRO>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)conv3lg_lds_bytes<16>()) != hipSuccess) {
            set_error("tcx_conv2d_h2: cannot enable %zu B of dynamic LDS", conv3lg_lds_bytes<16>());
            return TCX_EHIP;
        }
        attr = true;
    }
    const int grid = (p.M / L_TP) * p.n_nblk;
    void (*const kg)(ConvParams) = &k_conv3lg<16, PRO>;
    hipLaunchKernelGGL(kg, dim3(grid), dim3(64 * L_NW), conv3lg_lds_bytes<16>(), st, p);
    return check_launch("tcx_conv2d_h2(halo 3lg16)");
}

// conv3m.hip: the h2-source form on v_mfma_f32_16x16x32_f16
bool conv3m_takes(const ConvParams& p);
int launch_conv3m(const ConvParams& p, hipStream_t st);

int launch_conv3l(const ConvParams& p, hipStream_t st) {
    if (conv3m_takes(p)) return launch_conv3m(p, st);
    if (p.W == 16) return launch3lg16<0>(p, st);
    return p.W == 64 ? launch3l<64>(p, st) : launch3l<32>(p, st);
}

}  // namespace tcx
