// k_conv3g: the 3x3 stride-1 circular conv of the U-Net rows W >= 32 (every _ConvBlock conv and
// us*_conv at 64^2 / 32^2, and the 128^2 / 256^2 rows of config 5: /root/reference/src/toycrystals/
// models/sde_score_model.py:102,105,218,222) on the f16x3 split path, with the preceding
// GroupNorm + SiLU (:103-107) applied while the input halo is staged.
//
// Why a new tiling (k_conv3p, conv3h.hip, stays for 16^2): k_conv3p's 128-pixel x 96-channel tile
// re-reads the whole weight chunk from LDS per wave per 32 pixels, and stages the 12 KB weight chunk
// of every tap with ds_write_b128 for only 128 pixels: its LDS traffic is ~0.8 of the MFMA time
// (PMC r01_bh: MFMA busy 48 % at 64^2).  Here 8 waves each own 64 pixels (two
// 32-row blocks) x 96 channels (a 512-pixel tile = whole rows), so every B fragment read from LDS
// feeds two MFMAs, and the input-channel chunk is 16 deep: per tap the weight chunk is 6 KB for 512
// pixels (1/8 of k_conv3p's staging per FLOP) and each wave issues 18 MFMAs per 10 ds_read_b128
// (k_conv3p: 9 per 8).  Two waves per SIMD, one 512-thread workgroup per CU.
//
// LDS: two halo buffers [(TR+2)*(W+2)][20 floats] (16 channels h2 = 64 B per pixel + 16 B pad: the
// 80-B pixel stride makes the ds_read_b128 of 32 consecutive pixels conflict free for every tap
// offset), weights [2][96][20 floats], GroupNorm tables [2][Cin] of the tile's image: 124 KB at
// W = 64, 143 KB at W = 128 (W = 256 would not fit: those rows stay on the im2col kernel).
//
// Prologue: a source may be h2 (copied) or fp32 + a per-(image, channel) GroupNorm scale/shift table
// (tcx_gn_finalize): x -> silu(x*sc + sh) is computed per 8-channel unit two taps after its load and
// split to h2 in registers right before the unit is stored.  The normalised tensor is
// never written to HBM (the k_gn_apply_tab_h2 pass it replaces read and wrote every element).
// SiLU here is x * rcp(1 + exp2(-x log2 e)) (v_exp_f32 / v_rcp_f32, ~2 ulp of fp32): the value is
// rounded to the 22-bit h2 split right after, so the difference to expf/IEEE division is below the
// split's own rounding (h2.hpp).
//
// Pipeline per tap t of chunk j (c = 9j + t; B set S = c & 1 in registers, A0 = tap t's row block 0;
// halo j in buffer j & 1, halo j+1 filled into the other buffer during taps 0..UPT+1):
//   read A1(t) | 9 MFMAs (row block 0) | read A0(t+1), B(t+1) into set S^1 | 9 MFMAs (row block 1) |
//   [t < UPT: load halo unit t of j+1]  [2 <= t < UPT+2: GN+SiLU+split and store unit t-2]
//   store weights c+2 | barrier | load weights c+4
// The weights of chunk c+2 go into LDS buffer c & 1, whose data (chunk c) every wave read into
// registers before the previous barrier; halo buffer (j+1) & 1 was last read (taps 8 of chunk j-1)
// before the last barrier of chunk j-1, and is complete before the barrier of tap 5 (UPT <= 4),
// ahead of its first read (A0 of tap 0 of chunk j+1, read during tap 8).
#include "conv_common.hpp"

#include <type_traits>

namespace tcx {
namespace {

constexpr int G_PXF = 20;   // floats per staged pixel / weight row: 16 channels h2 (64 B) + 16 B pad
constexpr int G_KC = 16;    // input channels per chunk
constexpr int G_TP = 512;   // output pixels per tile
constexpr int G_NT = 3;     // 32-channel accumulator tiles per wave (96 output channels)

__host__ __device__ constexpr int g_npx(int W) { return (G_TP / W + 2) * (W + 2); }
__host__ __device__ constexpr int g_units(int W) { return (2 * g_npx(W) + 511) / 512; }  // 8-ch units per thread

constexpr size_t conv3g_lds_bytes(int W, int Cin) {
    return ((size_t)2 * g_npx(W) * G_PXF + 2 * 96 * G_PXF + 2 * (size_t)Cin) * sizeof(float);
}

__device__ __forceinline__ float silu_split_src(float v, float sc, float sh) {
    const float y = fmaf(v, sc, sh);
    return y * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-1.4426950408889634f * y));
}

// 8 fp32 values -> h2 unit: hi halves (16 B) and lo halves (16 B)
__device__ __forceinline__ void split8(const float (&v)[8], float4& hi, float4& lo, bool& bad) {
    unsigned h[4], l[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const unsigned a = split1(v[2 * k]), b = split1(v[2 * k + 1]);
        h[k] = (a & 0xffffu) | (b << 16);
        l[k] = (a >> 16) | (b & 0xffff0000u);
        bad = bad || h2_bad(v[2 * k]) || h2_bad(v[2 * k + 1]);
    }
    hi = make_float4(__uint_as_float(h[0]), __uint_as_float(h[1]), __uint_as_float(h[2]), __uint_as_float(h[3]));
    lo = make_float4(__uint_as_float(l[0]), __uint_as_float(l[1]), __uint_as_float(l[2]), __uint_as_float(l[3]));
}

template <int W, bool CIRC>
__global__ __launch_bounds__(512, 2) void k_conv3g(ConvParams p) {
    constexpr int NW = 8, RT = 2, NT = G_NT, BN = 32 * NT, NTHR = 512;
    constexpr int W2 = W + 2;
    constexpr int NPX = g_npx(W);
    constexpr int NU = 2 * NPX;        // 8-channel halo units per chunk
    constexpr int UPT = g_units(W);
    constexpr int HBUF = NPX * G_PXF;
    constexpr int WBUF = BN * G_PXF;
    constexpr int WPC = BN * 4;        // 16-B weight pieces per chunk (384)
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float* const Hs = sm;                   // [2][NPX][PXF]
    float* const Bs = sm + 2 * HBUF;        // [2][BN][PXF]
    float* const Ts = Bs + 2 * WBUF;        // [2][Cin]: scale, shift of this tile's image

    const int tid = threadIdx.x;
    const int lane = tid & 63, wv = tid >> 6, li = lane & 31, lh = lane >> 5;
    const int tile = xcd_remap(blockIdx.x, gridDim.x);
    const int mblk = tile / p.n_nblk;
    const int nblk = tile - mblk * p.n_nblk;
    const int m0 = mblk * G_TP, n0 = nblk * BN;
    const int b = m0 / p.HoWo;
    const int r0 = (m0 - b * p.HoWo) / W;
    const int bs = p.bmod > 0 ? b % p.bmod : b;
    const int H = p.H;
    const int Cin = p.Cin;
    const int cpt = Cin / G_KC;        // chunks (even: Cin % 32 == 0)
    const int nch = 9 * cpt;
    const bool gn1 = p.sc1 != nullptr, gn2 = p.sc2 != nullptr;

    const __amdgpu_buffer_rsrc_t r1 = mk_rsrc(p.x1, p.bytes1);
    const __amdgpu_buffer_rsrc_t r2 = mk_rsrc(p.x2 ? p.x2 : p.x1, p.x2 ? p.bytes2 : p.bytes1);
    const __amdgpu_buffer_rsrc_t rw = mk_rsrc(p.w, p.bytesw);

    // ---- GroupNorm tables of this tile's image (concatenated channel order)
    if (gn1 || gn2) {
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

    // ---- halo plan: unit u = tid + 512 i -> halo pixel u >> 1, 8-channel group u & 1
    const int rowb = p.C1 * 4;  // bytes per source pixel (C2 == C1 when there are two sources)
    int hoff[UPT];              // source byte offset of the unit (kOOB: zero padding)
#pragma unroll
    for (int i = 0; i < UPT; ++i) {
        const int u = tid + NTHR * i;
        const int hp = u >> 1;
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
            hoff[i] = ok ? ((bs * H + y) * W + x) * rowb + (u & 1) * 32 : kOOB;
        }
    }
    static_assert(UPT <= 4, "halo units per thread: stores must finish by tap 5");
    float4 hv[UPT][2];  // unit i of the next halo (loaded at tap i, stored at tap i+2)
    auto src_of = [&](int j, __amdgpu_buffer_rsrc_t& rs, int& cc) {
        const int ci0 = j * G_KC;
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
    // fp32 source with a GroupNorm table: silu(x*sc+sh) -> h2 (zero padding stays 0); then LDS
    auto unit_store = [&](int j, int i, int buf) {
        const int u = tid + NTHR * i;
        if (!((i + 1) * NTHR <= NU || u < NU)) return;
        __amdgpu_buffer_rsrc_t rs;
        int cc;
        if (src_of(j, rs, cc)) {
            const int c = j * G_KC + (u & 1) * 8;
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
            split8(v, hv[i][0], hv[i][1], bad);
            h2_flag(p.ovf, bad);
        }
        float* d = &Hs[buf * HBUF + (u >> 1) * G_PXF + (u & 1) * 8];
        *reinterpret_cast<float4*>(d) = hv[i][0];
        *reinterpret_cast<float4*>(d + 4) = hv[i][1];
    };
    // ---- weight chunk c = 9 j + t: rows n0..n0+95, packed k = t*Cin + 16 j (4 pieces of 16 B)
    const bool wthr = tid < WPC;
    const int woff = ((n0 + (tid >> 2)) * p.kpad) * 4 + (tid & 3) * 16;
    const int wdst = (tid >> 2) * G_PXF + (tid & 3) * 4;
    float4 wr[2];
    auto w_load = [&](int c, float4& r) {
        const int j = c / 9, t = c - 9 * j;
        if (wthr) r = bld4(rw, woff, (t * Cin + j * G_KC) * 4);
    };
    auto w_store = [&](int buf, const float4& r) {
        if (wthr) *reinterpret_cast<float4*>(&Bs[buf * WBUF + wdst]) = r;
    };

    // ---- fragments
    int abase[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
        const int mloc = (wv * RT + rt) * 32 + li;
        abase[rt] = ((mloc / W) * W2 + (mloc % W)) * G_PXF + lh * 8;
    }
    const int bbase = li * G_PXF + lh * 8;
    f32x16 acc[RT][NT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int n = 0; n < NT; ++n) acc[rt][n] = (f32x16){};
    h8 a_h[RT], a_l[RT], b_h[2][NT], b_l[2][NT];
    auto rd_a = [&](int rt, int t, int hb) {
        const int dy = t / 3, dx = t - 3 * (t / 3);
        const float* A = &Hs[hb * HBUF + abase[rt] + (dy * W2 + dx) * G_PXF];
        a_h[rt] = __builtin_bit_cast(h8, ld4(A));
        a_l[rt] = __builtin_bit_cast(h8, ld4(A + 4));
    };
    auto rd_b = [&](int s, int buf) {
        const float* B = &Bs[buf * WBUF + bbase];
#pragma unroll
        for (int n = 0; n < NT; ++n) {
            b_h[s][n] = __builtin_bit_cast(h8, ld4(B + n * 32 * G_PXF));
            b_l[s][n] = __builtin_bit_cast(h8, ld4(B + n * 32 * G_PXF + 4));
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

    // ---- prologue: tables, halo 0 and weight chunks 0 and 1 in LDS; chunks 2, 3 in flight
    if (gn1 || gn2) __syncthreads();  // Ts before the first transform
#pragma unroll
    for (int i = 0; i < UPT; ++i) unit_load(0, i);
    w_load(0, wr[0]);
    w_load(1, wr[1]);
#pragma unroll
    for (int i = 0; i < UPT; ++i) unit_store(0, i, 0);
    w_store(0, wr[0]);
    w_store(1, wr[1]);
    w_load(2, wr[0]);
    w_load(3, wr[1]);
    __syncthreads();
    rd_a(0, 0, 0);
    rd_b(0, 0);

    // one tap: T compile-time tap index, S the register set of B(c) (c & 1), HB halo buffer of chunk j
    auto iter = [&](int j, auto T, auto S, auto HBc) {
        constexpr int t = decltype(T)::value;
        constexpr int s = decltype(S)::value;
        constexpr int hb = decltype(HBc)::value;
        const int c = 9 * j + t;
        const bool more = j + 1 < cpt;
        if (t != 8) rd_a(1, t, hb);  // A1(8) was read at the end of tap 7
        __builtin_amdgcn_sched_barrier(0);
        mf(0, s);
        __builtin_amdgcn_sched_barrier(0);
        if (c + 1 < nch) {
            if (t == 8) rd_a(0, 0, hb ^ 1);
            else rd_a(0, t + 1, hb);
            rd_b(s ^ 1, (c + 1) & 1);
        }
        __builtin_amdgcn_sched_barrier(0);
        mf(1, s);
        __builtin_amdgcn_sched_barrier(0);
        if (t == 7) rd_a(1, 8, hb);
        if constexpr (t < UPT) {
            if (more) unit_load(j + 1, t);
        }
        if constexpr (t >= 2 && t < UPT + 2) {
            if (more) unit_store(j + 1, t - 2, hb ^ 1);
        }
        if (c + 2 < nch) w_store(c & 1, wr[s]);
        __syncthreads();
        if (c + 4 < nch) w_load(c + 4, wr[s]);
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
    conv_epi_store<NT, true, RT * NW>(p, acc[0], m0, n0, RT * wv, lane, red);
    conv_epi_store<NT, true, RT * NW>(p, acc[1], m0, n0, RT * wv + 1, lane, red);
    if (p.gn) {
        __syncthreads();
        conv_epi_gn<NT, RT * NW>(p, m0, n0, tid, NTHR, red);
    }
}

template <int W>
int launch3g(const ConvParams& p, hipStream_t st) {
    const size_t shm = conv3g_lds_bytes(W, p.Cin);
    static bool attr[2] = {false, false};
    auto kc = p.circular ? &k_conv3g<W, true> : &k_conv3g<W, false>;
    if (!attr[p.circular ? 1 : 0]) {
        if (hipFuncSetAttribute(reinterpret_cast<const void*>(kc), hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)conv3g_lds_bytes(W, 512)) != hipSuccess) {
            set_error("tcx_conv2d_h2: cannot enable %zu B of dynamic LDS", conv3g_lds_bytes(W, 512));
            return TCX_EHIP;
        }
        attr[p.circular ? 1 : 0] = true;
    }
    const int grid = (p.M / G_TP) * p.n_nblk;
    hipLaunchKernelGGL(kc, dim3(grid), dim3(512), shm, st, p);
    return check_launch("tcx_conv2d_h2(halo 512)");
}

}  // namespace

// TCX_CONV3G=0 keeps k_conv3p on every row width (A/B measurements; no GroupNorm prologue then)
bool conv3g_enabled() {
    static const bool on = [] {
        const char* e = getenv("TCX_CONV3G");
        return !(e && e[0] == '0');
    }();
    return on;
}

bool conv3g_covers(int H, int W, int Cin, int cout_pad) {
    return conv3g_enabled() && (W == 32 || W == 64 || W == 128) && H % (G_TP / W) == 0 && (H * W) % G_TP == 0 &&
           Cin % 32 == 0 && Cin <= 512 && cout_pad % 96 == 0;
}

bool conv3g_applies(const ConvParams& p, int cout_pad) {
    if (!conv3g_enabled()) return false;
    const bool wok = p.W == 32 || p.W == 64 || p.W == 128;
    return wok && p.ks == 3 && p.stride == 1 && p.pad_y == 1 && p.pad_x == 1 && p.Hi == p.H && p.Wi == p.W &&
           p.H % (G_TP / p.W) == 0 && p.HoWo % G_TP == 0 && cout_pad % 96 == 0 && p.Cin % 32 == 0 &&
           p.Cin <= 512 && p.C1 % G_KC == 0 && (p.C2 == 0 || p.C2 == p.C1) && p.kpad == 9 * p.Cin && p.osy == 1 &&
           p.osx == 1;
}

int launch_conv3g(ConvParams& p, int cout_pad, hipStream_t st) {
    p.n_nblk = cout_pad / 96;
    if (p.M == 0) return TCX_OK;
    prof_begin(st);
    int rc;
    if (p.W == 64) rc = launch3g<64>(p, st);
    else if (p.W == 32) rc = launch3g<32>(p, st);
    else rc = launch3g<128>(p, st);
    prof_end(st, 2.0 * (double)p.M * p.Cout * 9 * p.Cin);
    return rc;
}

}  // namespace tcx
