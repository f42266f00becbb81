// k_conv3lb: the bf16 single-product 3x3 stride-1 circular conv of config 5 (256^2 images: rows of
// 256 / 128 / 64 pixels; /root/reference/src/toycrystals/models/sde_score_model.py:102,105,218,222)
// with ALL staging by LDS-DMA and split wave roles — k_conv3lg's structure (conv3l.hip) for the
// bf16 records, which k_conv3g (conv3g.hpp) served with register-staged halos and B fragments
// loaded from L2 by every wave.
//
// What k_conv3g's bf16 form measured at 256^2 (profiles/r03_o_cfg5_bf16_layers.txt): 0.22-0.35 of the
// 2.5 PFLOP/s bf16 peak.  A bf16 tap is 6 MFMAs per wave (one per product instead of f16x3's three),
// so the per-tap staging that k_conv3g hides behind 18 MFMAs at f16x3 (each wave pulls its own 3 KB
// of B per tap through the vector-memory return path, the halo through VGPRs with its stores) is
// exposed three times as much.
//
// Layout: a bf16 product reads only the hi halves of the records (h2.hpp: [C/8][8 hi][8 lo]), so a
// halo slot is the two 16-B hi pieces of its pixel's 16-channel chunk: 32 B, no pad.  The pieces are
// XOR-swizzled by (col >> 3) & 1: a ds_read_b128 16-lane group ({0-3,12-15,20-27}, {4-11,16-19,28-31}
// and the same + 32: MI355X_MICROARCH.md LDS table) reads 32-B slots of consecutive pixels, whose
// banks (a / 16 mod 16 = 2 slot + piece) collide only for lanes 8 or 24 apart with equal pieces —
// exactly the lanes whose columns differ in bit 3.  Row block 1 (32 pixels on) and the dy offsets keep
// the column's swizzle, so they are immediates.  The halo of a 256-px row (3 x 258 slots) is 24.8 KB:
// double-buffered plus the B ring, 63.5 KB — two workgroups per CU at every row width.
// B ring: a tap pair's hi fragments (2 taps x 3 n x 1 KB = 6 KB, from the fragment-ordered copy of
// tcx_pack_conv_weight_h2_frag, whose lo KBs a bf16 weight leaves unused) in two slots.
//
// Schedule (as k_conv3lg PRO 0): waves 0-1 DMA the weight pairs (pair k issued at the start of tap
// 2k-3, waited for at the end of 2k-2), waves 2-3 the halo of chunk j+1 over taps 0-3 of chunk j
// (waited for at tap 6 / 7); one raw barrier per two taps, preceded by lgkmcnt(0) (the wave's LDS
// reads of the slot being refilled are done) and, for the DMA waves, vmcnt(0).
#include "conv_common.hpp"

#include <cstdlib>
#include <type_traits>

namespace tcx {
namespace {

constexpr int B_KC = 16;                  // input channels per chunk
constexpr int B_NT = 3;                   // 32-channel accumulator tiles per wave
constexpr int B_NW = 4;                   // waves (256-pixel tiles)
constexpr int B_TP = 64 * B_NW;
constexpr int B_PAIR = 2 * B_NT * 1024;   // hi fragments of a tap pair (6 KB)

__host__ __device__ constexpr int b_npx(int W) { return (B_TP / W + 2) * (W + 2); }
__host__ __device__ constexpr int b_ni(int W) { return (b_npx(W) + 31) / 32; }  // 1-KB DMA pieces per chunk
constexpr size_t conv3lb_lds_bytes(int W, int NR = 2) { return (size_t)2 * b_ni(W) * 1024 + NR * (size_t)B_PAIR; }

__device__ __forceinline__ void lds_dma16b(__amdgpu_buffer_rsrc_t r, char* lds, int voff, int soff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, voff, soff, 0, 0);
}
constexpr int WAIT_VM0_B = 0x0F70;    // s_waitcnt vmcnt(0)
constexpr int WAIT_VM3_B = 0x0F73;    // s_waitcnt vmcnt(3): all but the last pair's 3 DMAs
constexpr int WAIT_LGKM0_B = 0xC07F;  // s_waitcnt lgkmcnt(0)

// NR (round 6): weight-ring slots.  NR = 2: pair k is DMA'd at the start of odd tap 2k - 3 and waited for at
// the barrier ending tap 2k - 2 — ONE tap pair (12 bf16 MFMAs per wave, ~0.3 us) to cover an L2 round trip,
// which the weight waves then stall on while the other waves wait at the barrier (PMC r06_a: MFMA busy 43 %,
// 0.26 of peak at 256-px rows).  NR = 3: pair k is issued at tap 2k - 5 into slot k % 3 (the slot of pair
// k - 3, whose last B reads were during tap 2k - 6) and each barrier waits with vmcnt(3) (every pair but the
// one issued last), so a pair has two tap pairs of cover.  Same arithmetic and order: bit-identical output.
template <int W, int NR>
__global__ __launch_bounds__(64 * B_NW, 2) void k_conv3lb(ConvParams p) {
    constexpr int RT = 2, NT = B_NT, NTHR = 64 * B_NW;
    constexpr int W2 = W + 2;
    constexpr int NPX = b_npx(W);
    constexpr int NI = b_ni(W);
    constexpr int NIH = (NI + 1) / 2;  // per halo wave (wave 2: even i, wave 3: odd i)
    constexpr int HB = NI * 1024;
    constexpr int RING = 2 * HB;
    constexpr int RT1 = 32 * 32;       // row block 1: 32 slots on, same row (W >= 64)
    static_assert(W == 64 || W == 128 || W == 256, "k_conv3lb: rows of 64, 128 or 256 pixels");
    auto sw = [](int col) { return (col >> 3) & 1; };
    extern __shared__ __attribute__((aligned(16))) float sm[];
    char* const smc = reinterpret_cast<char*>(sm);
    // LDS-DMA destinations from a base the optimiser cannot fold to a constant (conv3l.hip)
    int lz;
    asm volatile("s_mov_b32 %0, 0" : "=s"(lz));
    char* const smd = smc + lz;

    const int tid = threadIdx.x;
    const int lane = tid & 63, li = lane & 31, lh = lane >> 5;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int tile = xcd_remap(blockIdx.x, gridDim.x);
    const int mblk = tile / p.n_nblk;
    const int nblk = tile - mblk * p.n_nblk;
    const int m0 = mblk * B_TP, n0 = nblk * 32 * NT;
    const int b = m0 / p.HoWo;
    const int r0 = (m0 - b * p.HoWo) / W;
    const int bs = p.bmod > 0 ? b % p.bmod : b;
    const int H = p.H;
    const int cpt = p.Cin / B_KC;  // even (Cin % 32 == 0)
    const int nch = 9 * cpt;
    const int npair = nch / 2;

    const __amdgpu_buffer_rsrc_t r1 = mk_rsrc(p.x1, p.bytes1);
    const __amdgpu_buffer_rsrc_t r2 = mk_rsrc(p.x2 ? p.x2 : p.x1, p.x2 ? p.bytes2 : p.bytes1);
    const __amdgpu_buffer_rsrc_t rw = mk_rsrc(reinterpret_cast<const float*>(p.wf), p.bytesw);

    // halo waves: instruction i fills slots 32 i .. 32 i + 31; lane l -> slot 32 i + l / 2, physical
    // piece l & 1, which holds logical piece (l & 1) ^ sw(col) = the hi 16 B of 8-channel group g at
    // byte 32 g of the chunk's record
    const int hw = wv & 1;
    // b2 sources (p.bf == 2, h2.hpp): the 2-byte bf16 rows hold exactly the hi pieces, so every byte
    // offset (pixel stride, piece, chunk) is half the record's
    const int esz = p.bf == 2 ? 2 : 4;
    const int rowb = p.C1 * esz;
    const int img0 = bs * H;
    const int ls = lane >> 1;
    // chunk-major source 2 (p.cm2, config 5's concat convs, round 6): b2 planes [C2/8][pixels][16 B]
    // (gn_apply_b2cm); a 16-channel chunk is two planes, so the slot's piece selects the plane
    const int plane2 = p.cm2 ? (int)(p.bytes2 / (unsigned)(p.C2 / 8)) : 0;
    // rb: bytes per pixel (row stride of a plane or of the pixel-major row); ph: bytes between the chunk's
    // two 8-channel pieces
    auto halo_voff = [&](int i, int rb, int ph) {
        const int hr0 = (32 * i) / W2;           // compile-time after unrolling
        const int th = W2 * (hr0 + 1) - 32 * i;  // lanes with ls >= th are in row hr0 + 1
        const int y0 = wrap_idx(r0 + hr0 - 1, H), y1 = wrap_idx(r0 + hr0, H);
        const int yo0 = (img0 + y0) * W * rb, yo1 = (img0 + y1) * W * rb;
        const bool nx = ls >= th;
        int hc = 32 * i - hr0 * W2 + ls - (nx ? W2 : 0);
        const int sl = 32 * i + ls;
        const int hcs = hc;
        if (sl >= NPX) hc = (NPX - 1) % W2;  // padding slots read a valid pixel
        const int x = hc == 0 ? W - 1 : (hc == W + 1 ? 0 : hc - 1);
        const int yo = (sl >= NPX) ? (img0 + wrap_idx(r0 + (NPX - 1) / W2 - 1, H)) * W * rb : (nx ? yo1 : yo0);
        return yo + x * rb + ph * ((lane & 1) ^ sw(hcs));
    };
    auto halo_issue = [&](int j, int buf, int q0, int q1) {
        const int ci0 = j * B_KC;
        const bool s1 = ci0 < p.C1;
        const bool cm = !s1 && p.cm2;
        const int cc = cm ? ((ci0 - p.C1) / 8) * plane2 : (s1 ? ci0 : ci0 - p.C1) * esz;
        const int rb = cm ? 16 : rowb, ph = cm ? plane2 : 8 * esz;
        const __amdgpu_buffer_rsrc_t rs = s1 ? r1 : r2;
#pragma unroll
        for (int q = 0; q < NIH; ++q) {
            if (q < q0 || q >= q1) continue;
            const int i = 2 * q + hw;
            if (i < NI) lds_dma16b(rs, smd + buf * HB + i * 1024, halo_voff(i, rb, ph), cc);
        }
    };
    // weight waves: pair k -> ring slot k & 1 as [tap][n][lane][16 B]; wave w moves pieces 3w .. 3w+2
    // (the hi KB of fragment (2k + tap, n) lies at ((nblk nch + 2k + tap) NT + n) 2048)
    auto pair_issue = [&](int k) {
        const int slot = NR == 2 ? (k & 1) : k % 3;  // the slot of pair k (also when clamped below)
        k = k < npair ? k : npair - 1;
        const int base = (nblk * nch + 2 * k) * NT * 2048;
        char* const d = smd + RING + slot * B_PAIR;
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            const int idx = 3 * wv + q;  // = tap * NT + n
            lds_dma16b(rw, d + idx * 1024, lane * 16, base + idx * 2048);
        }
    };

    int xa[3];
    {
        const int mloc = (wv * RT) * 32 + li;
        const int rr = mloc / W, cc = mloc % W;
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) xa[dx] = (rr * W2 + cc + dx) * 32 + 16 * (lh ^ sw(cc + dx));
    }
    f32x16 acc[RT][NT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int n = 0; n < NT; ++n) acc[rt][n] = (f32x16){};
    bf8 a[RT], bb[2][NT];
    auto rd_a = [&](int rt, int t, int hb) {
        const int dy = t / 3, dx = t - 3 * (t / 3);
        const int off = hb * HB + rt * RT1 + dy * W2 * 32;
        a[rt] = __builtin_bit_cast(bf8, *reinterpret_cast<const float4*>(smc + xa[dx] + off));
    };
    const int bl = lane * 16;
    auto rd_b = [&](int s, int c) {
        const char* B = smc + RING + (NR == 2 ? ((c >> 1) & 1) : (c >> 1) % 3) * B_PAIR + (c & 1) * (B_PAIR / 2) + bl;
#pragma unroll
        for (int n = 0; n < NT; ++n) bb[s][n] = __builtin_bit_cast(bf8, *reinterpret_cast<const float4*>(B + n * 1024));
    };
    auto mf = [&](int rt, int s) {
#pragma unroll
        for (int n = 0; n < NT; ++n)
            acc[rt][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[rt], bb[s][n], acc[rt][n], 0, 0, 0);
    };
    auto barrier = [&]() {
        __builtin_amdgcn_s_waitcnt(WAIT_LGKM0_B);
        __builtin_amdgcn_s_barrier();
    };

    // ---- prologue: pairs 0, 1 and halo 0 in LDS
    if (wv < 2) {
        pair_issue(0);
        pair_issue(1);
        if constexpr (NR == 3) pair_issue(2);
    } else {
        halo_issue(0, 0, 0, NIH);
    }
    __builtin_amdgcn_s_waitcnt(WAIT_VM0_B);
    barrier();
    rd_b(0, 0);
    rd_a(0, 0, 0);

    auto iter = [&](int j, auto T, auto S, auto HBc) {
        constexpr int t = decltype(T)::value;
        constexpr int s = decltype(S)::value;
        constexpr int hb = decltype(HBc)::value;
        const int c = 9 * j + t;
        const bool more = j + 1 < cpt;
        if (wv < 2) {
            if constexpr (s == 1) pair_issue((c + (NR == 2 ? 3 : 5)) >> 1);
        } else if constexpr (t < 4) {
            constexpr int q0 = (NIH * t) / 4, q1 = (NIH * (t + 1)) / 4;
            if (more) halo_issue(j + 1, hb ^ 1, q0, q1);
        }
        __builtin_amdgcn_sched_barrier(0);
        rd_b(s ^ 1, c + 1);
        if (t != 8) rd_a(1, t, hb);
        __builtin_amdgcn_sched_barrier(0);
        mf(0, s);
        __builtin_amdgcn_sched_barrier(0);
        if (t == 8) rd_a(0, 0, hb ^ 1);
        else rd_a(0, t + 1, hb);
        __builtin_amdgcn_sched_barrier(0);
        mf(1, s);
        __builtin_amdgcn_sched_barrier(0);
        if (t == 7) rd_a(1, 8, hb);
        if constexpr (s == 0) {  // even tap: publishes pair c/2 + 1 and (tap 6 / 7) halo j + 1
            constexpr bool halo_wait = t == (hb ? 7 : 6);
            if (wv < 2) __builtin_amdgcn_s_waitcnt(NR == 2 ? WAIT_VM0_B : WAIT_VM3_B);
            else if (halo_wait) __builtin_amdgcn_s_waitcnt(WAIT_VM0_B);
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

    __builtin_amdgcn_s_waitcnt(WAIT_VM0_B);  // the clamped tail pairs land before LDS is reused
    __syncthreads();
    double* red = reinterpret_cast<double*>(sm);
    conv_epi_store_rt<NT, 2, RT * B_NW, RT>(p, acc, m0, n0, RT * wv, lane, red);
    if (p.gn) {
        __syncthreads();
        conv_epi_gn<NT, RT * B_NW>(p, m0, n0, tid, NTHR, red);
    }
}

// TCX_LB_RING=2: the two-slot weight ring (A/B); default three slots
int lb_ring() {
    static const int r = [] {
        const char* e = getenv("TCX_LB_RING");
        return (e && e[0] == '2') ? 2 : 3;
    }();
    return r;
}

template <int W>
int launch3lb(const ConvParams& p, hipStream_t st) {
    static bool attr[2] = {};
    const int nr = lb_ring();
    void (*const k)(ConvParams) = nr == 2 ? &k_conv3lb<W, 2> : &k_conv3lb<W, 3>;
    const size_t shm = conv3lb_lds_bytes(W, nr);
    static_assert(conv3lb_lds_bytes(W, 3) <= 80 * 1024, "two workgroups per CU");
    if (!attr[nr - 2]) {
        if (hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm) !=
            hipSuccess) {
            set_error("tcx_conv2d_h2: cannot enable %zu B of dynamic LDS", shm);
            return TCX_EHIP;
        }
        attr[nr - 2] = true;
    }
    const int grid = (p.M / B_TP) * p.n_nblk;
    hipLaunchKernelGGL(k, dim3(grid), dim3(64 * B_NW), shm, st, p);
    return check_launch("tcx_conv2d_h2(halo 3lb)");
}

}  // namespace

// TCX_CONV3LB=0 keeps k_conv3g for the bf16 rows (A/B measurements)
bool conv3lb_takes(const ConvParams& p) {
    static const bool on = [] {
        const char* e = getenv("TCX_CONV3LB");
        return !(e && e[0] == '0');
    }();
    if (!on || !p.bf || !p.circular || !(p.W == 64 || p.W == 128 || p.W == 256)) return false;
    if (p.M % B_TP != 0 || p.HoWo % B_TP != 0 || p.Cin % 32 != 0) return false;
    if (p.cm1 || (p.cm2 && (p.bf != 2 || p.C2 % 16 != 0))) return false;  // chunk-major: b2 source 2 only
    return p.sc1 == nullptr && !(p.C2 > 0 && p.sc2 != nullptr);  // h2 / bf16 record sources only
}

int launch_conv3lb(const ConvParams& p, hipStream_t st) {
    if (p.W == 256) return launch3lb<256>(p, st);
    if (p.W == 128) return launch3lb<128>(p, st);
    return launch3lb<64>(p, st);
}

}  // namespace tcx
