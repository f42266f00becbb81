// k_conv3mb: config 5's bf16 3x3 stride-1 circular conv (256^2 images, rows of 256 / 128 / 64 pixels;
// /root/reference/src/toycrystals/models/sde_score_model.py:102,105,218,222) on v_mfma_f32_16x16x32_bf16
// TAP PAIRS — k_conv3m's unit of work (conv3m.hip) for the 2-byte bf16 ("b2") tensors, replacing
// k_conv3lb's 32x32x16 taps.
//
// Why: at equal FLOPs and LDS bytes per FLOP the 16x16x32 loop runs 1.12-1.15x the 32x32x16 one on this
// chip (MI355X_MICROARCH.md: the smaller MFMA holds a higher clock under load; the f16 probe
// profiles/r04_b_mfma_shape.log), and a 32-deep k step = a pair of taps halves the barrier-separated steps.
// A bf16 product is ONE MFMA (hi x hi, fp32 accumulation), so a pair carries a third of k_conv3m's
// MFMAs per staged byte: the weight ring has THREE slots (two pairs of latency cover for the L2 round
// trip of a weight pair instead of one) and each pair's A and B fragments are read into a second
// register set at the start of the previous pair (a whole pair of cover for the LDS reads).
//
// Tile: 256 pixels x 96 output channels, 4 waves x 64 pixels (one run of a row: W >= 64), each wave
// 4 row blocks (16 px) x 6 column blocks (16 channels) of 16x16 accumulators = 24 MFMAs per pair.
// A 32-deep k step is the tap pair (2 q, 2 q + 1) of the two-chunk period c = 9 j + t (q = 0..8, pair 4
// straddles the chunks): lane l holds pixel l & 15 of the row block, k = 8 (l >> 4) + e: channel group
// (l >> 4) & 1 of tap 2 q + (l >> 5) — one ds_read_b128 of a 32-B halo slot (the two 16-B 8-channel b2
// pieces of the pixel's 16-channel chunk, NOT swizzled: the ds_read_b128 lane groups {0-3,12-15,20-27}
// etc. then cover 16 distinct 16-B bank positions at every tap offset, since pixels 8 apart take
// different pieces).  B: the hi KBs of the fragment-ordered weights (tcx_pack_conv_weight_h2_frag,
// k_conv3lb's pair layout [tap][32-col n][lane][16 B]) gathered per lane as in k_conv3m.
//
// Schedule of pair k (k = 9 pp + q), all waves past the barrier that ended pair k - 1:
//   waves 0-1: DMA weight pair k + 3 into ring slot k % 3 (pair k's B was read during pair k - 1);
//   waves 2-3: at q = 4 the halo of chunk 2 pp + 2 into buffer 0 (last read by A(4), read in pair 3),
//              at q = 8 the halo of chunk 2 pp + 3 into buffer 1 (last read by A(8), read in pair 7);
//   every wave: A(k + 1) (4 reads) and B(k + 1) (6 reads) into the other register set, then the 24 MFMAs
//   of pair k; lgkmcnt(0); weight waves vmcnt(3) (pair k + 2 landed: every pair DMA but the last),
//   halo waves vmcnt(0) at q = 7 (chunk 2 pp + 2, first read in pair 8) and q = 2 (chunk 2 pp + 1, first
//   read in pair 3); barrier.
// Halo DMA (LDS-DMA, lane-linear): instruction i fills slots 32 i .. 32 i + 31, lane l slot 32 i + l / 2,
// piece l & 1; padding slots re-read a valid pixel.  Chunk-major source 2 (gn_apply_b2cm planes): the
// piece selects the plane.  Epilogue: k_conv3m's quad-transposed 16x16 epilogue with fp32 or b2 stores
// and the fp64 GroupNorm partials per 128-pixel group.
#include "conv_common.hpp"

#include <type_traits>
#include <utility>

namespace tcx {
namespace {

constexpr int MB_KC = 16;      // input channels per chunk
constexpr int MB_NW = 4;       // waves per workgroup
constexpr int MB_TP = 256;     // pixels per tile
constexpr int MB_PAIR = 6144;  // hi B fragments of a tap pair: 2 taps x 3 x 1 KB
constexpr int MB_NR = 3;       // weight ring slots
constexpr int MB_BN = 96;      // output channels per tile

__host__ __device__ constexpr int mb_npx(int W) { return (MB_TP / W + 2) * (W + 2); }
__host__ __device__ constexpr int mb_ni(int W) { return (mb_npx(W) + 31) / 32; }  // 1-KB DMA pieces per chunk
constexpr size_t conv3mb_lds_bytes(int W) { return (size_t)2 * mb_ni(W) * 1024 + MB_NR * (size_t)MB_PAIR; }

constexpr int MB_WAIT_VM0 = 0x0F70;    // s_waitcnt vmcnt(0)
constexpr int MB_WAIT_VM3 = 0x0F73;    // s_waitcnt vmcnt(3)
constexpr int MB_WAIT_LGKM0 = 0xC07F;  // s_waitcnt lgkmcnt(0)

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void mb_dma16(__amdgpu_buffer_rsrc_t r, char* lds, int voff, int soff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, voff, soff, 0, 0);
}
template <typename F, int... Is>
__device__ __forceinline__ void mb_static_for(F&& f, std::integer_sequence<int, Is...>) {
    (f(std::integral_constant<int, Is>{}), ...);
}

// OB2: the output is 2-byte bf16 (p.out_h2 with p.bf == 2: the pre-GroupNorm outputs config 5 stores as b2),
// else fp32
template <int W, bool OB2>
__global__ __launch_bounds__(64 * MB_NW, 2) void k_conv3mb(ConvParams p) {
    constexpr int W2 = W + 2;
    constexpr int NPX = mb_npx(W);
    constexpr int NI = mb_ni(W);
    constexpr int NIH = (NI + 1) / 2;  // per halo wave (wave 2: even i, wave 3: odd i)
    constexpr int HB = NI * 1024;
    constexpr int RING = 2 * HB;
    static_assert(W == 64 || W == 128 || W == 256, "k_conv3mb: rows of 64, 128 or 256 pixels");
    static_assert(NI * 32 >= NPX, "k_conv3mb: halo slots");
    extern __shared__ __attribute__((aligned(16))) float sm[];
    char* const smc = reinterpret_cast<char*>(sm);
    // LDS-DMA destinations from a base the optimiser cannot fold to a constant (k_conv3lg's note)
    int lz;
    asm volatile("s_mov_b32 %0, 0" : "=s"(lz));
    char* const smd = smc + lz;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int tile = xcd_remap(blockIdx.x, gridDim.x);
    const int mblk = tile / p.n_nblk;
    const int nblk = tile - mblk * p.n_nblk;
    const int m0 = mblk * MB_TP, n0 = nblk * MB_BN;
    const int b = m0 / p.HoWo;
    const int r0 = (m0 - b * p.HoWo) / W;
    const int bs = p.bmod > 0 ? b % p.bmod : b;
    const int H = p.H;
    const int cpt = p.Cin / MB_KC;  // even (Cin % 32 == 0)
    const int nch = 9 * cpt;
    const int npair = nch / 2;
    const int npp = cpt / 2;        // 9-pair periods

    const __amdgpu_buffer_rsrc_t r1 = mk_rsrc(p.x1, p.bytes1);
    const __amdgpu_buffer_rsrc_t r2 = mk_rsrc(p.x2 ? p.x2 : p.x1, p.x2 ? p.bytes2 : p.bytes1);
    const __amdgpu_buffer_rsrc_t rw = mk_rsrc(reinterpret_cast<const float*>(p.wf), p.bytesw);

    // ---- halo DMA (waves 2, 3)
    const int hw = wv & 1;
    const int rowb = p.C1 * 2;
    const int img0 = bs * H;
    const int plane2 = p.cm2 ? (int)(p.bytes2 / (unsigned)(p.C2 / 8)) : 0;
    // rb: bytes per pixel (b2 row, or 16 in a chunk-major plane); ph: bytes between the chunk's two pieces
    auto halo_voff = [&](int i, int rb, int ph) __attribute__((always_inline)) {
        // recomputed at every issue from an opaque copy of the lane index: hoisted out of the pair loop, the
        // offsets of all NI instructions spilled beside the two fragment sets (k_conv3m's note)
        int ls;
        asm volatile("v_mov_b32 %0, %1" : "=v"(ls) : "v"(lane >> 1));
        const int hr0 = (32 * i) / W2;           // compile time after unrolling
        const int th = W2 * (hr0 + 1) - 32 * i;  // lanes with ls >= th are in row hr0 + 1
        const int y0 = wrap_idx(r0 + hr0 - 1, H), y1 = wrap_idx(r0 + hr0, H);
        const int yo0 = (img0 + y0) * W * rb, yo1 = (img0 + y1) * W * rb;
        const bool nx = ls >= th;
        int hc = 32 * i - hr0 * W2 + ls - (nx ? W2 : 0);
        const int sl = 32 * i + ls;
        if (sl >= NPX) hc = (NPX - 1) % W2;  // padding slots read a valid pixel
        const int x = hc == 0 ? W - 1 : (hc == W + 1 ? 0 : hc - 1);
        const int yo = (sl >= NPX) ? (img0 + wrap_idx(r0 + (NPX - 1) / W2 - 1, H)) * W * rb : (nx ? yo1 : yo0);
        return yo + x * rb + ph * (lane & 1);
    };
    auto halo_all = [&](int j, int buf) __attribute__((always_inline)) {
        const int ci0 = j * MB_KC;
        const bool s1 = ci0 < p.C1;
        const bool cm = !s1 && p.cm2;
        const int cc = cm ? ((ci0 - p.C1) / 8) * plane2 : (s1 ? ci0 : ci0 - p.C1) * 2;
        const int rb = cm ? 16 : rowb, ph = cm ? plane2 : 16;
        const __amdgpu_buffer_rsrc_t rs = s1 ? r1 : r2;
#pragma unroll
        for (int q = 0; q < NIH; ++q) {
            const int i = 2 * q + hw;
            if (i < NI) mb_dma16(rs, smd + buf * HB + i * 1024, halo_voff(i, rb, ph), cc);
        }
    };
    // weight pair k -> ring slot k % 3; wave w (0, 1) moves the hi KBs idx = 3 w .. 3 w + 2 (= tap * 3 + n)
    // of fragments (2 k + tap, n); past the last pair the last one is re-read (uniform vmcnt accounting)
    auto pair_issue = [&](int k) __attribute__((always_inline)) {
        const int slot = k % MB_NR;
        k = k < npair ? k : npair - 1;
        const int base = (nblk * nch + 2 * k) * 3 * 2048;
        char* const d = smd + RING + slot * MB_PAIR;
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            const int idx = 3 * wv + q;
            mb_dma16(rw, d + idx * 1024, lane * 16, base + idx * 2048);
        }
    };

    // ---- A addresses of row block 0 per pair type q (taps 2 q + th of the 18-tap period)
    const int li = lane & 15, g = (lane >> 4) & 1, th = lane >> 5;
    int aq[9];
    {
        const int mloc = wv * 64 + li;
        const int rr = mloc / W, cc = mloc % W;
#pragma unroll
        for (int q = 0; q < 9; ++q) {
            const int c = 2 * q + th;
            const int hb = c >= 9 ? 1 : 0;
            const int t = c - 9 * hb;
            const int dy = t / 3, dx = t - 3 * (t / 3);
            aq[q] = hb * HB + ((rr + dy) * W2 + cc + dx) * 32 + 16 * g;
        }
    }
    // B: per-lane gather address inside a ring slot ([tap][32-col n][lane][16 B] hi KBs)
    const int bq = RING + th * 3072 + g * 512 + li * 16;

    f32x4 acc[4][6];
#pragma unroll
    for (int rb = 0; rb < 4; ++rb)
#pragma unroll
        for (int n = 0; n < 6; ++n) acc[rb][n] = (f32x4){};
    bf8 av[2][4], bv[2][6];
    auto rd = [&](auto SETc, int q, int k) __attribute__((always_inline)) {
        constexpr int st = decltype(SETc)::value;
#pragma unroll
        for (int rb = 0; rb < 4; ++rb)
            av[st][rb] = __builtin_bit_cast(bf8, *reinterpret_cast<const float4*>(smc + aq[q] + rb * 16 * 32));
        const char* B = smc + bq + (k % MB_NR) * MB_PAIR;
#pragma unroll
        for (int nb = 0; nb < 6; ++nb)
            bv[st][nb] = __builtin_bit_cast(bf8, *reinterpret_cast<const float4*>(B + (nb >> 1) * 1024 + (nb & 1) * 256));
    };
    auto mma = [&](auto SETc) __attribute__((always_inline)) {
        constexpr int st = decltype(SETc)::value;
#pragma unroll
        for (int nb = 0; nb < 6; ++nb)
#pragma unroll
            for (int rb = 0; rb < 4; ++rb)
                acc[rb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[st][rb], bv[st][nb], acc[rb][nb], 0, 0, 0);
    };

    // ---- prologue: pairs 0-2 and halo chunk 0 landed, chunk 1 issued, pair 0's fragments in set 0
    if (wv < 2) {
        pair_issue(0);
        pair_issue(1);
        pair_issue(2);
    } else {
        halo_all(0, 0);
    }
    __builtin_amdgcn_s_waitcnt(MB_WAIT_VM0);
    __builtin_amdgcn_s_waitcnt(MB_WAIT_LGKM0);
    __builtin_amdgcn_s_barrier();
    rd(std::integral_constant<int, 0>{}, 0, 0);
    // pair 0's B must be read by every wave before pair 0 re-fills its ring slot with pair 3
    __builtin_amdgcn_s_waitcnt(MB_WAIT_LGKM0);
    __builtin_amdgcn_s_barrier();
    if (wv >= 2 && cpt > 1) halo_all(1, 1);

    // pair q of period pp; S: the register set of the period's pair 0 (pair k uses set (k & 1))
    auto pair_iter = [&](int pp, auto Q, auto S) __attribute__((always_inline)) {
        constexpr int q = decltype(Q)::value;
        constexpr int qn = q == 8 ? 0 : q + 1;
        constexpr int set = decltype(S)::value ^ (q & 1);
        const int k = 9 * pp + q;
        if (wv < 2) {
            pair_issue(k + 3);
        } else {
            if constexpr (q == 4) {
                if (2 * pp + 2 < cpt) halo_all(2 * pp + 2, 0);
            } else if constexpr (q == 8) {
                if (2 * pp + 3 < cpt) halo_all(2 * pp + 3, 1);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        if (k + 1 < npair) rd(std::integral_constant<int, set ^ 1>{}, qn, k + 1);
        __builtin_amdgcn_sched_barrier(0);
        mma(std::integral_constant<int, set>{});
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_waitcnt(MB_WAIT_LGKM0);
        if (wv < 2) __builtin_amdgcn_s_waitcnt(MB_WAIT_VM3);
        else if (q == 7 || q == 2) __builtin_amdgcn_s_waitcnt(MB_WAIT_VM0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
    };
    auto period = [&](int pp, auto S) __attribute__((always_inline)) {
        mb_static_for([&](auto Q) { pair_iter(pp, Q, S); }, std::make_integer_sequence<int, 9>{});
    };
    using S0 = std::integral_constant<int, 0>;
    using S1 = std::integral_constant<int, 1>;
    int pp = 0;
    for (; pp + 1 < npp; pp += 2) {
        period(pp, S0{});
        period(pp + 1, S1{});
    }
    if (pp < npp) period(pp, S0{});

    __builtin_amdgcn_s_waitcnt(MB_WAIT_VM0);  // the clamped tail pairs land before LDS is reused
    __syncthreads();

    // ---- epilogue (k_conv3m's 16x16 form): lane l holds column l & 15 of each block, rows 4 (l >> 4) .. + 3;
    // bias, the fp64 GroupNorm partials per 128-pixel group from the columns, a 4x4 quad transpose so lane l
    // holds row 4 (l >> 4) + (l & 3), channels 4 ((l & 15) >> 2) .. + 3: one 16-B (fp32) or 8-B (b2) store
    double* red = reinterpret_cast<double*>(sm);
    {
        const int col = lane & 15, rg = lane >> 4, qi = lane & 3, qc = col >> 2;
        const float wsc = *p.wscale;
        const __amdgpu_buffer_rsrc_t ry = mk_rsrc(p.y, (unsigned)((long long)p.M * p.Cout * (OB2 ? 2 : 4)));
        const int pixq = m0 + 64 * wv + 4 * rg + qi;  // this lane's pixel after the transpose (row block 0)
        const int vo = (pixq * p.Cout + n0 + 4 * qc) * (OB2 ? 2 : 4);
        float bcs[6];
#pragma unroll
        for (int nb = 0; nb < 6; ++nb) bcs[nb] = p.bias ? p.bias[n0 + 16 * nb + col] : 0.f;
#pragma unroll
        for (int nb = 0; nb < 6; ++nb) {
            const float bc = bcs[nb];
            float s = 0.f, ss = 0.f;
#pragma unroll
            for (int rb = 0; rb < 4; ++rb) {
                float v[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float x = fmaf(acc[rb][nb][r], wsc, bc);
                    v[r] = x;
                    s += x;
                    ss = fmaf(x, x, ss);
                }
                quad_transpose4(v, qi);
                const int so = (16 * rb * p.Cout + 16 * nb) * (OB2 ? 2 : 4);
                if constexpr (OB2) {
                    __builtin_amdgcn_raw_buffer_store_b64((u32x2){pack2_bf(v[0], v[1]), pack2_bf(v[2], v[3])}, ry, vo, so,
                                                          0);
                } else {
                    store_b128_guarded(__builtin_bit_cast(u32x4, make_float4(v[0], v[1], v[2], v[3])), ry, vo, so);
                }
            }
            if (p.gn) {
                double ds = (double)s, dss = (double)ss;
                ds += __shfl_xor(ds, 16);
                dss += __shfl_xor(dss, 16);
                ds += __shfl_xor(ds, 32);
                dss += __shfl_xor(dss, 32);
                if (rg == 0) {
                    red[(wv * MB_BN + 16 * nb + col) * 2 + 0] = ds;
                    red[(wv * MB_BN + 16 * nb + col) * 2 + 1] = dss;
                }
            }
        }
    }
    if (p.gn) {
        __syncthreads();
        for (int e = tid; e < 2 * MB_BN; e += 64 * MB_NW) {
            const int gi = e / MB_BN, cl = e - gi * MB_BN;
            const int co = n0 + cl;
            const double s = red[((2 * gi) * MB_BN + cl) * 2 + 0] + red[((2 * gi + 1) * MB_BN + cl) * 2 + 0];
            const double ss = red[((2 * gi) * MB_BN + cl) * 2 + 1] + red[((2 * gi + 1) * MB_BN + cl) * 2 + 1];
            const int mg = m0 + 128 * gi;
            const int bb = mg / p.HoWo;
            const int split = (mg - bb * p.HoWo) / 128;
            double* dst = p.gn + (((size_t)bb * p.nsplit + split) * p.Cout + co) * 2;
            dst[0] = s;
            dst[1] = ss;
        }
    }
}

template <int W>
int launch3mb(const ConvParams& p, hipStream_t st) {
    static bool attr[2] = {};
    const bool ob2 = p.out_h2 != 0;
    void (*const k)(ConvParams) = ob2 ? &k_conv3mb<W, true> : &k_conv3mb<W, false>;
    constexpr size_t shm = conv3mb_lds_bytes(W);
    static_assert(shm <= 80 * 1024, "two workgroups per CU");
    if (!attr[ob2]) {
        if (hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm) !=
            hipSuccess) {
            set_error("tcx_conv2d_h2: cannot enable %zu B of dynamic LDS", shm);
            return TCX_EHIP;
        }
        attr[ob2] = true;
    }
    const int grid = (p.M / MB_TP) * p.n_nblk;
    hipLaunchKernelGGL(k, dim3(grid), dim3(64 * MB_NW), shm, st, p);
    return check_launch("tcx_conv2d_h2(bf16 16x16x32 tap pairs)");
}

}  // namespace

// Where it runs (measured per layer against k_conv3lb with its 3-slot ring, tools/mbbench.py at Bt = 84,
// profiles/r06_c_cfg5_conv_layers_mb_vs_lb.txt): faster at Cin >= 192 with a b2 output (down2.net.3 879 vs
// 926 us, up2.net.0 824 vs 855, mid.net.0 211 vs 218), slower at Cin = 96 (down1.net.3 1336 vs 1269 us,
// up1.net.0 1954 vs 1908) and with an fp32 output (up2.net.3 318 vs 284, mid.net.3 234 vs 219).  Taking the
// Cin >= 192 b2-output layers (mode 1) measured 1.1 % SLOWER end to end than k_conv3lb everywhere (config 5,
// three alternating pairs: 9.164 / 9.168 / 9.173 vs 9.264 / 9.276 / 9.287 images/s, profiles/r06_u_cfg5_ab.txt;
// mode 1 also caught up1.net.0's 256^2 concat, the layer it loses most on), so the default is mode 0 and the
// kernel stays for A/B.  Same products, same k order: the two kernels' outputs are bit-identical
// (tests/test_gpu_bf16.py test_b2_conv3mb_equals_conv3lb_bit_for_bit; the GroupNorm partials agree to the fp32
// rounding of their per-lane sums, taken over the 16x16 vs 32x32 accumulator layouts).  TCX_CONV3MB=1: Cin >= 192
// with a b2 output, 2: every b2 shape, 0 (default): never.
thread_local int g_conv3mb_force = -1;  // tcx_debug_conv3mb (tests): overrides the environment on this thread
int conv3mb_mode() {
    static const int m = [] {
        const char* e = getenv("TCX_CONV3MB");
        return (e && (e[0] == '1' || e[0] == '2')) ? e[0] - '0' : 0;
    }();
    return g_conv3mb_force >= 0 ? g_conv3mb_force : m;
}
bool conv3mb_takes(const ConvParams& p) {
    const int mode = conv3mb_mode();
    if (mode == 0 || (mode == 1 && (p.Cin < 192 || !p.out_h2))) return false;
    if (p.bf != 2 || !p.circular || !(p.W == 64 || p.W == 128 || p.W == 256) || p.wf == nullptr) return false;
    if (p.M % MB_TP != 0 || p.HoWo % MB_TP != 0 || p.Cin % 32 != 0 || p.Cout % MB_BN != 0) return false;
    if (p.cm1 || (p.cm2 && p.C2 % 16 != 0) || p.sc1 != nullptr || p.sc2 != nullptr) return false;
    return p.act == 0 && p.bias_b == nullptr && p.resid == nullptr && p.osy == 1 && p.osx == 1 && p.H == p.Ho &&
           p.W == p.Wo && p.wscale != nullptr && (long long)p.M * p.Cout < (1ll << 29);
}

int launch_conv3mb(const ConvParams& p, hipStream_t st) {
    if (p.W == 256) return launch3mb<256>(p, st);
    if (p.W == 128) return launch3mb<128>(p, st);
    return launch3mb<64>(p, st);
}

}  // namespace tcx

// Test hook: k_conv3mb's selection on this host thread (0 never, 1 the measured default, 2 every b2 3x3 shape
// it covers; -1 back to TCX_CONV3MB).  Returns the previous override.
extern "C" int tcx_debug_conv3mb(int mode) {
    const int prev = tcx::g_conv3mb_force;
    tcx::g_conv3mb_force = mode < -1 ? -1 : (mode > 2 ? 2 : mode);
    return prev;
}
