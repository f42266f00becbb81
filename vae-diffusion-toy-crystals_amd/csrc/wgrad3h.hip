// f16x3 weight gradient of the 3x3 stride-1 convs from a staged halo (round 6): the training step's
// dW[co][ci][ky][kx] = sum over (b, y, x) of dY[b, y, x, co] * x[b, y - 1 + ky, x - 1 + kx, ci] for the
// score net's 3x3 convs (sde_score_model.py:102,105 ResBlock convs, :208-222 the up / down path), the
// autograd weight gradient of nn.Conv2d(padding=1, padding_mode="circular").
//
// k_wgrad_h2 (gemm.hip) gathers an im2col tile per 128-k block, so every input pixel is fetched once per
// tap it feeds (9x) and dY once per k block (7-27x): per 32-pixel chunk it moves 28 KB for 32 x 128 x 96
// MACs, more than the L1 return path sustains (0.26 of the f16x3 ceiling, profiles/r06_d_*).  Here a
// workgroup owns ALL nine taps of one 32-channel group x 96 output channels and walks chunks of 32 pixels
// (half a row at W = 64, a row at 32, two rows at 16; TCX_W3_CP=64: 64-pixel chunks, one workgroup per CU):
//   * the chunk's input halo ((rows + 2) x (cols + 2) pixels x 32 channels, h2 records, 128 B per pixel) and
//     its dY block (32 pixels x 96 channels, 384 B per pixel) land in LDS by LDS-DMA (buffer_load ... lds,
//     no registers), in a three-stage ring: chunks c + 1 and c + 2 stream in while chunk c is multiplied
//     (with two stages the DMA latency, not the MFMA, set the chunk time: 4.6 us per 64-pixel chunk at 64^2);
//     at 32-pixel chunks the ring is 3 x 21-25 KB, so two workgroups share a CU and one's DMA issue and
//     address VALU run beside the other's MFMAs (268 vs 310 us per 64^2 96 -> 96 launch);
//   * the MFMA operands (8 consecutive pixels of one channel per lane) come from ds_read_b64_tr_b16 on the
//     pixel-major images, each tap reading the halo at its own (dy, dx) offset — the halo is fetched once
//     for all nine taps;
//   * 4 waves: wave w takes the 16-channel half (w & 1) of the group and 48 output channels (w >> 1): 9 taps x
//     3 tiles of v_mfma_f32_16x16x32_f16, three products each (hi*lo, lo*hi, hi*hi as k_wgrad_h2).
// LDS images are unswizzled rows of 16-B pieces with piece' = piece ^ f(row), f = bit 1 | bit 3 << 2 of the
// row: the tr reads of a half-wave (8 rows of a k step, 2 pieces each) then hit 16 distinct bank groups
// (checked exhaustively for every start row, both images).  Each workgroup writes its partial plane
// [9 Cin][Cout] slice; tcx_conv_wgrad_h2's k_wgrad_reduce folds the planes in a fixed order.
#include "common.hpp"
#include "h2.hpp"

#include <algorithm>
#include <mutex>
#include <utility>

namespace tcx {

struct Wg3hArgs {
    const char* x1;
    const char* x2;   // h2 records [B][H][W][C1] / [C2] (4 B per element)
    const char* dy;   // h2 records [B][H][W][Cout]
    unsigned bx1, bx2, bdy;
    int B, H, W, C1, C2, Cin, Cout, circular;
    int RB;           // image rows per 64-pixel chunk (64 / W)
    int nchunk, cps;  // chunks (B H / RB), chunks per split
    int ncob;         // Cout / 96
    const float* comb;
    float* part;      // [nsplit][9 Cin][Cout]
};

namespace {

constexpr int W3_WAIT_VM0 = 0x0F70;    // s_waitcnt vmcnt(0)

// chunk geometry: CP pixels per chunk (32 or 64) as RB rows x SW columns of one image (SW = min(W, CP))
__host__ __device__ constexpr int w3_sw(int W, int CP) { return W < CP ? W : CP; }
__host__ __device__ constexpr int w3_rb(int W, int CP) { return CP / w3_sw(W, CP); }
__host__ __device__ constexpr int w3_halo_px(int W, int CP) { return (w3_rb(W, CP) + 2) * (w3_sw(W, CP) + 2); }
__host__ __device__ constexpr int w3_nh(int W, int CP) { return (w3_halo_px(W, CP) * 128 + 1023) / 1024; }
__host__ __device__ constexpr int w3_nt(int W, int CP) { return w3_nh(W, CP) + CP * 384 / 1024; }  // 1-KB DMAs
__host__ __device__ constexpr int w3_stage(int W, int CP) { return w3_nt(W, CP) * 1024; }
// NS: ring depth (chunks c + 1 .. c + NS - 1 stream in while chunk c is multiplied)
constexpr size_t wgrad3h_lds_bytes(int W, int CP, int NS) { return NS * (size_t)w3_stage(W, CP); }
static_assert(wgrad3h_lds_bytes(64, 64, 3) <= 160 * 1024 && wgrad3h_lds_bytes(64, 32, 3) <= 80 * 1024 &&
                  wgrad3h_lds_bytes(32, 32, 3) <= 80 * 1024 && wgrad3h_lds_bytes(16, 32, 3) <= 80 * 1024 &&
                  wgrad3h_lds_bytes(64, 32, 6) <= 160 * 1024 && wgrad3h_lds_bytes(16, 32, 6) <= 160 * 1024,
              "wgrad3h ring exceeds the CU's LDS");
// s_waitcnt vmcnt(n), n <= 63 (gfx9 split field), no expcnt / lgkmcnt wait
__host__ __device__ constexpr int w3_vm(int n) { return 0x0F70 | (n & 15) | ((n >> 4) << 14); }
template <typename F, int... Is>
__device__ __forceinline__ void w3_for(F&& f, std::integer_sequence<int, Is...>) {
    (f(std::integral_constant<int, Is>{}), ...);
}

__device__ __forceinline__ int w3_swz(int row) { return ((row >> 1) & 1) | (((row >> 3) & 1) << 2); }

__device__ __forceinline__ void w3_dma16(__amdgpu_buffer_rsrc_t r, char* lds, int voff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, voff, 0, 0, 0);
}

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short v4s __attribute__((ext_vector_type(4)));
typedef short v8s __attribute__((ext_vector_type(8)));

// CP = 64: one workgroup per CU (the ring is 3 x 49-52 KB); CP = 32, NWG = 2: two per CU (3 x 21-25 KB each),
// whose waves' DMA / VALU then run beside the other workgroup's MFMAs.  Measured and dropped: CP = 32 with a
// six-deep ring and one workgroup per CU (410 vs 268 us per 64^2 launch: not the DMA latency, the co-resident
// waves are the lever) and three workgroups per CU (two stages; 168 VGPRs: 80 spilled)
template <int W, int CP, int NS, int NWG>
__global__ __launch_bounds__(256, NWG) void k_wgrad3h(Wg3hArgs a) {
    constexpr int SW = w3_sw(W, CP), RB = w3_rb(W, CP), NSEG = W / SW, W2 = SW + 2;
    constexpr int HPX = w3_halo_px(W, CP);
    constexpr int NH = w3_nh(W, CP);   // halo DMA instructions per chunk (1 KB each)
    constexpr int HB = NH * 1024;
    constexpr int NT = w3_nt(W, CP);   // + the dY block's (CP x 384 B)
    constexpr int STG = NT * 1024;
    constexpr int PHI = (NT + 3) / 4, PLO = NT / 4;  // DMA instructions of waves wv < NT % 4 / the others
    static_assert(PHI <= 15, "vmcnt immediate");
    extern __shared__ __attribute__((aligned(1024))) char sm[];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int tile = blockIdx.x, split = blockIdx.y;
    const int grp = tile / a.ncob, cob = tile - (tile / a.ncob) * a.ncob;
    const int c0 = grp * 32;  // first channel of the group in the concatenated input
    const bool s1 = c0 < a.C1;
    const int Cs = s1 ? a.C1 : a.C2;
    const int cbyte = (s1 ? c0 : c0 - a.C1) * 4;  // byte offset of the group in the source record
    const __amdgpu_buffer_rsrc_t rx =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(s1 ? a.x1 : a.x2), 0, (int)(s1 ? a.bx1 : a.bx2), 0x00020000);
    const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(a.dy), 0, (int)a.bdy, 0x00020000);
    constexpr int OOB = (int)0x80000000u;
    const int H = a.H;
    const int ch0 = split * a.cps;
    const int ch1 = min(ch0 + a.cps, a.nchunk);

    // this wave's DMA instructions of a chunk: i = wv, wv + 4, ... below NT (halo first, then dY)
    auto issue = [&](int c, int buf) {
        const int rbk = c / NSEG, sg = c - (c / NSEG) * NSEG;
        const int row0 = rbk * RB;  // first image row of the chunk in the B H row space
        const int x0 = sg * SW;
        const int b = row0 / H, y0 = row0 - (row0 / H) * H;
        char* st = sm + buf * STG;
#pragma unroll
        for (int k = 0; k < PHI; ++k) {
            const int i = 4 * k + wv;
            if (i >= NT) break;
            if (i < NH) {
                const int u = i * 64 + lane;  // physical 16-B unit of the halo image
                const int hp = u >> 3, lp = (u & 7) ^ w3_swz(u >> 3);
                const int hr = hp / W2, hc = hp - (hp / W2) * W2;
                int y = y0 + hr - 1, x = x0 + hc - 1;
                bool ok = hp < HPX;
                if (a.circular) {
                    y = wrap_idx(y, H);
                    x = wrap_idx(x, W);
                } else {
                    ok = ok && y >= 0 && y < H && x >= 0 && x < W;
                }
                const int voff = ok ? ((b * H + y) * W + x) * (Cs * 4) + cbyte + 16 * lp : OOB;
                w3_dma16(rx, st + i * 1024, voff);
            } else {
                const int u = (i - NH) * 64 + lane;  // physical unit of the dY image: 24 per pixel
                const int px = u / 24, lp = (u - (u / 24) * 24) ^ w3_swz(u / 24);
                const int r = px / SW, xx = px - (px / SW) * SW;
                const int voff = (((row0 + r) * W + x0 + xx) * a.Cout + 96 * cob) * 4 + 16 * lp;
                w3_dma16(rd, st + HB + (i - NH) * 1024, voff);
            }
        }
    };

    // tr-read lane roles (16x16x32 operands): k group g = lane / 16 (8 pixels), row q = (lane / 4) % 4,
    // column pp = lane % 4 (4 channels: piece pp / 2, half pp % 2)
    const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
    const int half8 = 8 * (pp & 1);
    const int cbh = wv & 1;   // 16-channel half of the group: hi pieces 4 cbh, 4 cbh + 2
    const int coh = wv >> 1;  // output-channel half: 16-channel blocks 3 coh .. 3 coh + 2
    // The tr reads are inline asm: hipcc orders every C++ LDS read after a pending LDS-DMA with vmcnt(0),
    // which would wait for chunk c + 1's DMA before chunk c's first read.  Their lgkmcnt waits are explicit
    // asm that names the fragment registers (so no use is scheduled above its wait), and sched barriers keep
    // the next tap's reads ahead of this tap's MFMAs.
    const int lds0 = (int)(size_t)((__attribute__((address_space(3))) char*)sm);
    auto trd = [&](int addr) {
        v4s r;
        asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(addr));
        return r;
    };
    // rows r0 + q and r0 + 4 + q of an image at byte base (row bytes rby), logical piece L + 2 (pp / 2)
    auto frag2 = [&](int base, int rby, int r0, int L, v4s& u0, v4s& u1) {
        const int lp = L + 2 * (pp >> 1);
        const int ra = r0 + q, rb = r0 + 4 + q;
        u0 = trd(base + ra * rby + 16 * (lp ^ w3_swz(ra)) + half8);
        u1 = trd(base + rb * rby + 16 * (lp ^ w3_swz(rb)) + half8);
    };
    auto cat = [](v4s u0, v4s u1) -> h8 {
        return __builtin_bit_cast(h8, __builtin_shufflevector(u0, u1, 0, 1, 2, 3, 4, 5, 6, 7));
    };

    f32x4 acc[9][3];
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int j = 0; j < 3; ++j) acc[t][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

#pragma unroll
    for (int k = 0; k < NS - 1; ++k)
        if (ch0 + k < ch1) issue(ch0 + k, k);
    const bool whi = wv < NT % 4;  // this wave issues PHI DMA instructions per chunk, else PLO
    for (int c = ch0; c < ch1; ++c) {
        const int buf = (c - ch0) % NS;
        // this wave's DMA of chunk c landed (the newer chunks' may still be in flight)
        const int newer = min(NS - 2, ch1 - 1 - c);
        static_assert((NS - 2) * PHI <= 63, "vmcnt range");
        w3_for([&](auto K) {
            constexpr int k = decltype(K)::value;
            if (newer == k) {
                if (whi) __builtin_amdgcn_s_waitcnt(w3_vm(k * PHI));
                else __builtin_amdgcn_s_waitcnt(w3_vm(k * PLO));
            }
        }, std::make_integer_sequence<int, NS - 1>{});
        // every wave's; the stage of chunk c - 1 is no longer read.  A bare s_barrier: __syncthreads' fence
        // would drain vmcnt, i.e. chunk c + 1's DMA as well
        __builtin_amdgcn_s_barrier();
        if (c + NS - 1 < ch1) issue(c + NS - 1, (buf + NS - 1) % NS);
        const int X = lds0 + buf * STG;
        const int D = X + HB;
#pragma unroll
        for (int s = 0; s < CP / 32; ++s) {  // k steps of 32 pixels
            const int o = 32 * s + 8 * g;       // this lane group's first chunk pixel
            const int r = o / SW, x = o - (o / SW) * SW;
            v4s Bf[3][4], Af[2][4];             // [hi u0, hi u1, lo u0, lo u1]
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                const int m = 3 * coh + j;  // 16-channel block of the 96: hi pieces 4 m, 4 m + 2
                frag2(D, 384, o, 4 * m, Bf[j][0], Bf[j][1]);
                frag2(D, 384, o, 4 * m + 1, Bf[j][2], Bf[j][3]);
            }
            auto readA = [&](int t, v4s* A) {
                const int ty = t / 3, tx = t - (t / 3) * 3;
                const int h0 = (r + ty) * W2 + x + tx;  // halo row of the lane group's first pixel at tap t
                frag2(X, 128, h0, 4 * cbh, A[0], A[1]);
                frag2(X, 128, h0, 4 * cbh + 1, A[2], A[3]);
            };
            readA(0, Af[0]);
            asm volatile("s_waitcnt lgkmcnt(0)"
                         : "+v"(Bf[0][0]), "+v"(Bf[0][1]), "+v"(Bf[0][2]), "+v"(Bf[0][3]), "+v"(Bf[1][0]),
                           "+v"(Bf[1][1]), "+v"(Bf[1][2]), "+v"(Bf[1][3]), "+v"(Bf[2][0]), "+v"(Bf[2][1]),
                           "+v"(Bf[2][2]), "+v"(Bf[2][3]), "+v"(Af[0][0]), "+v"(Af[0][1]), "+v"(Af[0][2]),
                           "+v"(Af[0][3]));
            __builtin_amdgcn_sched_barrier(0);
            h8 bh[3], bl[3];
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                bh[j] = cat(Bf[j][0], Bf[j][1]);
                bl[j] = cat(Bf[j][2], Bf[j][3]);
            }
#pragma unroll
            for (int t = 0; t < 9; ++t) {
                v4s* An = Af[(t + 1) & 1];
                if (t < 8) readA(t + 1, An);
                __builtin_amdgcn_sched_barrier(0);
                const v4s* Ac = Af[t & 1];
                const h8 ah = cat(Ac[0], Ac[1]), al = cat(Ac[2], Ac[3]);
#pragma unroll
                for (int j = 0; j < 3; ++j) acc[t][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl[j], acc[t][j], 0, 0, 0);
#pragma unroll
                for (int j = 0; j < 3; ++j) acc[t][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh[j], acc[t][j], 0, 0, 0);
#pragma unroll
                for (int j = 0; j < 3; ++j) acc[t][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh[j], acc[t][j], 0, 0, 0);
                __builtin_amdgcn_sched_barrier(0);
                if (t < 8) asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(An[0]), "+v"(An[1]), "+v"(An[2]), "+v"(An[3]));
            }
        }
    }
    __builtin_amdgcn_s_waitcnt(W3_WAIT_VM0);
    // partial plane: k = tap Cin + ci, ci = c0 + 16 cbh + 4 g + e (rows of the 16x16 tile), co = l % 16
    const float sc = *a.comb;
    float* dst = a.part + (size_t)split * 9 * a.Cin * a.Cout;
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const int co = 96 * cob + 16 * (3 * coh + j) + (lane & 15);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int k = t * a.Cin + c0 + 16 * cbh + 4 * g + e;
                dst[(size_t)k * a.Cout + co] = acc[t][j][e] * sc;
            }
        }
}

thread_local int g_wgrad3h_force = -1;  // tcx_debug_wgrad3h: -1 default, 0 off, 1 on

}  // namespace

// tcx_conv_wgrad_h2 (gemm.hip): true when this 3x3 shape runs here
bool wgrad3h_takes(int B, int H, int W, int C1, int C2, int Cout, int ks, int stride, int pad, size_t in1, size_t in2,
                   size_t ind) {
    static const bool off = getenv("TCX_WGRAD3H") && getenv("TCX_WGRAD3H")[0] == '0';  // A/B: k_wgrad_h2
    const bool on = g_wgrad3h_force >= 0 ? g_wgrad3h_force == 1 : !off;
    const size_t lim = (size_t)1 << 31;
    return on && ks == 3 && stride == 1 && pad == 1 && (W == 16 || W == 32 || W == 64) && H % (64 / W) == 0 &&
           B > 0 && C1 % 32 == 0 && (C2 == 0 || C2 == C1) && Cout % 96 == 0 && in1 < lim && in2 < lim && ind < lim;
}

// max_split: the partial planes the caller's workspace holds; *nsplit: the planes written
int launch_wgrad3h(Wg3hArgs& a, int max_split, int* nsplit, hipStream_t st) {
    static const int cp = [] {  // chunk pixels: 32 (default) or 64 (one workgroup per CU, three stages; A/B)
        const char* e = getenv("TCX_W3_CP");
        return e && atoi(e) == 64 ? 64 : 32;
    }();
    const int per_cu = cp == 64 ? 1 : 2;
    a.nchunk = a.B * a.H * a.W / cp;
    a.ncob = a.Cout / 96;
    const int tiles = (a.Cin / 32) * a.ncob;
    int ns = std::max(1, std::min({max_split, std::max(1, 256 * per_cu / tiles), a.nchunk}));
    a.cps = cdiv(a.nchunk, ns);
    ns = cdiv(a.nchunk, a.cps);
    using K = void (*)(Wg3hArgs);
    K k;
    size_t lds;
    const int wi = a.W == 64 ? 0 : (a.W == 32 ? 1 : 2);
    int ki;
    if (cp == 64) {
        k = a.W == 64 ? &k_wgrad3h<64, 64, 3, 1> : (a.W == 32 ? &k_wgrad3h<32, 64, 3, 1> : &k_wgrad3h<16, 64, 3, 1>);
        lds = wgrad3h_lds_bytes(a.W, 64, 3);
        ki = wi;
    } else {
        k = a.W == 64 ? &k_wgrad3h<64, 32, 3, 2> : (a.W == 32 ? &k_wgrad3h<32, 32, 3, 2> : &k_wgrad3h<16, 32, 3, 2>);
        lds = wgrad3h_lds_bytes(a.W, 32, 3);
        ki = 3 + wi;
    }
    // the dynamic-LDS opt-in once per kernel variant (host threads may race to the first call)
    static std::once_flag once[6];
    static hipError_t attr_rc[6];
    std::call_once(once[ki], [&] {
        attr_rc[ki] = hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                          (int)lds);
    });
    if (attr_rc[ki] != hipSuccess) {
        set_error("tcx_conv_wgrad_h2: cannot enable %zu B of dynamic LDS", lds);
        return TCX_EHIP;
    }
    hipLaunchKernelGGL(k, dim3(tiles, ns), dim3(256), lds, st, a);
    *nsplit = ns;
    return check_launch("tcx_conv_wgrad_h2 (halo)");
}

}  // namespace tcx

extern "C" int tcx_debug_wgrad3h(int mode) {
    const int prev = tcx::g_wgrad3h_force;
    tcx::g_wgrad3h_force = mode < 0 ? -1 : (mode ? 1 : 0);
    return prev;
}
