// k_conv4s2g: the U-Net's 4x4 stride-2 circular downsamples ds1 / ds2 (/root/reference/src/toycrystals/
// models/sde_score_model.py:208,210) on the split path with ALL staging by LDS-DMA, in the manner of
// k_conv3lg (conv3l.hip).
//
// What it replaces: k_conv4s2h (conv4s2h.hip) stages the halo and the weights through registers with a
// barrier per tap pair, reads every B fragment right before its MFMAs (exposed LDS latency each pair)
// and keeps one halo buffer (an extra barrier per input-channel slice): 0.35 / 0.42 of the f16x3
// ceiling on ds1 / ds2.
//
// Geometry.  A workgroup owns 128 output pixels (TR = 128 / Wo whole output rows) x 96 output
// channels; 4 waves x 32 pixels.  The input is consumed in 8-channel chunks: one chunk's halo is
// (2 TR + 2) input rows x (2 Wo + 2) columns, stored column-parity deinterleaved (even columns, then
// odd, Wo + 1 each) in 32-B slots = the h2 record of 8 channels (16-B hi piece, 16-B lo piece), so the
// stride-2 taps of consecutive output pixels read consecutive slots.  A 16-deep MFMA k-step takes TWO
// taps of the chunk: lanes lh = 0 / 1 read taps (dy, 2p) / (dy, 2p + 1), so a chunk is 8 k-steps
// (dy = 0..3, p = 0..1), 9 MFMAs per k-step per wave (3 n-tiles x 3 split products).  The 16-B pieces
// are XOR-swizzled by (halo row & 1) ^ ((halo column >> 3) & 1) with two pad slots per halo row: the
// ds_read_b128 lane groups then hit distinct 16-B bank positions; the DMA writes lane-linearly (lane l -> slot 32 i + l / 2, physical piece l & 1), so the
// swizzle and the parity deinterleave ride on the per-lane source address.
//
// Pipeline (per wave, k-step c of chunk j = c / 8): B fragments come from a fragment-ordered weight
// copy (tcx_pack_conv_weight_h2_frag4: [n-block][k-step][n][hi, lo][lane][16 B]) in two-k-step pairs
// (12 KB) through a two-pair LDS ring, DMA'd by waves 0-1 at the start of odd k-step 2k - 3 and waited
// for at the barrier ending (even) k-step 2k - 2; the halo of chunk j + 1 is DMA'd by waves 2-3 into the other
// buffer over k-steps 0-3 of chunk j and waited for at the barrier ending k-step 6.  A and B of k-step
// c + 1 are read during k-step c's MFMAs.  One barrier per two k-steps, explicit s_waitcnt before raw
// s_barrier (hipcc's __syncthreads would drain every DMA in flight).  Epilogue shared with the conv
// kernels (conv_common.hpp).  BF: bf16 records, one MFMA of the hi halves per product.
#include "conv_common.hpp"

namespace tcx {
namespace {

constexpr int Q_TP = 128;                       // output pixels per tile and row block of waves (RT = 1)
constexpr int Q_PAIR = 2 * 3 * 2 * 1024;        // B fragments of two k-steps (12 KB)
__host__ __device__ constexpr int q_rs(int Wo) { return 2 * Wo + 4; }  // both parities (Wo + 1 each) + 2 pad
__host__ __device__ constexpr int q_npx(int Wo, int RT = 1) { return (2 * (RT * Q_TP / Wo) + 2) * q_rs(Wo); }
// SLIM (2-byte bf16 sources, h2.hpp "b2"): a slot is the 16-B hi piece of the 8-channel chunk only, 64
// slots per 1-KB DMA instruction, consecutive and unswizzled (a ds_read_b128 lane group reads 16
// consecutive 16-B slots of one parity row: every bank once); config 5's ds1 (Wo = 128) fits only so
__host__ __device__ constexpr int q_ni(int Wo, bool SLIM = false, int RT = 1) {
    return (q_npx(Wo, RT) + (SLIM ? 63 : 31)) / (SLIM ? 64 : 32);
}
constexpr size_t conv4s2g_lds_bytes(int Wo, bool SLIM = false, int RT = 1) {
    return (size_t)2 * q_ni(Wo, SLIM, RT) * 1024 + 2 * (size_t)Q_PAIR;
}
constexpr int Q_WAIT_VM0 = 0x0F70;
constexpr int Q_WAIT_LGKM0 = 0xC07F;

__device__ __forceinline__ void q_dma16(__amdgpu_buffer_rsrc_t r, char* lds, int voff, int soff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, voff, soff, 0, 0);
}

// RT (round 5): row blocks of 32 pixels per wave, so a tile is 128 RT pixels.  RT = 2 doubles the output
// rows of a tile, so fewer halo rows are staged per output row (6 input rows for 2 output rows at Wo = 128,
// where RT = 1 staged 4 for 1), and every B fragment read serves two A fragments (config 5's b2 forms)
template <int Wo, bool BF, bool SLIM = false, int RT = 1>
__global__ __launch_bounds__(256, 2) void k_conv4s2g(ConvParams p) {
    static_assert(!SLIM || BF, "the slim slot holds the bf16 hi piece only");
    constexpr int NT = 3;
    constexpr int TP = RT * Q_TP;        // output pixels per tile
    constexpr int TR = TP / Wo;          // output rows per tile
    constexpr int RS = q_rs(Wo);         // halo slots per halo row (both column parities + 2 pad)
    constexpr int NPX = q_npx(Wo, RT);
    constexpr int NI = q_ni(Wo, SLIM, RT);
    constexpr int NIH = (NI + 1) / 2;    // halo DMA instructions per halo wave
    constexpr int HB = NI * 1024;
    constexpr int RING = 2 * HB;
    static_assert(TR * Wo == TP, "tile = whole output rows");
    extern __shared__ __attribute__((aligned(16))) float sm[];
    char* const smc = reinterpret_cast<char*>(sm);
    int lz;  // LDS-DMA destinations from a base the optimiser cannot fold to a constant (conv3l.hip)
    asm volatile("s_mov_b32 %0, 0" : "=s"(lz));
    char* const smd = smc + lz;

    const int tid = threadIdx.x;
    const int lane = tid & 63, li = lane & 31, lh = lane >> 5;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int tile = xcd_remap(blockIdx.x, gridDim.x);
    const int mblk = tile / p.n_nblk;
    const int nblk = tile - mblk * p.n_nblk;
    const int m0 = mblk * TP, n0 = nblk * 32 * NT;
    const int b = m0 / p.HoWo;
    const int r0 = (m0 - b * p.HoWo) / Wo;  // first output row of the tile
    const int bs = p.bmod > 0 ? b % p.bmod : b;
    const int H = p.H, W = p.W;             // input dims (= 2 Ho, 2 Wo)
    const int nck = p.Cin / 8;              // 8-channel chunks
    const int nks = 8 * nck;                // k-steps
    const int npair = nks / 2;

    const __amdgpu_buffer_rsrc_t r1 = mk_rsrc(p.x1, p.bytes1);
    const __amdgpu_buffer_rsrc_t rw = mk_rsrc(reinterpret_cast<const float*>(p.wf), p.bytesw);

    // ---- halo DMA (waves 2-3: instruction i = 2 q + (wv & 1)); lane l -> slot 32 i + l / 2, physical
    // piece l & 1, logical piece (l & 1) ^ swz(slot); slots past the halo re-read its last pixel
    const int hw = wv & 1;
    // b2 sources (BF, p.bf == 2, h2.hpp): the 8-channel chunk is ONE 16-B hi piece at byte 16 j of the
    // pixel's 2-byte row; both DMA lanes of a slot read it (the lo slot half is never read by BF)
    const bool b2 = BF && p.bf == 2;
    // chunk-major source (p.cm1, ConvParams): the 8-channel chunk j is the plane at byte j * plane, a
    // pixel's record at 32 * pixel inside it (h2 records), or its 16-B b2 piece at 16 * pixel (config 5,
    // round 6: gn_apply_b2cm's planes)
    const bool cm = (!BF || b2) && p.cm1;
    const int rowb = cm ? (b2 ? 16 : 32) : p.C1 * (b2 ? 2 : 4);
    const int plane = cm ? (int)(p.bytes1 / (unsigned)(p.C1 / 8)) : 32;
    const int cstride = cm ? plane : (b2 ? 16 : plane);  // byte distance of consecutive chunks
    auto halo_voff = [&](int i) {
        // RT = 2: recomputed at every issue from an opaque copy of the lane index (hoisted out of the chunk
        // loop, the offsets of all NI instructions spilled beside the doubled accumulators; k_conv3m's note)
        int ln = lane;
        if constexpr (RT == 2) asm volatile("v_mov_b32 %0, %1" : "=v"(ln) : "v"(lane));
        int s = SLIM ? 64 * i + ln : 32 * i + (ln >> 1);
        s = s < NPX ? s : NPX - 1;
        const int hr = s / RS, hc = s - (s / RS) * RS;
        const int swz = SLIM ? 0 : (hr & 1) ^ ((hc >> 3) & 1);
        const int par = hc >= Wo + 1 ? 1 : 0;
        const int cc = min(hc - par * (Wo + 1), Wo);  // the 2 pad slots re-read column Wo
        const int y = wrap_idx(2 * r0 - 1 + hr, H), x = wrap_idx(2 * cc + par - 1, W);
        return ((bs * H + y) * W + x) * rowb + (b2 ? 0 : 16 * ((ln & 1) ^ swz));
    };
    auto halo_issue = [&](int j, int buf, int q0, int q1) {
#pragma unroll
        for (int q = 0; q < NIH; ++q) {
            if (q < q0 || q >= q1) continue;
            const int i = 2 * q + hw;
            if (i < NI) q_dma16(r1, smd + buf * HB + i * 1024, halo_voff(i), cstride * j);
        }
    };
    // ---- weight pairs (waves 0-1): pair k = k-steps 2k, 2k + 1 -> ring slot k & 1; wave w moves KB [6 w, 6 w + 6)
    auto pair_issue = [&](int k) {
        k = k < npair ? k : npair - 1;
        const int base = (nblk * nks + 2 * k) * NT * 2048 + wv * 6144;
        char* const d = smd + RING + (k & 1) * Q_PAIR + wv * 6144;
#pragma unroll
        for (int i = 0; i < 6; ++i) q_dma16(rw, d + i * 1024, lane * 16, base + i * 1024);
    };

    // ---- A fragments: lane (li, lh) of k-step (dy, p) reads tap (dy, dx = 2 p + lh) of its pixel:
    // slot (2 r + dy) RS + (dx & 1)(Wo + 1) + c + (dx >> 1), r / c = the pixel's row / column in the tile
    // row block rt of wave wv is virtual wave RT wv + rt (the epilogue's numbering)
    int abase[RT], asw0[RT], asw1[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
        const int mloc = (RT * wv + rt) * 32 + li;
        const int ahc = (mloc % Wo) + lh * (Wo + 1);  // halo column of k-step p = 0 (dx = 2 p + lh)
        abase[rt] = 2 * (mloc / Wo) * RS + ahc;       // + dy RS + p
        // piece swizzle of a slot (hr, hc): (hr & 1) ^ ((hc >> 3) & 1) — with the 2 pad slots per halo row,
        // conflict-free for every ds_read_b128 lane group, tap and row width 16 / 32 / 64 (exhaustive check);
        // hr = 2 r + dy, so its parity is dy's
        asw0[rt] = (ahc >> 3) & 1;
        asw1[rt] = ((ahc + 1) >> 3) & 1;
    }
    f32x16 acc[RT][NT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int n = 0; n < NT; ++n) acc[rt][n] = (f32x16){};
    h8 a_h[2][RT], a_l[2][RT], b_h[2][NT], b_l[2][NT];
    auto rd_a = [&](int set, int kc, int hb) {  // k-step kc = 2 dy + p of the chunk in halo buffer hb
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
            const int s = abase[rt] + (kc >> 1) * RS + (kc & 1);
            const int sw = ((kc >> 1) & 1) ^ ((kc & 1) ? asw1[rt] : asw0[rt]);
            const char* A = smc + hb * HB + s * (SLIM ? 16 : 32);
            a_h[set][rt] = __builtin_bit_cast(h8, *reinterpret_cast<const float4*>(A + (SLIM ? 0 : 16 * sw)));
            if constexpr (!BF)
                a_l[set][rt] = __builtin_bit_cast(h8, *reinterpret_cast<const float4*>(A + 16 * (sw ^ 1)));
        }
    };
    const int bl = lane * 16;
    auto rd_b = [&](int set, int c) {  // k-step c: ring slot (c >> 1) & 1, half c & 1
        const char* B = smc + RING + ((c >> 1) & 1) * Q_PAIR + (c & 1) * (Q_PAIR / 2) + bl;
#pragma unroll
        for (int n = 0; n < NT; ++n) {
            b_h[set][n] = __builtin_bit_cast(h8, *reinterpret_cast<const float4*>(B + n * 2048));
            if constexpr (!BF) b_l[set][n] = __builtin_bit_cast(h8, *reinterpret_cast<const float4*>(B + n * 2048 + 1024));
        }
    };
    auto mf = [&](int set) {
        if constexpr (BF) {
#pragma unroll
            for (int rt = 0; rt < RT; ++rt)
#pragma unroll
                for (int n = 0; n < NT; ++n)
                    acc[rt][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf8, a_h[set][rt]),
                                                                         __builtin_bit_cast(bf8, b_h[set][n]), acc[rt][n],
                                                                         0, 0, 0);
            return;
        }
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
            for (int n = 0; n < NT; ++n)
                acc[rt][n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a_h[set][rt], b_l[set][n], acc[rt][n], 0, 0, 0);
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
            for (int n = 0; n < NT; ++n)
                acc[rt][n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a_l[set][rt], b_h[set][n], acc[rt][n], 0, 0, 0);
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
            for (int n = 0; n < NT; ++n)
                acc[rt][n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a_h[set][rt], b_h[set][n], acc[rt][n], 0, 0, 0);
    };
    auto barrier = [&]() {
        __builtin_amdgcn_s_waitcnt(Q_WAIT_LGKM0);
        __builtin_amdgcn_s_barrier();
    };

    // ---- prologue: pairs 0, 1 and halo 0 in LDS, fragments of k-step 0 in registers
    if (wv < 2) {
        pair_issue(0);
        pair_issue(1);
    } else {
        halo_issue(0, 0, 0, NIH);
    }
    __builtin_amdgcn_s_waitcnt(Q_WAIT_VM0);
    barrier();
    rd_a(0, 0, 0);
    rd_b(0, 0);

    // k-step kc (compile time) of chunk j, register set s = kc & 1 holds its fragments
    auto step = [&](int j, auto KC, auto HBc) {
        constexpr int kc = decltype(KC)::value;
        constexpr int s = kc & 1;
        constexpr int hb = decltype(HBc)::value;
        const int c = 8 * j + kc;
        const bool more = j + 1 < nck;
        if (wv < 2) {
            if constexpr (s == 1) pair_issue((c + 3) >> 1);
        } else if constexpr (kc < 4) {
            constexpr int q0 = (NIH * kc) / 4, q1 = (NIH * (kc + 1)) / 4;
            if (more) halo_issue(j + 1, hb ^ 1, q0, q1);
        }
        __builtin_amdgcn_sched_barrier(0);
        // fragments of k-step c + 1 (the next chunk's k-step 0 from the other halo buffer)
        if (c + 1 < nks) {
            if constexpr (kc == 7) rd_a(s ^ 1, 0, hb ^ 1);
            else rd_a(s ^ 1, kc + 1, hb);
            rd_b(s ^ 1, c + 1);
        }
        __builtin_amdgcn_sched_barrier(0);
        mf(s);
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (s == 0) {  // even k-step 2k - 2: the barrier that publishes pair k (DMA'd from the
                                 // start of k-step 2k - 3) and, at kc = 6, the halo of chunk j + 1 (first
                                 // read at kc = 7); it also frees the ring slot / halo buffer read before it
            if (wv < 2 || kc == 6) __builtin_amdgcn_s_waitcnt(Q_WAIT_VM0);
            barrier();
        }
    };
    using H0 = std::integral_constant<int, 0>;
    using H1 = std::integral_constant<int, 1>;
    auto chunk = [&](int j, auto HBc) {
        step(j, std::integral_constant<int, 0>{}, HBc);
        step(j, std::integral_constant<int, 1>{}, HBc);
        step(j, std::integral_constant<int, 2>{}, HBc);
        step(j, std::integral_constant<int, 3>{}, HBc);
        step(j, std::integral_constant<int, 4>{}, HBc);
        step(j, std::integral_constant<int, 5>{}, HBc);
        step(j, std::integral_constant<int, 6>{}, HBc);
        step(j, std::integral_constant<int, 7>{}, HBc);
    };
    int j = 0;
    for (; j + 1 < nck; j += 2) {
        chunk(j, H0{});
        chunk(j + 1, H1{});
    }
    if (j < nck) chunk(j, H0{});

    __builtin_amdgcn_s_waitcnt(Q_WAIT_VM0);  // the clamped tail pairs land before LDS is reused
    __syncthreads();
    double* red = reinterpret_cast<double*>(sm);
    conv_epi_store_rt<NT, BF ? 2 : 1, RT * 4, RT>(p, acc, m0, n0, RT * wv, lane, red);
    if (p.gn) {
        __syncthreads();
        conv_epi_gn<NT, RT * 4>(p, m0, n0, tid, 256, red);
    }
}

// fragment-ordered copy of a 4x4 h2 weight [cout_pad][16 Cin] (k = (4 dy + dx) Cin + ci):
// wf[nb][k-step c = 8 j + 2 dy + p][n][hi, lo][lane][16 B] = the 8 hi (or lo) halves of row
// 96 nb + 32 n + (lane & 31) at k = (4 dy + 2 p + (lane >> 5)) Cin + 8 j
__global__ void k_pack_frag4(const char* __restrict__ wh, char* __restrict__ wf, int kpad, int Cin, int nblk_n) {
    const int nks = Cin;  // 8 k-steps per 8-channel chunk
    const size_t n16 = (size_t)nblk_n * nks * 3 * 2 * 64;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
        const int lane = (int)(i & 63);
        size_t q = i >> 6;
        const int hl = (int)(q & 1);
        q >>= 1;
        const int n = (int)(q % 3);
        q /= 3;
        const int c = (int)(q % nks);
        const int nb = (int)(q / nks);
        const int jj = c >> 3, kc = c & 7;
        const int dy = kc >> 1, pp = kc & 1;
        const int row = nb * 96 + n * 32 + (lane & 31);
        const int k = (4 * dy + 2 * pp + (lane >> 5)) * Cin + 8 * jj;
        *reinterpret_cast<float4*>(wf + i * 16) =
            *reinterpret_cast<const float4*>(wh + ((size_t)row * kpad + k) * 4 + hl * 16);
    }
}

// row blocks per wave of the slim b2 forms: 2 at Wo = 64 (config 5's ds2: 786 -> 672 us), 1 at Wo = 128
// (config 5's ds1: 1051 -> 1313 us with RT = 2; profiles/r05_r_*); TCX_DS_RT=1 / 2 forces it (A/B, tests)
int ds_rt(bool slim, int Wo) {
    static const int forced = [] {
        const char* e = getenv("TCX_DS_RT");
        return e && (e[0] == '1' || e[0] == '2') ? e[0] - '0' : 0;
    }();
    return forced ? forced : (slim && Wo == 64 ? 2 : 1);
}

template <int Wo, bool BF, bool SLIM, int RT>
int launch_q_one(const ConvParams& p, hipStream_t st) {
    constexpr size_t shm = conv4s2g_lds_bytes(Wo, SLIM, RT);
    static_assert(shm <= 160 * 1024, "LDS");
    static bool attr = false;
    auto kc = &k_conv4s2g<Wo, BF, SLIM, RT>;
    if (!attr) {
        if (hipFuncSetAttribute(reinterpret_cast<const void*>(kc), hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)shm) != hipSuccess) {
            set_error("tcx_conv2d_h2: cannot enable %zu B of dynamic LDS", shm);
            return TCX_EHIP;
        }
        attr = true;
    }
    hipLaunchKernelGGL(kc, dim3((p.M / (RT * Q_TP)) * p.n_nblk), dim3(256), shm, st, p);
    return check_launch("tcx_conv2d_h2(4x4/s2 lds-dma)");
}

template <int Wo>
int launch_q(const ConvParams& p, hipStream_t st) {
    const int ai = p.bf == 2 ? 2 : p.bf ? 1 : 0;  // b2 sources take the slim slots
    const bool rt2 = ds_rt(ai == 2, Wo) == 2 && p.HoWo % (2 * Q_TP) == 0;
    if (ai == 2) return rt2 ? launch_q_one<Wo, true, true, 2>(p, st) : launch_q_one<Wo, true, true, 1>(p, st);
    // the 32-B-slot forms stay at RT = 1: at RT = 2 they spill (255 VGPRs + 144-176 B of scratch) and the
    // headline fell from 79.2 to 64.6 images/s with it (r05_r)
    if (ai == 1) return launch_q_one<Wo, true, false, 1>(p, st);
    return launch_q_one<Wo, false, false, 1>(p, st);
}
// Wo = 128 (config 5's ds1): the slim b2 form only (the 32-B slots would not leave two workgroups per CU)
int launch_q128(const ConvParams& p, hipStream_t st) {
    static_assert(conv4s2g_lds_bytes(128, true) <= 80 * 1024 && conv4s2g_lds_bytes(128, true, 2) <= 80 * 1024,
                  "two workgroups per CU");
    const bool rt2 = ds_rt(true, 128) == 2 && p.HoWo % (2 * Q_TP) == 0;
    return rt2 ? launch_q_one<128, true, true, 2>(p, st) : launch_q_one<128, true, true, 1>(p, st);
}

}  // namespace

// Host dispatch (conv.hip): the fragment-ordered 4x4 weights exist and the shape is the U-Net's
bool conv4s2g_applies(const ConvParams& p, int cout_pad) {
    return p.wf != nullptr && p.ks == 4 && p.stride == 2 && p.pad_y == 1 && p.pad_x == 1 && p.circular &&
           p.Hi == p.H && p.Wi == p.W && (p.Wo == 16 || p.Wo == 32 || p.Wo == 64 || (p.Wo == 128 && p.bf == 2)) &&
           p.H == 2 * p.Ho &&
           p.W == 2 * p.Wo && p.HoWo % Q_TP == 0 && cout_pad % 96 == 0 && p.Cin % 8 == 0 && p.C2 == 0 &&
           p.x2 == nullptr && p.kpad == 16 * p.Cin && p.osy == 1 && p.osx == 1 && p.sc1 == nullptr &&
           !(p.cm1 && p.bf == 1) && !p.cm2;
}

int launch_conv4s2g(ConvParams& p, int cout_pad, hipStream_t st) {
    p.n_nblk = cout_pad / 96;
    if (p.M == 0) return TCX_OK;
    prof_begin(st);
    int rc;
    if (p.Wo == 32) rc = launch_q<32>(p, st);
    else if (p.Wo == 16) rc = launch_q<16>(p, st);
    else if (p.Wo == 64) rc = launch_q<64>(p, st);
    else rc = launch_q128(p, st);
    prof_end(st, 2.0 * (double)p.M * p.Cout * 16 * p.Cin);
    return rc;
}

}  // namespace tcx

using namespace tcx;

extern "C" size_t tcx_conv_weight_h2_frag4_bytes(int cout_pad, int Cin) {
    return (cout_pad % 96 == 0 && Cin % 8 == 0) ? (size_t)cout_pad * 16 * Cin * 4 : 0;
}

extern "C" int tcx_pack_conv_weight_h2_frag4(const void* wh, void* wf, int cout_pad, int kpad, int Cin, void* stream) {
    TCX_REQUIRE(wh && wf && cout_pad > 0 && cout_pad % 96 == 0 && Cin > 0 && Cin % 8 == 0 && kpad == 16 * Cin,
                "tcx_pack_conv_weight_h2_frag4: needs a 4x4 h2 weight with cout_pad %% 96 == 0, Cin %% 8 == 0");
    TCX_REQUIRE(aligned16(wh) && aligned16(wf), "tcx_pack_conv_weight_h2_frag4: 16-B alignment");
    const size_t n16 = (size_t)cout_pad * 16 * Cin * 4 / 16;
    const int blocks = (int)std::min<size_t>((n16 + 255) / 256, 4096);
    hipLaunchKernelGGL(k_pack_frag4, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const char*)wh, (char*)wf, kpad,
                       Cin, cout_pad / 96);
    return check_launch("tcx_pack_conv_weight_h2_frag4");
}
