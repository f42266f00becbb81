// k_conv3m: the U-Net's 3x3 stride-1 circular conv with h2 sources at rows of 16 / 32 / 64 pixels
// (every _ConvBlock / us*_conv conv without a GroupNorm prologue: /root/reference/src/toycrystals/
// models/sde_score_model.py:102,105,218,222) on v_mfma_f32_16x16x32_f16 instead of k_conv3lg's
// v_mfma_f32_32x32x16_f16.
//
// Why: at equal FLOPs and equal LDS bytes per FLOP the 16x16x32 loop runs 1.12x the 32x32x16 loop
// on this chip (tools/probe/mfma_shape_probe.hip, profiles/r04_b_mfma_shape.log: 1,670 vs 1,490
// TFLOP/s of f16 MFMA on random operands read from LDS; MI355X_MICROARCH.md "DVFS give-back" item 7
// measured the same for bf16): the smaller MFMA holds a higher clock under load.
//
// Same tile (256 pixels x 96 output channels, 4 waves of 64 pixels), the same LDS-DMA staging with
// split wave roles as k_conv3lg (waves 0-1 move the fragment-ordered weights, waves 2-3 the halo:
// no wave's vmcnt mixes L2 and HBM loads), the same 16-channel halo chunks (64-B h2 slots) and the
// same weight copy (tcx_pack_conv_weight_h2_frag).  What changes is the unit of work: a 32-deep
// MFMA k step is a PAIR of taps of the global tap sequence c = 9 j + t (j chunk, t tap), k = 2 q and
// 2 q + 1 — exactly the weight ring's pair — with lanes 0-31 reading tap 2q and lanes 32-63 tap
// 2q + 1 (the A operand's k = 8 (lane >> 4) + e: k blocks 0, 1 = channels 0-7, 8-15 of the first
// tap, 2, 3 of the second).  Two chunks = 18 taps = 9 pairs (q = 0..8), one of which (q = 4) pairs
// tap 8 of the even chunk with tap 0 of the odd one: the loop body is that 9-pair period with every
// lane's halo address a precomputed VGPR per pair type (aq[q]) plus an immediate per 16-pixel
// row block.
//
// Per wave: 4 row blocks (16 px) x 6 column blocks (16 channels) of 16x16 accumulators, 3 MFMAs
// (hi.lo, lo.hi, hi.hi) each per pair = 72 MFMAs per pair in two halves by column blocks 0-2 / 3-5,
// one barrier per pair between them:
//   H1: ds_read B(k, cols 3-5) -> set 1 | 36 MFMAs with A(k), B set 0
//   mid: lgkmcnt(0) [+ weight waves vmcnt(0): pair k+1 landed; halo waves at q = 3 / 8: chunk landed]
//        s_barrier; weight waves DMA pair k+2 into slot k & 1 (its B fragments are all in registers);
//        halo waves DMA a third of the next chunk when its buffer has been freed
//   H2: ds_read B(k+1, cols 0-2) -> set 0 | per row block: 9 MFMAs with B set 1, then A(k+1) of
//       that row block (its last use of A(k) has issued)
// Halo of chunk J (buffer J & 1) is issued in thirds at the mids of pairs 4, 5, 6 (even J) / 8, 0,
// 1 (odd J) of the period in which its buffer's previous chunk was last read, waited for at the
// mid of pair 8 / 3: at least one pair of latency cover after the last third, four after the first.
//
// Halo slot: 64 B = pieces [hi c0-7][lo c0-7][hi c8-15][lo c8-15] (logical 2 g + h), physical piece
// = logical ^ ((col >> 2) & 1): the A read of a ds_read_b128 lane group ({0-3,12-15,20-27} etc.:
// 16 pixels of a row block, two 8-channel groups) lands on 16 distinct 16-B bank quads at every tap
// offset (exhaustive check over the three column phases of a tap; the k_conv3lg swizzle (col >> 2) & 3
// would be 2-way here).  B reads come from the weight ring as laid out by k_conv3lg (per tap [32-col
// n][hi, lo][lane][16 B]) with a per-lane gather address (conflict-free).
#include "conv_common.hpp"

#include <type_traits>
#include <utility>

namespace tcx {
namespace {

constexpr int M_KC = 16;               // input channels per chunk
constexpr int M_NW = 4;                // waves per workgroup
constexpr int M_TP = 64 * M_NW;        // pixels per tile
constexpr int M_PAIR = 12288;          // bytes of B fragments per tap pair (2 taps x 3 x [hi, lo] x 1 KB)
constexpr int M_BN = 96;               // output channels per tile

__host__ __device__ constexpr int m_npx(int W) { return (M_TP / W + 2) * (W + 2); }
// PRO 1: + the image's GroupNorm tables [scale | shift][Cin <= 384] after the ring
template <int W, int PRO = 0>
constexpr size_t conv3m_lds_bytes() {
    return (size_t)2 * ((m_npx(W) + 15) / 16) * 16 * 64 + 2 * (size_t)M_PAIR + (PRO == 1 ? 2 * 384 * sizeof(float) : 0);
}
// PRO 1 transform units per thread: the 2 NPX 8-channel halo units of a chunk over 256 threads
__host__ __device__ constexpr int m_tu(int W) { return (2 * m_npx(W) + 255) / 256; }
// PRO 1 transform lane map (found by search over the ds_read_b128 16-lane groups and the ds_write_b128
// 8-lane groups at 16/32/64-px rows, tools/emu/conv3mg_lanemap.py: <= 1.29 / 1.18 average ways, 2
// worst): lane l takes slot 32 wv + 128 i + 2 perm[l >> 2] + (l & 1), 8-channel group (l >> 1) & 1
constexpr unsigned long long M_TPERM = 0x46dfb9a83e52701cull;  // nibble h = perm[h]

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void m_dma16(__amdgpu_buffer_rsrc_t r, char* lds, int voff, int soff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, voff, soff, 0, 0);
}
// Diagnostic timeline (tcx_debug_conv_stamps; null in production, a uniform branch): per workgroup
// [entry, prologue done, tap loop done, epilogue stores issued, exit] s_memrealtime (100 MHz), the
// s_memtime (shader clock) at entry and at loop end, and HW_ID | XCC_ID << 16, from wave 0
__device__ unsigned long long* g_m_stamps = nullptr;
__device__ int g_m_stamps_n = 0;

// PRO 1: the transform unit's tasks over the 36 MFMA gaps of a half-pair, as (gap, task) in issue
// order: task 0 load (two ds_read_b128 + the scale / shift of values 0-1), 1..8 value task - 1 part A
// (y = x sc + sh, e = exp2(-y log2 e)), 9..16 part B (y rcp(1 + e)), 17..20 the h2 split of channel
// pair task - 17, 21 the write-back (two ds_write_b128) and the range flag, 22..24 the scale / shift
// of value pair task - 21 (two ds_read_b64; the pair buffer they refill is free by then).
struct MTask {
    int gap, task;
};
// Two parts of a value back to back, one value per other gap.  Measured per layer against the
// alternatives (tools/gpu/r05f.sh, profiles/r05_f_conv.txt: up1_1 496 / 493 / 532 us, h2-source form
// 409): an exp2 pair then its reciprocals two gaps later (equal), a whole value pair per gap (bursts,
// 7 % slower), and each value's parts spread over separate gaps (r05_e: 5 % slower).  The transform's
// VALU (two quarter-rate transcendentals per value, 1.3-1.55 halo values per output pixel) is what the
// form costs over the h2-source one: without the transform tasks (a diagnostic build, wrong results)
// it runs at the h2-source form's speed (r05_c).
constexpr MTask kMSched[] = {{0, 0},   {3, 1},   {3, 9},   {4, 22},  {5, 2},   {5, 10},  {7, 17},
                             {9, 3},   {9, 11},  {10, 23}, {11, 4},  {11, 12}, {13, 18}, {15, 5},
                             {15, 13}, {16, 24}, {17, 6},  {17, 14}, {19, 19}, {21, 7},  {21, 15},
                             {23, 8},  {23, 16}, {25, 20}, {27, 21}};
constexpr const MTask* m_sched() { return kMSched; }
constexpr int M_NTASK = 25;
template <typename F, int... Is>
__device__ __forceinline__ void m_static_for(F&& f, std::integer_sequence<int, Is...>) {
    (f(std::integral_constant<int, Is>{}), ...);
}

constexpr int M_WAIT_VM0 = 0x0F70;    // s_waitcnt vmcnt(0)
constexpr int M_WAIT_LGKM0 = 0xC07F;  // s_waitcnt lgkmcnt(0)

// FAST: no activation and an fp32 output (every U-Net conv k_conv3m serves: a GroupNorm follows), so
// the epilogue is straight-line code; otherwise the activation / h2 output are run-time branches.
// PRO 1: the source is the previous conv's fp32 output and the halo is staged as
// h2(silu(x * scale[b][c] + shift[b][c])) — the GroupNorm + SiLU of the _ConvBlock feeding this conv
// (sde_score_model.py:103-107), never written to memory.  The raw fp32 chunk (16 channels = 64 B per
// pixel, the size of its h2 slot) is DMA'd into the slot image as for an h2 source, in one shot at
// the mid of pair 4 (even chunk, buffer 0) / 8 (odd, buffer 1), waited for at the mid of pair 6 / 1,
// and rewritten IN PLACE by all four waves during the next four half-pairs (6.H2, 7.H1, 7.H2, 8.H1 /
// 1.H2, 2.H1, 2.H2, 3.H1): one 8-channel unit per thread and half-pair, its two ds_read_b128, eight
// values, four channel-pair splits and two ds_write_b128 spread one task per MFMA gap over the half's
// 36 MFMAs.  It is published by the same barriers as an h2 chunk (mids 8 / 3), so the MFMA pipeline,
// the weight ring and the epilogue are k_conv3m's.
template <int W, bool FAST, int PRO>
__global__ __launch_bounds__(64 * M_NW, 2) void k_conv3m(ConvParams p) {
    constexpr int W2 = W + 2;
    constexpr int NPX = m_npx(W);
    constexpr int NI = (NPX + 15) / 16;  // halo DMA instructions per chunk (16 slots each)
    constexpr int NIH = (NI + 1) / 2;    // per halo wave (wave 2: even i, wave 3: odd i)
    constexpr int HB = NI * 16 * 64;
    constexpr int RING = 2 * HB;
    constexpr int TAB = RING + 2 * M_PAIR;  // PRO 1: [scale | shift][Cin]
    constexpr int TU = m_tu(W);             // PRO 1: transform units per thread and chunk (3 or 4)
    static_assert(W == 16 || W == 32 || W == 64, "k_conv3m: rows of 16, 32 or 64 pixels");
    static_assert(NI * 16 >= NPX + 4, "k_conv3m: idle transform lanes use 4 padding slots");
    static_assert(TU <= 4, "k_conv3m: at most 4 transform half-pairs per chunk");
    auto sw = [](int col) { return (col >> 2) & 1; };
    extern __shared__ __attribute__((aligned(16))) float sm[];
    char* const smc = reinterpret_cast<char*>(sm);
    // LDS-DMA destinations from a base the optimiser cannot fold to a constant (k_conv3lg's note)
    int lz;
    asm volatile("s_mov_b32 %0, 0" : "=s"(lz));
    char* const smd = smc + lz;
    // accumulators in VGPRs (hipcc's all-VGPR MFMA form; the AGPR form of round 4, common.hpp
    // mfma_agpr_form, measured equal and is not needed: r05_c, with the co-run and lane tests green)

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    unsigned long long* const stp = g_m_stamps;
    const bool stamp = stp != nullptr && (int)blockIdx.x < g_m_stamps_n && wv == 0;
    unsigned long long ts[7] = {};
    if (stamp) {
        ts[0] = __builtin_amdgcn_s_memrealtime();
        ts[5] = __builtin_amdgcn_s_memtime();
    }
    const int tile = xcd_remap(blockIdx.x, gridDim.x);
    const int mblk = tile / p.n_nblk;
    const int nblk = tile - mblk * p.n_nblk;
    const int m0 = mblk * M_TP, n0 = nblk * M_BN;
    const int b = m0 / p.HoWo;
    const int r0 = (m0 - b * p.HoWo) / W;
    const int bs = p.bmod > 0 ? b % p.bmod : b;
    const int H = p.H;
    const int cpt = p.Cin / M_KC;
    const int npair = 9 * cpt / 2;

    const __amdgpu_buffer_rsrc_t r1 = mk_rsrc(p.x1, p.bytes1);
    const __amdgpu_buffer_rsrc_t r2 = mk_rsrc(p.x2 ? p.x2 : p.x1, p.x2 ? p.bytes2 : p.bytes1);
    const __amdgpu_buffer_rsrc_t rw = mk_rsrc(reinterpret_cast<const float*>(p.wf), p.bytesw);

    // ---- halo DMA (waves 2, 3): lane l of instruction i fills slot 16 i + l / 4, physical piece l % 4,
    // so it reads logical piece (l % 4) ^ sw(col) of that pixel (the swizzle rides on the source address).
    // An h2 record and an fp32 chunk of 16 channels are both 64 B: the same offsets serve PRO 0 and 1
    const int hw = wv & 1;
    const int rowb = p.C1 * 4;
    const int img0 = bs * H;
    // rb: bytes per pixel of the source (C1 * 4 pixel-major; 32 in a chunk-major source's 8-channel plane);
    // ph: the byte distance of the chunk's second record (32 pixel-major; one plane chunk-major)
    auto halo_voff = [&](int i, int rb, int ph) __attribute__((always_inline)) {
        // PRO 1 at 64-px rows: recomputed at every issue (an opaque copy of the lane index keeps hipcc from
        // hoisting all 13 offsets out of the tap loop, where they spilled with the transform's registers)
        int ls = lane >> 2;
        if constexpr (PRO == 1) asm volatile("v_mov_b32 %0, %1" : "=v"(ls) : "v"(lane >> 2));
        const int hr0 = (16 * i) / W2;
        const int th = W2 * (hr0 + 1) - 16 * i;
        const int y0 = wrap_idx(r0 + hr0 - 1, H), y1 = wrap_idx(r0 + hr0, H);
        const int yo0 = (img0 + y0) * W * rb, yo1 = (img0 + y1) * W * rb;
        const bool nx = ls >= th;
        int hc = 16 * i - hr0 * W2 + ls - (nx ? W2 : 0);
        const int sl = 16 * i + ls;
        const int hcs = hc;
        if (sl >= NPX) hc = (NPX - 1) % W2;  // padding slots read a valid pixel
        const int x = hc == 0 ? W - 1 : (hc == W + 1 ? 0 : hc - 1);
        const int yo = (sl >= NPX) ? (img0 + wrap_idx(r0 + (NPX - 1) / W2 - 1, H)) * W * rb : (nx ? yo1 : yo0);
        const int pc = (lane & 3) ^ sw(hcs);
        if constexpr (PRO != 2) return yo + x * rb + 16 * pc;  // pixel-major only (rb = rowb, ph = 32)
        else return yo + x * rb + 16 * (pc & 1) + (pc >> 1) * ph;
    };
    // PRO 3: PRO 0 with an h2 output and no activation (the epilogue's h2 path straight-line)
    // PRO 2 (p.cm2): PRO 0 with source 2 chunk-major, the 16-channel chunk two planes of 32-B pixel records
    const int plane2 = PRO == 2 ? (int)(p.bytes2 / (unsigned)(p.C2 / 8)) : 0;
    // third `th` (0..2) of chunk j's halo into buffer buf
    auto halo_third = [&](int j, int buf, int th) __attribute__((always_inline)) {
        const int ci0 = j * M_KC;
        const bool s1 = ci0 < p.C1;
        const bool cm = PRO == 2 && !s1;
        const int cc = cm ? ((ci0 - p.C1) / 8) * plane2 : (s1 ? ci0 : ci0 - p.C1) * 4;
        const int rb = cm ? 32 : rowb, ph = cm ? plane2 : 32;
        const __amdgpu_buffer_rsrc_t rs = s1 ? r1 : r2;
        const int q0 = (NIH * th) / 3, q1 = (NIH * (th + 1)) / 3;
#pragma unroll
        for (int q = 0; q < NIH; ++q) {
            if (q < q0 || q >= q1) continue;
            const int i = 2 * q + hw;
            if (i < NI) m_dma16(rs, smd + buf * HB + i * 1024, halo_voff(i, rb, ph), cc);
        }
    };
    auto halo_all = [&](int j, int buf) __attribute__((always_inline)) {
#pragma unroll
        for (int t3 = 0; t3 < 3; ++t3) halo_third(j, buf, t3);
    };
    // weight pair k (12 KB) -> ring slot k & 1; wave w (0, 1) moves KB [6 w, 6 w + 6)
    auto pair_issue = [&](int k) __attribute__((always_inline)) {
        const int base = (nblk * 2 * npair + 2 * k) * 6144 + wv * 6144;
        char* const d = smd + RING + (k & 1) * M_PAIR + wv * 6144;
#pragma unroll
        for (int i = 0; i < 6; ++i) m_dma16(rw, d + i * 1024, lane * 16, base + i * 1024);
    };

    // ---- A addresses: lane (li = pixel in a 16-px row block, k block kb: g = kb & 1 channel group,
    // tap half th = kb >> 1) of row block 0 for pair type q (taps c = 2 q + th of the 18-tap period)
    const int li = lane & 15, g = (lane >> 4) & 1, th = lane >> 5;
    int aq[9];
    {
        const int mloc = wv * 64 + li;
        const int rr = mloc / W, cc = mloc % W;
#pragma unroll
        for (int q = 0; q < 9; ++q) {
            const int c = 2 * q + th;  // 0..17
            const int hb = c >= 9 ? 1 : 0;
            const int t = c - 9 * hb;
            const int dy = t / 3, dx = t - 3 * (t / 3);
            aq[q] = hb * HB + ((rr + dy) * W2 + cc + dx) * 64 + 16 * ((2 * g) ^ sw(cc + dx));
        }
    }
    // row block rb of a wave: 16 px on in the row (W = 64), half / next row (32), next row (16)
    auto rbo = [](int rb) {
        return W == 64 ? rb * 16 * 64 : (W == 32 ? (rb >> 1) * W2 * 64 + (rb & 1) * 16 * 64 : rb * W2 * 64);
    };
    // B: per-lane gather address inside a pair slot of the ring (k_conv3lg's [tap][32-col n][hi, lo][lane])
    const int bq = RING + (lane >> 5) * 6144 + ((lane >> 4) & 1) * 512 + (lane & 15) * 16;

    f32x4 acc[4][6];
#pragma unroll
    for (int rb = 0; rb < 4; ++rb)
#pragma unroll
        for (int n = 0; n < 6; ++n) acc[rb][n] = (f32x4){};
    h8 a_h[4], a_l[4], b_h[3], b_l[3];
    auto rd_a = [&](int q, int rb) __attribute__((always_inline)) {
        a_h[rb] = __builtin_bit_cast(h8, *reinterpret_cast<const float4*>(smc + aq[q] + rbo(rb)));
        a_l[rb] = __builtin_bit_cast(h8, *reinterpret_cast<const float4*>(smc + (aq[q] ^ 16) + rbo(rb)));
    };
    // B fragments (hi, lo) of pair k, column block nb, into register slot i
    auto rd_b = [&](int i, int k, int nb) __attribute__((always_inline)) {
        const char* B = smc + bq + (k & 1) * M_PAIR + (nb >> 1) * 2048 + (nb & 1) * 256;
        b_h[i] = __builtin_bit_cast(h8, *reinterpret_cast<const float4*>(B));
        b_l[i] = __builtin_bit_cast(h8, *reinterpret_cast<const float4*>(B + 1024));
    };
    // MFMA number k (0..11) of column block nb with B slot i: product k >> 2 (hi.lo, lo.hi, hi.hi) of
    // row block k & 3 (4 independent accumulators between the dependent products of one block)
    auto mfk = [&](int k, int nb, int i) __attribute__((always_inline)) {
        const int rb = k & 3, pr = k >> 2;
        acc[rb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(pr == 1 ? a_l[rb] : a_h[rb], pr == 0 ? b_l[i] : b_h[i],
                                                             acc[rb][nb], 0, 0, 0);
    };

    // ---- PRO 1 transform (in-place fp32 -> h2 of the GroupNorm + SiLU value).  Registers are the
    // limit (128 VGPRs beside the 96 accumulator AGPRs): the unit's LDS offset is recomputed per unit
    // and its scale / shift pairs are read from the LDS tables two values ahead of use
    const int t_so = 2 * (int)((M_TPERM >> (4 * (lane >> 2))) & 15ull) + (lane & 1);
    const int t_g = (lane >> 1) & 1;
    const float* const Tw = reinterpret_cast<const float*>(smc + TAB);
    int tdst = 0;        // LDS byte offset (buffer 0) of the current unit's first piece
    bool tlive = false;  // the unit is a real halo slot (idle lanes rewrite a padding slot)
    int tj = 0;          // chunk being transformed
    float ux[8];
    f32x2 tsc[2], tsh[2];  // scale / shift of two values, double-buffered by value pair
    unsigned uh[4], ul[4];
    float um = 0.f;
    typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
    auto t_addr = [&](int i) __attribute__((always_inline)) {
        const int sl0 = 128 * i + 32 * wv + t_so;
        tlive = sl0 < NPX;
        const int sl = tlive ? sl0 : NPX + (lane & 3);
        tdst = sl * 64 + 16 * ((2 * t_g) ^ sw(sl % W2));
    };
    auto t_tab = [&](int q) __attribute__((always_inline)) {  // channels 2 q, 2 q + 1 of the lane's group
        const float* t = Tw + tj * M_KC + 8 * t_g + 2 * q;
        tsc[q & 1] = *reinterpret_cast<const f32x2*>(t);
        tsh[q & 1] = *reinterpret_cast<const f32x2*>(t + p.C1);
    };
    // the unit's LDS reads / writes as inline asm: the compiler counts every C++ LDS read after an
    // LDS-DMA issue as a possible alias of the DMA and waits for vmcnt(0) first (it stalled the weight
    // waves on the pair they had just issued, one L2 round trip per transform half); the halo buffer a
    // unit rewrites is never a DMA target while it is transformed (the raw chunk landed at the previous
    // mid), so the reads need only lgkmcnt, which t_val 0's explicit wait provides
    const int lds_base = (int)(size_t)((__attribute__((address_space(3))) char*)smc);
    auto lds_rd16 = [&](int a) __attribute__((always_inline)) {
        f32x4 v;
        asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(a));
        return v;
    };
    auto lds_wr16 = [&](int a, u32x4 v) __attribute__((always_inline)) {
        asm volatile("ds_write_b128 %0, %1" : : "v"(a), "v"(v) : "memory");
    };
    auto t_load = [&](int i, int buf) __attribute__((always_inline)) {
        t_addr(i);
        const int lb = lds_base + buf * HB;
        const f32x4 x0 = lds_rd16(lb + tdst);
        const f32x4 x1 = lds_rd16(lb + (tdst ^ 16));
        ux[0] = x0[0]; ux[1] = x0[1]; ux[2] = x0[2]; ux[3] = x0[3]; ux[4] = x1[0]; ux[5] = x1[1]; ux[6] = x1[2]; ux[7] = x1[3];
        um = 0.f;
        t_tab(0);
    };
    float ue[2];  // exp2 of value k between its parts A and B
    auto t_valA = [&](int k) __attribute__((always_inline)) {
        if (k == 0) __builtin_amdgcn_s_waitcnt(M_WAIT_LGKM0);  // the unit's asm reads (t_load)
        const int q = k >> 1, e = k & 1;
        ux[k] = fmaf(ux[k], tsc[q & 1][e], tsh[q & 1][e]);  // u = -log2(e) t (the tables' staging)
        ue[k & 1] = __builtin_amdgcn_exp2f(ux[k]);
    };
    auto t_valB = [&](int k) __attribute__((always_inline)) { ux[k] = ux[k] * __builtin_amdgcn_rcpf(1.0f + ue[k & 1]); };
    auto t_val = [&](int k) __attribute__((always_inline)) {
        t_valA(k);
        t_valB(k);
    };
    auto t_pair = [&](int q) __attribute__((always_inline)) {
        const f32x2 v = {ux[2 * q], ux[2 * q + 1]};
        const f16x2 h = __builtin_convertvector(v, f16x2);
        const f32x2 r = v - __builtin_convertvector(h, f32x2);
        const f16x2 l = __builtin_convertvector(r, f16x2);
        uh[q] = __builtin_bit_cast(unsigned, h);
        ul[q] = __builtin_bit_cast(unsigned, l);
        um = fmaxf(um, fmaxf(fabsf(v[0]), fabsf(v[1])));
    };
    auto t_store = [&](int buf, bool live) __attribute__((always_inline)) {
        const int lb = lds_base + buf * HB;
        lds_wr16(lb + tdst, (u32x4){uh[0], uh[1], uh[2], uh[3]});
        lds_wr16(lb + (tdst ^ 16), (u32x4){ul[0], ul[1], ul[2], ul[3]});
        h2_flag(p.ovf, !(um < kH2Max) && live && tlive);
    };
    // one task (m_tcode) of a transform unit
    auto t_task = [&](auto Cc, int U, int buf, bool live) __attribute__((always_inline)) {
        constexpr int code = decltype(Cc)::value;
        if constexpr (code == 0) t_load(U, buf);
        else if constexpr (code <= 8) t_valA(code - 1);
        else if constexpr (code <= 16) t_valB(code - 9);
        else if constexpr (code <= 20) t_pair(code - 17);
        else if constexpr (code == 21) t_store(buf, live);
        else t_tab(code - 21);  // 22..24: tables of value pair 1..3
    };
    // the tasks scheduled into MFMA gap G (m_sched order), fenced by sched barriers
    auto t_gap = [&](auto Gc, int U, int buf, bool live) __attribute__((always_inline)) {
        constexpr int G = decltype(Gc)::value;
        constexpr bool any = [] {
            for (int e = 0; e < M_NTASK; ++e)
                if (m_sched()[e].gap == G) return true;
            return false;
        }();
        if constexpr (any) {
            __builtin_amdgcn_sched_barrier(0);
            m_static_for([&](auto E) {
                constexpr int e = decltype(E)::value;
                if constexpr (m_sched()[e].gap == G)
                    t_task(std::integral_constant<int, m_sched()[e].task>{}, U, buf, live);
            }, std::make_integer_sequence<int, M_NTASK>{});
            __builtin_amdgcn_sched_barrier(0);
        }
    };

    // ---- prologue: pairs 0, 1 and halo chunk 0 in LDS; the first third of chunk 1 issued
    // (PRO 1: chunk 0 raw + the image's tables, then chunk 1 raw in full while chunk 0 is transformed)
    if (wv < 2) {
        pair_issue(0);
        pair_issue(1);
    } else {
        halo_all(0, 0);
    }
    if constexpr (PRO == 1) {
        float* const Twr = reinterpret_cast<float*>(smc + TAB);
        // staged as -log2(e) * (scale, shift): the transform's fma gives u = -log2(e) t (t the GroupNorm
        // value), exp2(u) = e^-t directly, and it stages u / (1 + e^-t) = -log2(e) silu(t); the constant
        // factor of every input of this single-source conv comes out in the epilogue (wscale * -ln 2).
        // One multiply per value fewer than the t-based form, no register for a constant
        for (int c = tid; c < p.C1; c += 64 * M_NW) {
            Twr[c] = -1.4426950408889634f * p.sc1[(size_t)b * p.C1 + c];
            Twr[p.C1 + c] = -1.4426950408889634f * p.sh1[(size_t)b * p.C1 + c];
        }
    }
    __builtin_amdgcn_s_waitcnt(M_WAIT_VM0);
    __builtin_amdgcn_s_waitcnt(M_WAIT_LGKM0);
    __builtin_amdgcn_s_barrier();
    if (stamp) ts[1] = __builtin_amdgcn_s_memrealtime();
    if constexpr (PRO == 1) {
        if (wv >= 2) halo_all(1, 1);  // cpt >= 2
        tj = 0;
#pragma unroll
        for (int i = 0; i < TU; ++i) {
            t_load(i, 0);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                if (q < 3) t_tab(q + 1);
                t_val(2 * q);
                t_val(2 * q + 1);
                t_pair(q);
            }
            t_store(0, true);
        }
        __builtin_amdgcn_s_waitcnt(M_WAIT_LGKM0);
        __builtin_amdgcn_s_barrier();
    } else {
        if (wv >= 2 && cpt > 1) halo_third(1, 1, 0);
    }
#pragma unroll
    for (int rb = 0; rb < 4; ++rb) rd_a(0, rb);
#pragma unroll
    for (int i = 0; i < 3; ++i) rd_b(i, 0, i);

    // the 12 MFMAs of column block nb (B slot i) as gaps G0 .. G0 + 11 of a half-pair, each followed
    // by its transform task when the half carries unit U (U < 0: none) of buffer BUF, chunk live `tl`
    auto mf_col = [&](int nb, int i, auto G0c, auto Uc, auto BUFc, bool tl) __attribute__((always_inline)) {
        constexpr int G0 = decltype(G0c)::value, U = decltype(Uc)::value, BUF = decltype(BUFc)::value;
        m_static_for([&](auto K) {
            constexpr int k = decltype(K)::value;
            mfk(k, nb, i);
            if constexpr (U >= 0) t_gap(std::integral_constant<int, G0 + k>{}, U, BUF, tl);
        }, std::make_integer_sequence<int, 12>{});
    };
    // the 3 MFMAs of row block rb, column block nb (B slot i) as gaps G0 .. G0 + 2
    auto mf3 = [&](int rb, int nb, int i, auto G0c, auto Uc, auto BUFc, bool tl) __attribute__((always_inline)) {
        constexpr int G0 = decltype(G0c)::value, U = decltype(Uc)::value, BUF = decltype(BUFc)::value;
        m_static_for([&](auto K) {
            constexpr int pr = decltype(K)::value;
            mfk(4 * pr + rb, nb, i);
            if constexpr (U >= 0) t_gap(std::integral_constant<int, G0 + pr>{}, U, BUF, tl);
        }, std::make_integer_sequence<int, 3>{});
    };

    auto pair_iter = [&](int pp, auto Q) __attribute__((always_inline)) {
        constexpr int q = decltype(Q)::value;
        constexpr int qn = q == 8 ? 0 : q + 1;
        const int k = 9 * pp + q;
        // PRO 1 transform units of this pair's two halves: odd chunk 2 pp + 1 (buffer 1) in 1.H2, 2.H1,
        // 2.H2, 3.H1; even chunk 2 pp + 2 (buffer 0) in 6.H2, 7.H1, 7.H2, 8.H1 (the first TU of them)
        constexpr int U1 = PRO != 1 ? -1 : (q == 2 ? 1 : q == 3 ? 3 : q == 7 ? 1 : q == 8 ? 3 : -1);
        constexpr int U2 = PRO != 1 ? -1 : (q == 1 ? 0 : q == 2 ? 2 : q == 6 ? 0 : q == 7 ? 2 : -1);
        constexpr int UH1 = U1 < TU ? U1 : -1, UH2 = U2 < TU ? U2 : -1;
        constexpr int BUF = q <= 4 ? 1 : 0;
        const bool tl = BUF == 1 ? true : 2 * pp + 2 < cpt;  // the even chunk after the last is not staged
        using Uh1 = std::integral_constant<int, UH1>;
        using Uh2 = std::integral_constant<int, UH2>;
        using Bc = std::integral_constant<int, BUF>;
        if constexpr (UH1 >= 0 || UH2 >= 0) tj = BUF == 1 ? 2 * pp + 1 : 2 * pp + 2;  // chunk being transformed
        // H1: column blocks 0-2 (B slots 0-2); each slot, once its 12 MFMAs have issued, takes block 3 + i
        mf_col(0, 0, std::integral_constant<int, 0>{}, Uh1{}, Bc{}, tl);
        __builtin_amdgcn_sched_barrier(0);
        rd_b(0, k, 3);
        __builtin_amdgcn_sched_barrier(0);
        mf_col(1, 1, std::integral_constant<int, 12>{}, Uh1{}, Bc{}, tl);
        __builtin_amdgcn_sched_barrier(0);
        rd_b(1, k, 4);
        __builtin_amdgcn_sched_barrier(0);
        mf_col(2, 2, std::integral_constant<int, 24>{}, Uh1{}, Bc{}, tl);
        __builtin_amdgcn_sched_barrier(0);
        rd_b(2, k, 5);
        __builtin_amdgcn_sched_barrier(0);
        // mid: every wave's ring reads of pair k done; pair k+1 (weights) / a halo chunk published
        // (PRO 1: the raw chunk landed at mids 1 / 6, the transformed one published at 3 / 8)
        __builtin_amdgcn_s_waitcnt(M_WAIT_LGKM0);
        constexpr bool halo_wait = PRO == 1 ? (q == 1 || q == 6) : (q == 3 || q == 8);
        if (wv < 2 || halo_wait) __builtin_amdgcn_s_waitcnt(M_WAIT_VM0);
        __builtin_amdgcn_s_barrier();
        if (wv < 2) {
            if (k + 2 < npair) pair_issue(k + 2);
        } else if constexpr (PRO == 1) {
            // (the raw chunk in two parts over mids 4-5 / 8-0 measured no faster: r05_c)
            if constexpr (q == 4) {     // chunk 2 pp + 2 -> buffer 0 (chunk 2 pp was last read by pair 4)
                if (2 * pp + 2 < cpt) halo_all(2 * pp + 2, 0);
            } else if constexpr (q == 8) {     // chunk 2 pp + 3 -> buffer 1 (chunk 2 pp + 1 last read by pair 8)
                if (2 * pp + 3 < cpt) halo_all(2 * pp + 3, 1);
            }
        } else {
            if constexpr (q >= 4 && q <= 6) {  // chunk 2 pp + 2 -> buffer 0 (chunk 2 pp was last read by pair 4)
                if (2 * pp + 2 < cpt) halo_third(2 * pp + 2, 0, q - 4);
            } else if constexpr (q == 8) {     // chunk 2 pp + 3 -> buffer 1 (chunk 2 pp + 1 last read by pair 8)
                if (2 * pp + 3 < cpt) halo_third(2 * pp + 3, 1, 0);
            } else if constexpr (q <= 1) {     // the rest of chunk 2 pp + 1 (its first third: pair 8 before)
                if (2 * pp + 1 < cpt) halo_third(2 * pp + 1, 1, q + 1);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        // H2: column blocks 3-5; slots 0, 1 then take B(k+1) blocks 0, 1; block 5 runs row block by row
        // block so that A(k+1) of each row block is read right after its last use of A(k), then slot 2
        // takes B(k+1) block 2
        mf_col(3, 0, std::integral_constant<int, 0>{}, Uh2{}, Bc{}, tl);
        __builtin_amdgcn_sched_barrier(0);
        rd_b(0, k + 1, 0);
        __builtin_amdgcn_sched_barrier(0);
        mf_col(4, 1, std::integral_constant<int, 12>{}, Uh2{}, Bc{}, tl);
        __builtin_amdgcn_sched_barrier(0);
        rd_b(1, k + 1, 1);
        __builtin_amdgcn_sched_barrier(0);
        m_static_for([&](auto RB) {
            constexpr int rb = decltype(RB)::value;
            mf3(rb, 5, 2, std::integral_constant<int, 24 + 3 * rb>{}, Uh2{}, Bc{}, tl);
            __builtin_amdgcn_sched_barrier(0);
            rd_a(qn, rb);
            __builtin_amdgcn_sched_barrier(0);
        }, std::make_integer_sequence<int, 4>{});
        rd_b(2, k + 1, 2);
        __builtin_amdgcn_sched_barrier(0);
    };
    for (int pp = 0; pp < cpt / 2; ++pp) {
        pair_iter(pp, std::integral_constant<int, 0>{});
        pair_iter(pp, std::integral_constant<int, 1>{});
        pair_iter(pp, std::integral_constant<int, 2>{});
        pair_iter(pp, std::integral_constant<int, 3>{});
        pair_iter(pp, std::integral_constant<int, 4>{});
        pair_iter(pp, std::integral_constant<int, 5>{});
        pair_iter(pp, std::integral_constant<int, 6>{});
        pair_iter(pp, std::integral_constant<int, 7>{});
        pair_iter(pp, std::integral_constant<int, 8>{});
    }

    if (stamp) {
        ts[2] = __builtin_amdgcn_s_memrealtime();
        ts[6] = __builtin_amdgcn_s_memtime();
    }
    __builtin_amdgcn_s_waitcnt(M_WAIT_VM0);
    __syncthreads();  // LDS -> epilogue reduction scratch

    // ---- epilogue (the fast path of conv_common.hpp for the 16x16 accumulator layout: lane l holds
    // column l & 15 of each 16x16 block, rows 4 (l >> 4) .. + 3): bias, activation, fp64 GroupNorm
    // partials per 128-pixel group (waves 0-1, 2-3) from the columns, then a 4x4 quad transpose
    // (quad_transpose4) so that lane l holds row 4 (l >> 4) + (l & 3) of 4 consecutive channels
    // 4 ((l & 15) >> 2) .. + 3: one 16-B store per lane and block (fp32), or the 8-B hi and lo
    // halves of the pixel's h2 record
    double* red = reinterpret_cast<double*>(sm);
    {
        const int col = lane & 15, rg = lane >> 4, qi = lane & 3, qc = col >> 2;
        // PRO 1: the staged inputs are -log2(e) silu(.) (the transform's tables)
        const float wsc = PRO == 1 ? *p.wscale * -0.6931471805599453f : *p.wscale;
        const __amdgpu_buffer_rsrc_t ry = mk_rsrc(p.y, (unsigned)((long long)p.M * p.Cout * 4));
        const int rowo = p.Cout * 4;
        const int pixq = m0 + 64 * wv + 4 * rg + qi;  // this lane's pixel after the transpose (row block 0)
        const int vo32 = (pixq * p.Cout + n0 + 4 * qc) * 4;
        const int voh = pixq * rowo + (n0 + 4 * qc) / 8 * 32 + (qc & 1) * 8;
        // every load before the first store: vmcnt counts loads and stores in order, so a load issued
        // after a store would wait for that store's acknowledgement
        float bcs[6];
#pragma unroll
        for (int nb = 0; nb < 6; ++nb) bcs[nb] = p.bias ? p.bias[n0 + 16 * nb + col] : 0.f;
#pragma unroll
        for (int nb = 0; nb < 6; ++nb) {
            const float bc = bcs[nb];
            float s = 0.f, ss = 0.f;
            bool bad = false;
#pragma unroll
            for (int rb = 0; rb < 4; ++rb) {
                float v[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    float x = fmaf(acc[rb][nb][r], wsc, bc);
                    if constexpr (!FAST) {
                        if (p.act == 1) x = fmaxf(x, 0.f);
                        else if (p.act == 2) x = 1.f / (1.f + expf(-x));
                        else if (p.act == 3) x = silu_f(x);
                    }
                    v[r] = x;
                    s += x;
                    ss = fmaf(x, x, ss);
                }
                quad_transpose4(v, qi);
                const int so = (16 * rb * p.Cout + 16 * nb) * 4;
                if ((!FAST && p.out_h2) || PRO == 3) {
                    const unsigned a0 = split1(v[0]), a1 = split1(v[1]), a2 = split1(v[2]), a3 = split1(v[3]);
                    const unsigned hi0 = (a0 & 0xffffu) | (a1 << 16), hi1 = (a2 & 0xffffu) | (a3 << 16);
                    const unsigned lo0 = (a0 >> 16) | (a1 & 0xffff0000u), lo1 = (a2 >> 16) | (a3 & 0xffff0000u);
                    const int sh = (16 * rb * p.Cout + 16 * nb) * 4;  // 16 channels = two whole records
                    if (p.h2pair) {
                        store_h2_pair((u32x2_h2){hi0, hi1}, (u32x2_h2){lo0, lo1}, (qc & 1) != 0, ry,
                                      voh - (qc & 1) * 8, sh);
                    } else {
                        __builtin_amdgcn_raw_buffer_store_b64((u32x2){hi0, hi1}, ry, voh, sh, 0);
                        __builtin_amdgcn_raw_buffer_store_b64((u32x2){lo0, lo1}, ry, voh + 16, sh, 0);
                    }
                    bad = bad || h2_bad(v[0]) || h2_bad(v[1]) || h2_bad(v[2]) || h2_bad(v[3]);
                } else {
                    store_b128_guarded(__builtin_bit_cast(u32x4, make_float4(v[0], v[1], v[2], v[3])), ry, vo32, so);
                }
            }
            if constexpr (!FAST || PRO == 3) h2_flag(p.ovf, bad);
            if (p.gn) {
                double ds = (double)s, dss = (double)ss;
                ds += __shfl_xor(ds, 16);
                dss += __shfl_xor(dss, 16);
                ds += __shfl_xor(ds, 32);
                dss += __shfl_xor(dss, 32);
                if (rg == 0) {
                    red[(wv * M_BN + 16 * nb + col) * 2 + 0] = ds;
                    red[(wv * M_BN + 16 * nb + col) * 2 + 1] = dss;
                }
            }
        }
    }
    if (stamp) ts[3] = __builtin_amdgcn_s_memrealtime();
    if (p.gn) {
        __syncthreads();
        for (int e = tid; e < 2 * M_BN; e += 64 * M_NW) {
            const int gi = e / M_BN, cl = e - gi * M_BN;
            const int co = n0 + cl;
            const double s = red[((2 * gi) * M_BN + cl) * 2 + 0] + red[((2 * gi + 1) * M_BN + cl) * 2 + 0];
            const double ss = red[((2 * gi) * M_BN + cl) * 2 + 1] + red[((2 * gi + 1) * M_BN + cl) * 2 + 1];
            const int mg = m0 + 128 * gi;
            const int bb = mg / p.HoWo;
            const int split = (mg - bb * p.HoWo) / 128;
            double* dst = p.gn + (((size_t)bb * p.nsplit + split) * p.Cout + co) * 2;
            dst[0] = s;
            dst[1] = ss;
        }
    }
    if (stamp) {  // vector stores from lanes 0..7 of wave 0
        const unsigned long long t4 = __builtin_amdgcn_s_memrealtime();
        const unsigned hw = __builtin_amdgcn_s_getreg(0xF804) & 0xffffu;  // HW_ID
        const unsigned xcc = __builtin_amdgcn_s_getreg(0xF814) & 0xffffu; // XCC_ID
        unsigned long long v = lane == 0 ? ts[0] : lane == 1 ? ts[1] : lane == 2 ? ts[2] : lane == 3 ? ts[3]
                             : lane == 4 ? t4 : lane == 5 ? ts[5] : lane == 6 ? ts[6]
                             : ((unsigned long long)hw | ((unsigned long long)xcc << 16));
        if (lane < 8) stp[(size_t)blockIdx.x * 8 + lane] = v;
    }
}

// TCX_CONV3M_OH2=0: h2-output convs on the generic epilogue (FAST false) instead of PRO 3 (A/B)
bool conv3m_oh2_enabled() {
    static const bool on = [] {
        const char* e = getenv("TCX_CONV3M_OH2");
        return !(e && e[0] == '0');
    }();
    return on;
}

template <int W>
int launch3m(const ConvParams& p, hipStream_t st) {
    static bool attr[5] = {};
    const bool pro = p.sc1 != nullptr;
    const bool fast = p.act == 0 && !p.out_h2;
    const bool oh2 = p.act == 0 && p.out_h2 && !p.cm2 && conv3m_oh2_enabled();  // PRO 3: h2 output, no act
    const int ai = pro ? 2 : p.cm2 ? 3 : oh2 ? 4 : (int)fast;
    void (*const k)(ConvParams) = pro ? &k_conv3m<W, true, 1>
                                  : p.cm2 ? &k_conv3m<W, true, 2>
                                  : oh2 ? &k_conv3m<W, true, 3>
                                  : fast ? &k_conv3m<W, true, 0> : &k_conv3m<W, false, 0>;
    const size_t lds = pro ? conv3m_lds_bytes<W, 1>() : conv3m_lds_bytes<W, 0>();
    if (!attr[ai]) {
        if (hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) !=
            hipSuccess) {
            set_error("tcx_conv2d_h2: cannot enable %zu B of dynamic LDS", lds);
            return TCX_EHIP;
        }
        attr[ai] = true;
    }
    const int grid = (p.M / M_TP) * p.n_nblk;
    hipLaunchKernelGGL(k, dim3(grid), dim3(64 * M_NW), lds, st, p);
    return check_launch("tcx_conv2d_h2(3x3 16x16x32)");
}

}  // namespace

// Default for the h2-source 3x3 convs it covers (round 4).  It had been opt-in: with other kernels
// sharing its CUs a few 16x16 blocks per launch got one wrong channel.  The cause was the store-data
// hazard of its quad epilogue (a 16-B store's first data VGPR rewritten across an if/else join with no
// wait state, conv_common.hpp store_b128_guarded), not the MFMA / ds_read order: with the pad, the
// co-run and sampler probes are deterministic (profiles/r04_m2_*), and since round 5 also without the
// AGPR accumulator form (tests/test_gpu_headline.py co-run repeats, profiles/r05_c_*).

// TCX_CONV3MG=0 keeps the GroupNorm-prologue convs on k_conv3lg / k_conv3g (A/B measurements)
bool conv3mg_enabled() {
    static const bool on = [] {
        const char* e = getenv("TCX_CONV3MG");
        return !(e && e[0] == '0');
    }();
    return on;
}

// called by launch_conv3l: k_conv3lg's conditions plus the fast epilogue's (dense NHWC fp32 / h2 output,
// no per-batch bias or residual, 32-bit offsets); h2 sources (PRO 0), or ONE fp32 source with its
// GroupNorm+SiLU tables and an fp32 output (PRO 1)
bool conv3m_takes(const ConvParams& p) {
    const bool pro = p.sc1 != nullptr;
    if (pro && (!conv3mg_enabled() || p.C2 != 0 || p.act != 0 || p.out_h2 || p.sh1 == nullptr)) return false;
    // chunk-major: source 2 of the h2 form (PRO 2), fp32 output, no activation
    if (p.cm1 || (p.cm2 && (pro || p.C2 % 16 != 0 || p.act != 0 || p.out_h2))) return false;
    return !p.bf && p.circular && !(p.C2 > 0 && p.sc2 != nullptr) &&
           (p.W == 16 || p.W == 32 || p.W == 64) && p.M % M_TP == 0 && p.HoWo % M_TP == 0 && p.Cin % 32 == 0 &&
           p.Cin <= 384 && p.Cout % M_BN == 0 && p.osy == 1 && p.osx == 1 && p.bias_b == nullptr &&
           p.resid == nullptr && (long long)p.M * p.Cout < (1ll << 29) && p.wscale != nullptr;
}

extern "C" int tcx_debug_conv_stamps(void* buf, int n) {
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_m_stamps), &buf, sizeof(buf)) != hipSuccess ||
        hipMemcpyToSymbol(HIP_SYMBOL(g_m_stamps_n), &n, sizeof(n)) != hipSuccess) {
        set_error("tcx_debug_conv_stamps: hipMemcpyToSymbol failed");
        return TCX_EHIP;
    }
    return TCX_OK;
}

int launch_conv3m(const ConvParams& p, hipStream_t st) {
    if (p.W == 64) return launch3m<64>(p, st);
    if (p.W == 32) return launch3m<32>(p, st);
    return launch3m<16>(p, st);
}

}  // namespace tcx
