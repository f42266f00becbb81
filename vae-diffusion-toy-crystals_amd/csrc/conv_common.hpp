// Shared pieces of the implicit-GEMM conv kernels (conv.hip: k_conv, conv3h.hip: k_conv3h):
// parameters, raw-buffer helpers and the fused epilogue.
#pragma once
#include "common.hpp"
#include "h2.hpp"

namespace tcx {

struct ConvParams {
    const float* x1;
    const float* x2;
    int C1, C2, Cin;
    int bmod, H, W;    // source image dims (pre-upsample)
    int Hi, Wi;        // im2col input dims (2H,2W when upsampling)
    int Ho, Wo, HoWo, M;
    const float* w;
    const float* bias;
    const float* bias_b;
    const float* resid;
    float* y;
    int Cout, kpad, nchunks;
    int ks, stride, pad_y, pad_x, circular;
    // output placement (sub-pixel phases of a transposed conv): row = oy*osy + ooy
    int Hy, Wy, osy, ooy, osx, oox;
    int act;       // 0 none, 1 relu, 2 sigmoid, 3 silu
    double* gn;    // [Bt][nsplit][Cout][2] or null
    int nsplit;
    int n_nblk;
    // GroupNorm+SiLU prologue of each source: x -> silu(x * scale[b][c] + shift[b][c]) applied
    // when the staged chunk is written to LDS (tables from tcx_gn_finalize; null = raw source)
    const float *sc1, *sh1, *sc2, *sh2;
    unsigned bytes1, bytes2, bytesw;  // buffer extents for the MODE 3 raw-buffer loads
    // f16x3 path (SPL): sources and weights in the h2 split format (h2.hpp), *wscale = 2^-e
    // undoes the weights' power-of-two scale; out_h2 writes the output in h2 (ovf: range flag)
    const float* wscale;
    int out_h2;
    unsigned* ovf;
    // fragment-ordered copy of the h2 weights (tcx_pack_conv_weight_h2_frag) or null: k_conv3g only
    const void* wf;
    // bf16 single-product mode (h2.hpp): the records hold bf16 halves, weights unscaled, one
    // v_mfma_f32_32x32x16_bf16 (hi x hi) per product instead of three f16 ones
    int bf;
    // chunk-major h2 sources (round 5): [C/8][B][H][W][32 B], one plane of h2 records per 8 channels,
    // read by k_conv4s2g (source 1) and k_conv3m (source 2) only
    int cm1, cm2;
    // h2 outputs as one 16-B store per lane pair half (store_h2_pair; TCX_H2_PAIR=0: two 8-B stores)
    int h2pair;
    // quad epilogue with the output form compiled in (conv_epi_store_quad OUT; TCX_EPI_STATIC=0: run time)
    int epi_static;
};

// Halo-staged 3x3 kernel (conv3h.hip): applicability test and launcher for tcx_conv2d_h2.
bool conv3h_applies(const ConvParams& p, int cout_pad);
int launch_conv3h(ConvParams& p, int cout_pad, hipStream_t st);
// 512-pixel-tile 3x3 kernel with the GroupNorm+SiLU prologue (conv3g.hip): rows W >= 32.
bool conv3g_applies(const ConvParams& p, int cout_pad);
// true when a 3x3 stride-1 circular conv of an H x W image with Cin inputs runs on k_conv3g (and so
// can take the GroupNorm+SiLU prologue of tcx_conv2d_h2_pro)
bool conv3g_covers(int H, int W, int Cin, int cout_pad, bool bf = false);
int launch_conv3g(ConvParams& p, int cout_pad, hipStream_t st);
// bf16 LDS-DMA 3x3 kernel (conv3lb.hip): config 5's rows of 64 / 128 / 256 px.
bool conv3lb_takes(const ConvParams& p);
// 1x1 split GEMM (lin1x1.hip): the attention block's qkv / proj convs.
bool lin1x1_applies(const ConvParams& p, int cout_pad);
int launch_lin1x1(ConvParams& p, int cout_pad, hipStream_t st);
// LDS-DMA 4x4 stride-2 kernel (conv4s2g.hip): the U-Net downsamples with fragment-ordered weights.
bool conv4s2g_applies(const ConvParams& p, int cout_pad);
int launch_conv4s2g(ConvParams& p, int cout_pad, hipStream_t st);
// Halo-staged 4x4 stride-2 kernel (conv4s2h.hip): the U-Net downsamples on the split path.
bool conv4s2h_applies(const ConvParams& p, int cout_pad);
int launch_conv4s2h(ConvParams& p, int cout_pad, hipStream_t st);

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

// 16 zero bytes: masked-out im2col elements load from here (an address select, not a value
// select after the load, which hipcc lowers through scratch memory).
__device__ __attribute__((aligned(16))) float g_zero4[4] = {0.f, 0.f, 0.f, 0.f};

constexpr int BM = 128;
constexpr int BK = 32;
constexpr int LDA = 36;  // padded LDS row (floats)



constexpr int PRO_MAXC = 384;  // max channels per source for the fused GN prologue

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
// Raw buffer load (32-bit byte offset, hardware range check: an offset past num_records reads 0)
__device__ __forceinline__ float4 bld4(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
    return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t mk_rsrc(const float* p, unsigned bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), 0, (int)bytes, 0x00020000);
}
// 0x80000000: beyond every num_records (extents are < 2^31) with or without the SGPR offset
// added, and no 32-bit wrap -> the load returns zeros
constexpr int kOOB = (int)0x80000000u;
constexpr int MAXTAP = 16;  // MODE 3 offset table: up to 4x4 kernels

__device__ __forceinline__ float4 f4_fma(float s, float4 a, float4 acc) {
    return make_float4(fmaf(s, a.x, acc.x), fmaf(s, a.y, acc.y), fmaf(s, a.z, acc.z), fmaf(s, a.w, acc.w));
}

// Bilinear x2 (align_corners=False) tap: mirrors ATen's upsample_bilinear2d CPU kernel:
// src = 0.5*(d+0.5)-0.5 clamped at 0, i1 = i0 + (i0 < n-1), l1 = src - i0, l0 = 1 - l1,
// out = l0y*(l0x*a00 + l1x*a01) + l1y*(l0x*a10 + l1x*a11).
__device__ __forceinline__ void bilin_axis(int d, int n, int& i0, int& i1, float& l0, float& l1) {
    float s = 0.5f * ((float)d + 0.5f) - 0.5f;
    s = s < 0.f ? 0.f : s;
    i0 = (int)s;
    i1 = i0 + (i0 < n - 1 ? 1 : 0);
    l1 = s - (float)i0;
    l0 = 1.f - l1;
}

// Fast path (every U-Net conv): dense NHWC output, whole tiles inside one image, no per-batch bias,
// output columns all valid, 32-bit element offsets.  Every load (weight scale, bias, residual) is
// issued before the first store: on gfx950 one counter (vmcnt) tracks loads AND stores, so a load
// after a store makes the wave wait until that store is acknowledged (the round-1 form loaded the
// bias per 32-channel tile after the previous tile's 16 stores: 2-3 % of a 64^2 launch).  Stores go
// through a buffer resource with the wave-uniform row offset in soffset, and the scale/bias and
// GroupNorm sums run on packed fp32 pairs (v_pk_fma_f32), to keep the epilogue's VALU small.
// RT row blocks of 32 pixels per wave (wave wv owns virtual waves wv0 .. wv0 + RT - 1).
template <int NT, int SPL, int NW, int RT>
__device__ __forceinline__ bool conv_epi_fast(const ConvParams& p, int m0) {
    constexpr int BN = 32 * NT;
    return p.osy == 1 && p.osx == 1 && p.bias_b == nullptr && p.M % (32 * NW) == 0 && p.HoWo % (32 * NW) == 0 &&
           p.Cout % BN == 0 && (long long)p.M * p.Cout < (1ll << 29);
}

typedef float f32x2 __attribute__((ext_vector_type(2)));

// A VMEM store of more than 8 bytes reads its data VGPRs after it issues, so a VALU write to those
// VGPRs must not follow it directly.  hipcc pads that hazard inside a basic block but not across the
// join of an if / else whose branch ends in the store: the next block's first instruction rewrote
// the store's first dword with no wait state, and the stored value was the old or the new one at
// random — the bf16 quad-epilogue nondeterminism (one dword per 32 x 32 block: rt 0, n 1, rows
// 24-31, channels 12 / 28, tools/lbbench.py WHERE=1, profiles/r04_lbwhere.log) and k_conv3m's
// co-run differences (45 such sites).  Every 16-B epilogue store goes through this: a sched_barrier
// keeps the scheduler from moving the overwrite above the s_nop.  tools/store_hazard_check.py scans
// the assembly for the pattern (0 sites at HEAD).
// AUX: the store's cache policy.  EPI_NT (non-temporal) for the bf16 convs' fp32 output, which at 256^2
// (1.1 GB per launch) leaves the caches long before the apply pass reads it: k_conv3lb 64-px rows
// 136-141 -> 124-125 us, 256-px rows 827-838 -> 787-822 us, config 5 7.00-7.02 -> 7.07-7.08 images/s
// (profiles/r04_nt_*, alternating libraries in one call).
constexpr int EPI_NT = 2;
template <int AUX = 0>
__device__ __forceinline__ void store_b128_guarded(u32x4 v, __amdgpu_buffer_rsrc_t r, int voff, int soff) {
    __builtin_amdgcn_raw_buffer_store_b128(v, r, voff, soff, AUX);
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_nop 1");
    __builtin_amdgcn_sched_barrier(0);
}

// Store of one lane's 4 channels of an h2 record (hi, lo: 8 B each) after quad_transpose4, where lane ^ 4
// holds the record's other 4 channels: the lanes swap 8 B (ds_swizzle, xor 4) so the even lane (`odd`
// false) stores the record's 16-B hi half and the odd lane its lo half — one 16-B store per lane, the fp32
// output's instruction count, instead of two 8-B stores.  vrec: byte offset of the record.
typedef unsigned int u32x2_h2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void store_h2_pair(u32x2_h2 hi, u32x2_h2 lo, bool odd, __amdgpu_buffer_rsrc_t r, int vrec,
                                              int soff) {
    const int s0 = (int)(odd ? hi.x : lo.x), s1 = (int)(odd ? hi.y : lo.y);
    const unsigned r0 = (unsigned)__builtin_amdgcn_ds_swizzle(s0, 0x101F);  // and 0x1F, xor 4
    const unsigned r1 = (unsigned)__builtin_amdgcn_ds_swizzle(s1, 0x101F);
    const u32x4 v = odd ? (u32x4){r0, r1, lo.x, lo.y} : (u32x4){hi.x, hi.y, r0, r1};
    store_b128_guarded(v, r, vrec + (odd ? 16 : 0), soff);
}

// 4x4 transpose across the 4 lanes of a DPP quad (lane i = lane & 3): element r of lane i becomes
// element i of lane r, in two butterfly stages of quad_perm moves (xor 1, xor 2).  An accumulator
// column (one channel, 4 consecutive output rows per lane) turns into 4 consecutive channels of one
// row per lane, so the epilogue stores 16 B per lane instead of 4 (cdna_hip_programming.md T21: the
// store tail is issue-bound; k_conv3m's dword-store epilogue took 19 us of a 56-us workgroup,
// profiles/r04_d_stamps_down1_1.txt).
__device__ __forceinline__ float dpp_qxor1(float x) {
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), 0xB1, 0xF, 0xF, false));
}
__device__ __forceinline__ float dpp_qxor2(float x) {
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), 0x4E, 0xF, 0xF, false));
}
__device__ __forceinline__ void quad_transpose4(float (&a)[4], int i) {
    const bool o = (i & 1) != 0, t = (i & 2) != 0;
    float y = dpp_qxor1(o ? a[0] : a[1]);
    if (o) a[0] = y; else a[1] = y;
    y = dpp_qxor1(o ? a[2] : a[3]);
    if (o) a[2] = y; else a[3] = y;
    y = dpp_qxor2(t ? a[0] : a[2]);
    if (t) a[0] = y; else a[2] = y;
    y = dpp_qxor2(t ? a[1] : a[3]);
    if (t) a[1] = y; else a[3] = y;
}

template <int NT, int SPL, int NW, int RT>
__device__ __forceinline__ void conv_epi_store_cols(const ConvParams& p, f32x16 (&acc)[RT][NT], int m0, int n0,
                                                    int wv0, int lane, double* red) {
    constexpr int BN = 32 * NT;
    const int li = lane & 31;
    const int lh = lane >> 5;
    const bool gn = p.gn != nullptr;
    const bool bf = SPL == 2 || (SPL == 0 && p.bf != 0);
    const float wsc = SPL ? *p.wscale : 1.f;
    float bco[NT];
#pragma unroll
    for (int n = 0; n < NT; ++n) bco[n] = p.bias ? p.bias[n0 + n * 32 + li] : 0.f;
    // accumulator row r of a lane is output pixel pix0 + (r & 3) + 8 (r >> 2): a per-lane byte
    // offset (VGPR) plus a wave-uniform row offset (SGPR soffset)
    const __amdgpu_buffer_rsrc_t ry = mk_rsrc(p.y, (unsigned)((long long)p.M * p.Cout * 4));
    const bool b2 = p.out_h2 && p.bf == 2;  // 2-byte bf16 output (h2.hpp "b2")
    const int rowb = p.Cout * (b2 ? 2 : 4);
    const f32x2 wsc2 = {wsc, wsc};
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
        const int wv = wv0 + rt;
        const int pix0 = m0 + wv * 32 + 4 * lh;
#pragma unroll
        for (int n = 0; n < NT; ++n) {
            const int co = n0 + n * 32 + li;
            // fp32: the element; h2: the lane's dword of its 8-channel group record (even lane the
            // hi pair, odd lane the lo pair)
            const bool odd = (li & 1) != 0;
            const int vo = b2 ? (pix0 * p.Cout + co) * 2
                              : p.out_h2 ? pix0 * rowb + (co & ~7) * 4 + (odd ? 16 : 0) + 2 * ((co & 7) & ~1)
                                         : (pix0 * p.Cout + co) * 4;
            f32x2 add[8];
            if (p.resid) {  // attention proj only: the 16 residuals of this block before its stores
#pragma unroll
                for (int r = 0; r < 16; ++r)
                    add[r >> 1][r & 1] = bco[n] + p.resid[(pix0 + (r & 3) + 8 * (r >> 2)) * p.Cout + co];
            } else {
#pragma unroll
                for (int k = 0; k < 8; ++k) add[k] = (f32x2){bco[n], bco[n]};
            }
            f32x2 s2 = {0.f, 0.f}, ss2 = {0.f, 0.f};
            bool bad = false;
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const f32x2 a = {acc[rt][n][2 * k], acc[rt][n][2 * k + 1]};
                f32x2 v2 = SPL ? a * wsc2 + add[k] : a + add[k];
#pragma unroll
                for (int e = 0; e < 2; ++e) {
                    const int r = 2 * k + e;
                    float v = v2[e];
                    if (p.act == 1) v = fmaxf(v, 0.f);
                    else if (p.act == 2) v = 1.f / (1.f + expf(-v));
                    else if (p.act == 3) v = silu_f(v);
                    v2[e] = v;
                    const int so = ((r & 3) + 8 * (r >> 2)) * rowb;
                    if (b2) {
                        __builtin_amdgcn_raw_buffer_store_b16(bf16_bits((__bf16)v), ry, vo, so, 0);
                    } else if (p.out_h2) {
                        // lane pairs (2j, 2j+1) of an 8-channel group swap halves
                        const unsigned sp = split1x(v, bf);
                        const unsigned oth = (unsigned)__shfl_xor((int)(odd ? (sp & 0xffffu) : (sp >> 16)), 1);
                        const unsigned word = odd ? (oth | (sp & 0xffff0000u)) : ((sp & 0xffffu) | (oth << 16));
                        __builtin_amdgcn_raw_buffer_store_b32(word, ry, vo, so, 0);
                        bad = bad || (!bf && h2_bad(v));
                    } else {
                        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), ry, vo, so, 0);
                    }
                }
                s2 += v2;
                ss2 = v2 * v2 + ss2;
            }
            h2_flag(p.ovf, bad);
            if (gn) {
                double ds = (double)s2.x + (double)s2.y, dss = (double)ss2.x + (double)ss2.y;
                ds += __shfl_xor(ds, 32);
                dss += __shfl_xor(dss, 32);
                if (lh == 0) {
                    red[(wv * BN + n * 32 + li) * 2 + 0] = ds;
                    red[(wv * BN + n * 32 + li) * 2 + 1] = dss;
                }
            }
        }
    }
}

// No residual: each 4-row group of a column (rows 8 j + 4 (lane >> 5) + 0..3) is quad-transposed
// (quad_transpose4) so that lane l holds one row and 4 consecutive channels 4 ((l & 31) >> 2) .. + 3:
// one 16-B store (fp32) or two 8-B stores (the hi and lo halves of the h2 record) per lane and group,
// 4 instead of 16 store instructions per 32x32 block.  ACT: the activation is a run-time branch
// (false: none, straight-line code).  GroupNorm partials from the columns before the transpose.
// OUT (round 5): the output form compiled in (0 fp32, 1 h2 records, 2 two-byte bf16) or -1: chosen at
// run time per group (a run-time branch per store split k_conv3m's epilogue into blocks the scheduler
// could not overlap: 27 us of a 440-us 64^2 conv, r05_x)
template <int NT, int SPL, int NW, int RT, bool ACT, int OUT = -1>
__device__ __forceinline__ void conv_epi_store_quad(const ConvParams& p, f32x16 (&acc)[RT][NT], int m0, int n0,
                                                    int wv0, int lane, double* red) {
    constexpr int BN = 32 * NT;
    const int li = lane & 31;
    const int lh = lane >> 5;
    const int qi = lane & 3, qc = li >> 2;
    const bool gn = p.gn != nullptr;
    const bool bf = SPL == 2 || (SPL == 0 && p.bf != 0);
    const float wsc = SPL ? *p.wscale : 1.f;
    float bco[NT];
#pragma unroll
    for (int n = 0; n < NT; ++n) bco[n] = p.bias ? p.bias[n0 + n * 32 + li] : 0.f;
    const __amdgpu_buffer_rsrc_t ry = mk_rsrc(p.y, (unsigned)((long long)p.M * p.Cout * 4));
    // 2-byte bf16 output (h2.hpp "b2"): one 8-B store per lane and group
    const bool b2 = OUT >= 0 ? OUT == 2 : (p.out_h2 && p.bf == 2);
    const bool oh2 = OUT >= 0 ? OUT == 1 : (bool)p.out_h2;
    const int rowb = p.Cout * (b2 ? 2 : 4);
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
        const int wv = wv0 + rt;
        const int pixq = m0 + wv * 32 + 4 * lh + qi;  // this lane's row of group 0 after the transpose
#pragma unroll
        for (int n = 0; n < NT; ++n) {
            const int c4 = n0 + n * 32 + 4 * qc;  // first of this lane's 4 channels after the transpose
            const int vo32 = (pixq * p.Cout + c4) * 4;
            const int voh = pixq * rowb + (c4 >> 3) * 32 + (qc & 1) * 8;
            float s = 0.f, ss = 0.f;
            bool bad = false;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                float v[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    float x = SPL ? fmaf(acc[rt][n][4 * j + e], wsc, bco[n]) : acc[rt][n][4 * j + e] + bco[n];
                    if constexpr (ACT) {
                        if (p.act == 1) x = fmaxf(x, 0.f);
                        else if (p.act == 2) x = 1.f / (1.f + expf(-x));
                        else if (p.act == 3) x = silu_f(x);
                    }
                    v[e] = x;
                    s += x;
                    ss = fmaf(x, x, ss);
                }
                quad_transpose4(v, qi);
                const int so = 8 * j * rowb;
                typedef unsigned int u32x2_ __attribute__((ext_vector_type(2)));
                if (b2) {
                    const u32x2_ w2 = {pack2_bf(v[0], v[1]), pack2_bf(v[2], v[3])};
                    __builtin_amdgcn_raw_buffer_store_b64(w2, ry, (pixq * p.Cout + c4) * 2, so, 0);
                } else if (oh2) {
                    const unsigned a0 = split1x(v[0], bf), a1 = split1x(v[1], bf), a2 = split1x(v[2], bf),
                                   a3 = split1x(v[3], bf);
                    const u32x2_ hi = {(a0 & 0xffffu) | (a1 << 16), (a2 & 0xffffu) | (a3 << 16)};
                    const u32x2_ lo = {(a0 >> 16) | (a1 & 0xffff0000u), (a2 >> 16) | (a3 & 0xffff0000u)};
                    if (p.h2pair) {
                        store_h2_pair((u32x2_h2){hi.x, hi.y}, (u32x2_h2){lo.x, lo.y}, (qc & 1) != 0, ry,
                                      voh - (qc & 1) * 8, so);
                    } else {
                        __builtin_amdgcn_raw_buffer_store_b64(hi, ry, voh, so, 0);
                        __builtin_amdgcn_raw_buffer_store_b64(lo, ry, voh + 16, so, 0);
                    }
                    bad = bad || (!bf && (h2_bad(v[0]) || h2_bad(v[1]) || h2_bad(v[2]) || h2_bad(v[3])));
                } else {
                    store_b128_guarded<SPL == 2 ? EPI_NT : 0>(__builtin_bit_cast(u32x4, make_float4(v[0], v[1], v[2], v[3])), ry, vo32, so);
                }
            }
            h2_flag(p.ovf, bad);
            if (gn) {
                double ds = (double)s, dss = (double)ss;
                ds += __shfl_xor(ds, 32);
                dss += __shfl_xor(dss, 32);
                if (lh == 0) {
                    red[(wv * BN + n * 32 + li) * 2 + 0] = ds;
                    red[(wv * BN + n * 32 + li) * 2 + 1] = dss;
                }
            }
        }
    }
}

// (Round 4: bf16 had kept the column form after the quad form gave run-to-run different outputs in
// k_conv3lb; the cause was the store-data hazard of store_b128_guarded, now padded.)
template <int NT, int SPL, int NW, int RT>
__device__ __forceinline__ void conv_epi_store_fast(const ConvParams& p, f32x16 (&acc)[RT][NT], int m0, int n0,
                                                    int wv0, int lane, double* red) {
    if (p.resid) conv_epi_store_cols<NT, SPL, NW, RT>(p, acc, m0, n0, wv0, lane, red);  // attention proj
    else if (p.act == 0 && !p.epi_static) conv_epi_store_quad<NT, SPL, NW, RT, false>(p, acc, m0, n0, wv0, lane, red);
    else if (p.act == 0 && p.out_h2 && p.bf == 2) conv_epi_store_quad<NT, SPL, NW, RT, false, 2>(p, acc, m0, n0, wv0, lane, red);
    else if (p.act == 0 && p.out_h2) conv_epi_store_quad<NT, SPL, NW, RT, false, 1>(p, acc, m0, n0, wv0, lane, red);
    else if (p.act == 0) conv_epi_store_quad<NT, SPL, NW, RT, false, 0>(p, acc, m0, n0, wv0, lane, red);
    else conv_epi_store_quad<NT, SPL, NW, RT, true>(p, acc, m0, n0, wv0, lane, red);
}

// Fused epilogue of a conv tile: wave wv owns output rows m0 + 32*wv + [0, 32) and columns
// n0 + [0, 32*NT).  C/D map of the 32x32 MFMAs: col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5).
// bias / per-batch bias / residual / activation, fp32 or h2 store, and the fp64 GroupNorm partials
// of every 128-pixel group of waves (4 waves each; red: LDS scratch [NW][32*NT][2] doubles).
// conv_epi_store: one wave's 32 x 32*NT block (NW = waves of 32 rows in the tile, virtual waves
// when a wave owns several row blocks); conv_epi_gn: the per-128-pixel-group reduction of the
// partials in `red`, after a barrier.
// SPL: 0 = fp32 MFMA accumulators (an h2 output follows p.bf), 1 = f16x3, 2 = bf16 single product
template <int NT, int SPL, int NW>
__device__ __forceinline__ void conv_epi_store_general(const ConvParams& p, f32x16 (&acc)[NT], int m0, int n0, int wv,
                                                       int lane, double* red) {
    constexpr int BN = 32 * NT;
    const int li = lane & 31;
    const int lh = lane >> 5;
    const bool gn = p.gn != nullptr;
    const bool bf = SPL == 2 || (SPL == 0 && p.bf != 0);  // compile-time for the split kernels
    const bool dense_out = p.osy == 1 && p.osx == 1;
    const bool one_img = p.HoWo % (32 * NW) == 0;  // the whole tile belongs to image m0 / HoWo
    const int btile = m0 / p.HoWo;
#pragma unroll
    for (int n = 0; n < NT; ++n) {
        const int co = n0 + n * 32 + li;
        const bool cv = co < p.Cout;
        const int coc = cv ? co : 0;
        const float bco = p.bias ? p.bias[coc] : 0.f;
        const float bbt = (p.bias_b && one_img) ? p.bias_b[(size_t)btile * p.Cout + coc] : 0.f;
        size_t oidx[16];
        bool ok[16];
        float add[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int row = (r & 3) + 8 * (r >> 2) + 4 * lh;
            const int m = m0 + wv * 32 + row;
            ok[r] = m < p.M && cv;
            const int mm = m < p.M ? m : p.M - 1;
            add[r] = bco + bbt;
            if (dense_out) {
                oidx[r] = (size_t)mm * p.Cout + coc;
                if (p.bias_b && !one_img) add[r] += p.bias_b[(size_t)(mm / p.HoWo) * p.Cout + coc];
            } else {
                const int b = mm / p.HoWo;
                const int rr = mm - b * p.HoWo;
                const int oy = rr / p.Wo, ox = rr - (rr / p.Wo) * p.Wo;
                oidx[r] = ((size_t)b * p.Hy * p.Wy + (size_t)(oy * p.osy + p.ooy) * p.Wy + (ox * p.osx + p.oox)) * p.Cout + coc;
                if (p.bias_b) add[r] += p.bias_b[(size_t)b * p.Cout + coc] - bbt;
            }
        }
        if (p.resid) {
#pragma unroll
            for (int r = 0; r < 16; ++r) add[r] += p.resid[oidx[r]];
        }
        double s = 0.0, ss = 0.0;
        const float wsc = SPL ? *p.wscale : 1.f;
        bool bad = false;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            float v = (SPL ? acc[n][r] * wsc : acc[n][r]) + add[r];
            if (p.act == 1) v = fmaxf(v, 0.f);
            else if (p.act == 2) v = 1.f / (1.f + expf(-v));
            else if (p.act == 3) v = silu_f(v);
            if (p.out_h2 && p.bf == 2) {  // 2-byte bf16 output (h2.hpp "b2")
                if (ok[r]) *reinterpret_cast<unsigned short*>(reinterpret_cast<char*>(p.y) + oidx[r] * 2) = bf16_bits((__bf16)v);
            } else if (p.out_h2) {
                // h2 record of the pixel: lane pairs (2j, 2j+1) of an 8-channel group swap halves so
                // the even lane stores the hi pair and the odd lane the lo pair (one dword each)
                const unsigned sp = split1x(v, bf);
                const bool odd = (li & 1) != 0;
                const unsigned oth = (unsigned)__shfl_xor((int)(odd ? (sp & 0xffffu) : (sp >> 16)), 1);
                const unsigned word = odd ? (oth | (sp & 0xffff0000u)) : ((sp & 0xffffu) | (oth << 16));
                const size_t pe = oidx[r] - (size_t)coc;  // pixel's first element
                const int c8 = coc & ~7, j = (coc & 7) & ~1;
                if (ok[r]) {
                    *reinterpret_cast<unsigned*>(reinterpret_cast<char*>(p.y) + pe * 4 + (size_t)c8 * 4 + (odd ? 16 : 0) + 2 * j) = word;
                    bad = bad || (!bf && h2_bad(v));
                }
            } else if (ok[r]) {
                p.y[oidx[r]] = v;
            }
            if (ok[r]) {
                s += (double)v;
                ss += (double)v * (double)v;
            }
        }
        h2_flag(p.ovf, bad);
        if (gn) {
            s += __shfl_xor(s, 32);
            ss += __shfl_xor(ss, 32);
            if (lh == 0) {
                red[(wv * BN + n * 32 + li) * 2 + 0] = s;
                red[(wv * BN + n * 32 + li) * 2 + 1] = ss;
            }
        }
    }
}

// RT row blocks per wave (acc[rt] is virtual wave wv0 + rt)
template <int NT, int SPL, int NW, int RT>
__device__ __forceinline__ void conv_epi_store_rt(const ConvParams& p, f32x16 (&acc)[RT][NT], int m0, int n0, int wv0,
                                                  int lane, double* red) {
    if (conv_epi_fast<NT, SPL, NW, RT>(p, m0)) {
        conv_epi_store_fast<NT, SPL, NW, RT>(p, acc, m0, n0, wv0, lane, red);
    } else {
        // explicit calls, not a loop: a rolled loop over the (large) inlined general epilogue would
        // index acc dynamically and keep the whole accumulator array in scratch
        static_assert(RT == 1 || RT == 2, "RT is 1 or 2");
        conv_epi_store_general<NT, SPL, NW>(p, acc[0], m0, n0, wv0, lane, red);
        if constexpr (RT == 2) conv_epi_store_general<NT, SPL, NW>(p, acc[1], m0, n0, wv0 + 1, lane, red);
    }
}

template <int NT, int SPL, int NW>
__device__ __forceinline__ void conv_epi_store(const ConvParams& p, f32x16 (&acc)[NT], int m0, int n0, int wv,
                                               int lane, double* red) {
    conv_epi_store_rt<NT, SPL, NW, 1>(p, reinterpret_cast<f32x16(&)[1][NT]>(acc), m0, n0, wv, lane, red);
}

template <int NT, int NW>
__device__ __forceinline__ void conv_epi_gn(const ConvParams& p, int m0, int n0, int tid, int nthr,
                                            const double* red) {
    constexpr int BN = 32 * NT;
    {
        for (int e = tid; e < (NW / 4) * BN; e += nthr) {
            const int g = e / BN, cl = e - g * BN;  // 128-pixel group g of the tile, tile column cl
            const int co = n0 + cl;
            if (co < p.Cout) {
                double s = 0.0, ss = 0.0;
#pragma unroll
                for (int w = 0; w < 4; ++w) {
                    s += red[((4 * g + w) * BN + cl) * 2 + 0];
                    ss += red[((4 * g + w) * BN + cl) * 2 + 1];
                }
                const int mg = m0 + 128 * g;
                const int b = mg / p.HoWo;
                const int split = (mg - b * p.HoWo) / 128;
                double* dst = p.gn + (((size_t)b * p.nsplit + split) * p.Cout + co) * 2;
                dst[0] = s;
                dst[1] = ss;
            }
        }
    }
}

template <int NT, int SPL, int NW>
__device__ __forceinline__ void conv_epilogue(const ConvParams& p, f32x16 (&acc)[NT], int m0, int n0, int wv,
                                              int tid, double* red) {
    conv_epi_store<NT, SPL, NW>(p, acc, m0, n0, wv, tid & 63, red);
    if (p.gn) {
        __syncthreads();
        conv_epi_gn<NT, NW>(p, m0, n0, tid, NW * 64, red);
    }
}

}  // namespace
}  // namespace tcx
