// Implicit-GEMM 2-D convolution on fp32 MFMA (v_mfma_f32_32x32x2_f32), NHWC, gfx950.
//
// GEMM view: out[m = pixel][co] = sum_k A[m][k] * B[k][co],  k = (dy*ks + dx)*Cin + ci,
//   A[m][k] = x[b, wrap(oy*s - pad + dy), wrap(ox*s - pad + dx), ci]   (im2col, never stored)
//   B[k][co] = packed weight wpk[co][k]   (tcx_pack_conv_weight)
// Replaces nn.Conv2d(..., padding_mode="circular") of CondUNetTiny
// (/root/reference/src/toycrystals/models/sde_score_model.py:102,105,133-134,208,210,218,222,225)
// and the zero-padded Conv2d / ConvTranspose2d of CondVAE (models/vae.py:19-26,35-42).
//
// Tile: BM = 128 pixels x BN = 32*NT output channels, BK = 32; 4 waves, each owning a
// 32-pixel x BN slab (NT 32x32 accumulators = 16*NT AGPR/VGPR).  K is consumed in 32-deep
// chunks staged through LDS (register-staged double buffer: the next chunk's global loads are
// in flight while the current chunk's MFMAs run).  Inside a chunk the K order is permuted so
// that lane half h owns k = 16h + s (s = 0..15): each lane reads 4 consecutive k with one
// ds_read_b128, and A/B rows padded to 36 floats keep those reads bank-conflict free
// (row stride 144 B -> 9r mod 16 distinct in every 16-lane group).
// Fusions: channel concat (two sources), CFG batch aliasing (bmod), bilinear x2 upsample on
// the A load, bias / per-batch bias / residual / activation epilogue, and GroupNorm partial
// statistics of the output (fp64) for the following GroupNorm.
#include "conv_common.hpp"
#include "thin.hpp"

namespace tcx {
bool conv3m_takes(const ConvParams& p);  // conv3m.hip
namespace {

// MODE 0: float4 loads, per-lane (tap, ci) decode (Cin % 4 == 0)
// MODE 1: scalar loads, any Cin (the Cin = 1 first convs)
// MODE 2: float4 loads through a bilinear x2 upsample of the source
// MODE 3: float4 raw-buffer loads, chunk-uniform (SGPR) decode: Cin % 32 == 0, C1 % 32 == 0 and
//         C2 in {0, C1}, so a 32-deep K chunk is one tap of one source (every 3x3/4x4 layer of
//         the U-Net).  The byte offset of each (tap, tile pixel) is built once per workgroup in
//         an LDS table; per chunk a thread reads its 4 pixels' offsets with one ds_read_b128 and
//         the channel offset rides in the scalar soffset — no per-chunk im2col VALU.
// SPL: the f16x3 split path (h2.hpp): MODE 3 staging unchanged (4 bytes per element either
//      way); per 32-deep chunk two k16 steps, lane half h of step s owns the 8-channel group
//      2s + h = one hi and one lo b128 read per operand; 3 MFMA 32x32x16 f16 per accumulator.
template <int NT, int MODE, bool CIRC, bool PRO, int SPL = 0>  // SPL: 0 fp32, 1 f16x3, 2 bf16 (one product)
__global__ __launch_bounds__(256, 2) void k_conv(ConvParams p) {
    static_assert(!SPL || (MODE == 3 && !PRO), "split path: MODE 3 staging only, no prologue");
    constexpr int BN = 32 * NT;
    __shared__ __attribute__((aligned(16))) float As[2][BM * LDA];
    __shared__ __attribute__((aligned(16))) float Bs[2][BN * LDA];
    // fused GN prologue tables of this tile's image: [src1 scale, src1 shift, src2 scale, src2 shift]
    __shared__ __attribute__((aligned(16))) float Tr[PRO ? 4 * PRO_MAXC : 4];
    // MODE 3: [tap][prow][i] byte offset of tile pixel prow + 32 i at that tap (kOOB if masked)
    __shared__ __attribute__((aligned(16))) int Ptab[MODE == 3 ? MAXTAP * BM : 4];

    const int nwg = gridDim.x;
    const int tile = xcd_remap(blockIdx.x, nwg);
    const int mblk = tile / p.n_nblk;
    const int nblk = tile - mblk * p.n_nblk;
    const int m0 = mblk * BM;
    const int n0 = nblk * BN;

    const int tid = threadIdx.x;
    const int k4 = tid & 7;
    const int prow = tid >> 3;  // 0..31

    // per-thread pixel decode (4 pixel rows of the A tile)
    int pbase[4], piy[4], pix[4];
    bool pv[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int m = m0 + prow + 32 * i;
        pv[i] = m < p.M;
        const int mm = pv[i] ? m : 0;
        const int b = mm / p.HoWo;
        const int r = mm - b * p.HoWo;
        const int oy = r / p.Wo;
        const int ox = r - oy * p.Wo;
        const int bs = p.bmod > 0 ? b % p.bmod : b;
        pbase[i] = bs * p.H * p.W;
        piy[i] = oy * p.stride - p.pad_y;
        pix[i] = ox * p.stride - p.pad_x;
    }

    float4 ra[4];
    float4 rb[NT];

    // ---- per-chunk decode of k -> (tap, source, channel offset)
    struct Dec {
        const float* src;
        int cs, cc, dy, dx;
        bool kval;
        int tsel;  // which prologue table (0 = source 1, 2 = source 2)
        bool tr;   // apply the GN+SiLU prologue to this chunk
        int cb;    // chunk's first channel within its source (MODE 3)
        int tap;   // chunk's tap (MODE 3, uniform)
        bool s1;   // chunk comes from source 1 (MODE 3, uniform)
    };
    auto decode = [&](int c) -> Dec {
        Dec d;
        if constexpr (MODE == 3) {
            const int kc = c * BK;                 // uniform: SGPR arithmetic
            int tap = kc / p.Cin;
            const int ci0 = kc - tap * p.Cin;
            d.kval = tap < p.ks * p.ks;
            tap = d.kval ? tap : 0;
            d.tap = tap;
            d.dy = tap / p.ks;
            d.dx = tap - d.dy * p.ks;
            const bool s1 = ci0 < p.C1;
            d.src = s1 ? p.x1 : p.x2;
            d.cs = s1 ? p.C1 : p.C2;
            d.cc = (s1 ? ci0 : ci0 - p.C1) * 4;  // byte offset within the pixel (soffset)
            d.tsel = s1 ? 0 : 2;
            d.tr = s1 ? p.sc1 != nullptr : p.sc2 != nullptr;
            d.cb = s1 ? ci0 : ci0 - p.C1;
            d.s1 = s1;
        } else {
            const int k = c * BK + k4 * 4;
            int tap = k / p.Cin;
            const int ci = k - tap * p.Cin;
            d.kval = tap < p.ks * p.ks;
            tap = d.kval ? tap : 0;
            d.dy = tap / p.ks;
            d.dx = tap - d.dy * p.ks;
            const bool s1 = ci < p.C1;
            d.src = s1 ? p.x1 : p.x2;
            d.cs = s1 ? p.C1 : p.C2;
            d.cc = s1 ? ci : ci - p.C1;
            d.tsel = 0;
            d.tr = false;
            d.cb = 0;
            d.tap = 0;
            d.s1 = s1;
        }
        return d;
    };

    __amdgpu_buffer_rsrc_t r1, r2, rw;
    int boffw[NT];
    int4 poff;  // MODE 3: byte offsets of the thread's 4 pixels at the prefetched chunk's tap
    if constexpr (MODE == 3) {
        r1 = mk_rsrc(p.x1, p.bytes1);
        r2 = mk_rsrc(p.x2 ? p.x2 : p.x1, p.x2 ? p.bytes2 : p.bytes1);
        rw = mk_rsrc(p.w, p.bytesw);
#pragma unroll
        for (int j = 0; j < NT; ++j) boffw[j] = ((n0 + prow + 32 * j) * p.kpad + k4 * 4) * 4;
        const int ntap = p.ks * p.ks;
        const int rowb = p.C1 * 4;  // bytes per source pixel (C2 == C1 when there are two)
        for (int e = tid; e < ntap * BM; e += 256) {
            const int tap = e / BM, q = e - tap * BM;
            const int m = m0 + q;
            const int mm = m < p.M ? m : 0;
            const int b = mm / p.HoWo;
            const int r = mm - b * p.HoWo;
            const int oy = r / p.Wo, ox = r - (r / p.Wo) * p.Wo;
            const int bs = p.bmod > 0 ? b % p.bmod : b;
            const int dy = tap / p.ks, dx = tap - (tap / p.ks) * p.ks;
            int yr = oy * p.stride - p.pad_y + dy, xr = ox * p.stride - p.pad_x + dx;
            bool ok = m < p.M;
            if (CIRC) {
                yr = wrap_idx(yr, p.Hi);
                xr = wrap_idx(xr, p.Wi);
            } else {
                ok = ok && yr >= 0 && yr < p.Hi && xr >= 0 && xr < p.Wi;
            }
            Ptab[tap * BM + (q & 31) * 4 + (q >> 5)] = ok ? ((bs * p.H + yr) * p.W + xr) * rowb : kOOB;
        }
        __syncthreads();
    }
    auto read_poff = [&](const Dec& d) {
        poff = *reinterpret_cast<const int4*>(&Ptab[d.tap * BM + prow * 4]);
    };

    // A gather for pixel row i (all loads unconditional: masked elements read g_zero4; a
    // `cond ? load : 0` value select makes hipcc branch/wait per element or go through scratch).
    auto load_a = [&](const Dec& d, int c, int i) {
        constexpr bool circ = CIRC;
        if constexpr (MODE == 1) {
            float v[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int k = c * BK + k4 * 4 + e;
                int tap = k / p.Cin;
                const int ci = k - tap * p.Cin;
                const bool kval = tap < p.ks * p.ks;
                tap = kval ? tap : 0;
                const int dy = tap / p.ks, dx = tap - (tap / p.ks) * p.ks;
                const int yr = piy[i] + dy, xr = pix[i] + dx;
                const bool inb = yr >= 0 && yr < p.Hi && xr >= 0 && xr < p.Wi;
                const int yy = circ ? wrap_idx(yr, p.Hi) : min(max(yr, 0), p.Hi - 1);
                const int xx = circ ? wrap_idx(xr, p.Wi) : min(max(xr, 0), p.Wi - 1);
                const bool ok = pv[i] && kval && (circ || inb);
                const float* a = p.x1 + (size_t)(pbase[i] + yy * p.W + xx) * p.C1 + ci;
                v[e] = *(ok ? a : g_zero4);
            }
            ra[i] = make_float4(v[0], v[1], v[2], v[3]);
        } else if constexpr (MODE == 3) {
            // masked pixels carry kOOB: the buffer unit returns zeros (kpad == K: no K tail)
            const int po = i == 0 ? poff.x : i == 1 ? poff.y : i == 2 ? poff.z : poff.w;
            ra[i] = bld4(d.s1 ? r1 : r2, po + k4 * 16, d.cc);
        } else {
            const int yr = piy[i] + d.dy, xr = pix[i] + d.dx;
            const bool inb = yr >= 0 && yr < p.Hi && xr >= 0 && xr < p.Wi;
            const int yy = circ ? wrap_idx(yr, p.Hi) : min(max(yr, 0), p.Hi - 1);
            const int xx = circ ? wrap_idx(xr, p.Wi) : min(max(xr, 0), p.Wi - 1);
            const bool ok = pv[i] && d.kval && (circ || inb);
            if constexpr (MODE != 2) {
                const float* a = d.src + (size_t)(pbase[i] + yy * p.W + xx) * d.cs + d.cc;
                ra[i] = ld4(ok ? a : g_zero4);
            } else {
                int y0, y1, x0, x1;
                float ly0, ly1, lx0, lx1;
                bilin_axis(yy, p.H, y0, y1, ly0, ly1);
                bilin_axis(xx, p.W, x0, x1, lx0, lx1);
                const float* b0 = d.src + (size_t)pbase[i] * d.cs + d.cc;
                const float4 a00 = ld4(b0 + (size_t)(y0 * p.W + x0) * d.cs);
                const float4 a01 = ld4(b0 + (size_t)(y0 * p.W + x1) * d.cs);
                const float4 a10 = ld4(b0 + (size_t)(y1 * p.W + x0) * d.cs);
                const float4 a11 = ld4(b0 + (size_t)(y1 * p.W + x1) * d.cs);
                float4 r0 = make_float4(lx0 * a00.x, lx0 * a00.y, lx0 * a00.z, lx0 * a00.w);
                r0 = f4_fma(lx1, a01, r0);
                float4 r1 = make_float4(lx0 * a10.x, lx0 * a10.y, lx0 * a10.z, lx0 * a10.w);
                r1 = f4_fma(lx1, a11, r1);
                float4 acc = make_float4(ly0 * r0.x, ly0 * r0.y, ly0 * r0.z, ly0 * r0.w);
                acc = f4_fma(ly1, r1, acc);
                ra[i] = make_float4(ok ? acc.x : 0.f, ok ? acc.y : 0.f, ok ? acc.z : 0.f, ok ? acc.w : 0.f);
            }
        }
    };
    auto load_b = [&](int c) {
        if constexpr (MODE == 3) {
#pragma unroll
            for (int j = 0; j < NT; ++j) rb[j] = bld4(rw, boffw[j], c * BK * 4);
        } else {
#pragma unroll
            for (int j = 0; j < NT; ++j) {
                const int co = n0 + prow + 32 * j;
                rb[j] = ld4(p.w + (size_t)co * p.kpad + c * BK + k4 * 4);
            }
        }
    };
    auto store_chunk = [&](int buf) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
            *reinterpret_cast<float4*>(&As[buf][(prow + 32 * i) * LDA + k4 * 4]) = ra[i];
#pragma unroll
        for (int j = 0; j < NT; ++j)
            *reinterpret_cast<float4*>(&Bs[buf][(prow + 32 * j) * LDA + k4 * 4]) = rb[j];
    };

    f32x16 acc[NT];
#pragma unroll
    for (int n = 0; n < NT; ++n) acc[n] = (f32x16){};

    const int lane = tid & 63;
    const int wv = tid >> 6;
    const int li = lane & 31;
    const int lh = lane >> 5;

    if constexpr (PRO) {
        const int bimg = m0 / p.HoWo;  // host guarantees Ho*Wo % 128 == 0: one image per tile
        for (int c = tid; c < p.C1; c += 256) {
            Tr[c] = p.sc1 ? p.sc1[(size_t)bimg * p.C1 + c] : 1.f;
            Tr[PRO_MAXC + c] = p.sh1 ? p.sh1[(size_t)bimg * p.C1 + c] : 0.f;
        }
        for (int c = tid; c < p.C2; c += 256) {
            Tr[2 * PRO_MAXC + c] = p.sc2 ? p.sc2[(size_t)bimg * p.C2 + c] : 1.f;
            Tr[3 * PRO_MAXC + c] = p.sh2 ? p.sh2[(size_t)bimg * p.C2 + c] : 0.f;
        }
        __syncthreads();
    }
    {
        const Dec d0 = decode(0);
        if constexpr (MODE == 3) read_poff(d0);
#pragma unroll
        for (int i = 0; i < 4; ++i) load_a(d0, 0, i);
        load_b(0);
        store_chunk(0);
    }
    __syncthreads();

    // MFMA fragments, double-buffered in registers: group g (4 k-steps) computes from one set
    // while the reads of group g+1 are in flight into the other.
    float4 fa0, fa1, fb0[NT], fb1[NT];
    // GN+SiLU prologue (PRO): each A element of the LDS tile is read by exactly one lane, so the
    // source's silu(x*scale + shift) is applied to the fragment right after its read — the VALU
    // then issues in the shadow of the previous group's MFMAs (same work as a store-time pass).
    auto read_frags = [&](int buf, int g, const Dec& dc, float4& fa, float4 (&fb)[NT]) {
        const float* Ab = &As[buf][(wv * 32 + li) * LDA + lh * 16 + g * 4];
        const float* Bb = &Bs[buf][li * LDA + lh * 16 + g * 4];
        fa = ld4(Ab);
#pragma unroll
        for (int n = 0; n < NT; ++n) fb[n] = ld4(Bb + n * 32 * LDA);
        if constexpr (PRO) {
            if (dc.tr) {
                const int ch = dc.cb + lh * 16 + g * 4;
                const float4 sc = *reinterpret_cast<const float4*>(&Tr[dc.tsel * PRO_MAXC + ch]);
                const float4 sh = *reinterpret_cast<const float4*>(&Tr[(dc.tsel + 1) * PRO_MAXC + ch]);
                fa.x = silu_f(fmaf(fa.x, sc.x, sh.x));
                fa.y = silu_f(fmaf(fa.y, sc.y, sh.y));
                fa.z = silu_f(fmaf(fa.z, sc.z, sh.z));
                fa.w = silu_f(fmaf(fa.w, sc.w, sh.w));
            }
        }
    };
    auto mfma_group = [&](const float4& a, const float4 (&b)[NT]) {
#pragma unroll
        for (int n = 0; n < NT; ++n) acc[n] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, b[n].x, acc[n], 0, 0, 0);
#pragma unroll
        for (int n = 0; n < NT; ++n) acc[n] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, b[n].y, acc[n], 0, 0, 0);
#pragma unroll
        for (int n = 0; n < NT; ++n) acc[n] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, b[n].z, acc[n], 0, 0, 0);
#pragma unroll
        for (int n = 0; n < NT; ++n) acc[n] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, b[n].w, acc[n], 0, 0, 0);
    };

    if constexpr (SPL) {
        // fragments of both k16 steps of the chunk being computed (hi, lo per operand)
        h8 ah0, al0, ah1, al1, bh0[NT], bl0[NT], bh1[NT], bl1[NT];
        auto rd = [&](int buf, int s, h8& ah, h8& al, h8 (&bh)[NT], h8 (&bl)[NT]) {
            const float* Ab = &As[buf][(wv * 32 + li) * LDA + (2 * s + lh) * 8];
            ah = __builtin_bit_cast(h8, ld4(Ab));
            al = __builtin_bit_cast(h8, ld4(Ab + 4));
            const float* Bb = &Bs[buf][li * LDA + (2 * s + lh) * 8];
#pragma unroll
            for (int n = 0; n < NT; ++n) {
                bh[n] = __builtin_bit_cast(h8, ld4(Bb + n * 32 * LDA));
                bl[n] = __builtin_bit_cast(h8, ld4(Bb + n * 32 * LDA + 4));
            }
        };
        auto mf = [&](const h8& ah, const h8& al, const h8 (&bh)[NT], const h8 (&bl)[NT]) {
            if constexpr (SPL == 2) {  // bf16: hi x hi only
#pragma unroll
                for (int n = 0; n < NT; ++n)
                    acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf8, ah),
                                                                     __builtin_bit_cast(bf8, bh[n]), acc[n], 0, 0, 0);
                return;
            }
#pragma unroll
            for (int n = 0; n < NT; ++n) acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl[n], acc[n], 0, 0, 0);
#pragma unroll
            for (int n = 0; n < NT; ++n) acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh[n], acc[n], 0, 0, 0);
#pragma unroll
            for (int n = 0; n < NT; ++n) acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh[n], acc[n], 0, 0, 0);
        };
        // Two register staging sets, prefetch distance 2: chunk c+2 is loaded while chunk c computes
        // and chunk c+1 (loaded one iteration earlier, so its latency is covered by a whole chunk)
        // goes to LDS at the end of the iteration.  One f16x3 chunk is only 18 MFMAs per wave,
        // too short to hide an L2 round trip at distance 1.  MODE 3 staging: A = 4 pixel rows of
        // 16 B at the tap's byte offset, B = NT weight rows of 16 B.
        float4 sa1[4], sb1[NT];
        // running (tap, channel) of the load stream (wave-uniform, SGPRs): chunks are loaded in
        // order, so advance by 32 channels per chunk instead of dividing; past the last chunk the
        // state stays put (the last chunk is re-loaded into a set nothing stores)
        int ld_c = 1, ld_tap = BK / p.Cin, ld_ci = BK % p.Cin;
        auto ld_set = [&](float4 (&xa)[4], float4 (&xb)[NT]) {
            const bool s1 = ld_ci < p.C1;
            const int cc = (s1 ? ld_ci : ld_ci - p.C1) * 4;
            const int4 po = *reinterpret_cast<const int4*>(&Ptab[ld_tap * BM + prow * 4]);
            const __amdgpu_buffer_rsrc_t rs = s1 ? r1 : r2;
            xa[0] = bld4(rs, po.x + k4 * 16, cc);
            xa[1] = bld4(rs, po.y + k4 * 16, cc);
            xa[2] = bld4(rs, po.z + k4 * 16, cc);
            xa[3] = bld4(rs, po.w + k4 * 16, cc);
#pragma unroll
            for (int j = 0; j < NT; ++j) xb[j] = bld4(rw, boffw[j], ld_c * BK * 4);
            if (ld_c + 1 < p.nchunks) {
                ++ld_c;
                ld_ci += BK;
                if (ld_ci == p.Cin) {
                    ld_ci = 0;
                    ++ld_tap;
                }
            }
        };
        auto st_set = [&](const float4 (&xa)[4], const float4 (&xb)[NT], int buf) {
#pragma unroll
            for (int i = 0; i < 4; ++i) *reinterpret_cast<float4*>(&As[buf][(prow + 32 * i) * LDA + k4 * 4]) = xa[i];
#pragma unroll
            for (int j = 0; j < NT; ++j) *reinterpret_cast<float4*>(&Bs[buf][(prow + 32 * j) * LDA + k4 * 4]) = xb[j];
        };
        // chunk 0 is in LDS buffer 0 (common prologue); chunk 1 -> set 1
        ld_set(sa1, sb1);
        rd(0, 0, ah0, al0, bh0, bl0);
        auto iter = [&](int c, float4 (&la)[4], float4 (&lb)[NT], const float4 (&sa)[4], const float4 (&sb)[NT]) {
            const int cur = c & 1;
            ld_set(la, lb);  // chunk c + 2
            rd(cur, 1, ah1, al1, bh1, bl1);
            __builtin_amdgcn_sched_barrier(0);
            mf(ah0, al0, bh0, bl0);
            mf(ah1, al1, bh1, bl1);
            __builtin_amdgcn_sched_barrier(0);
            st_set(sa, sb, cur ^ 1);
            __syncthreads();
            rd(cur ^ 1, 0, ah0, al0, bh0, bl0);
        };
        // pairs of iterations with the staging sets swapped (static registers, no branch inside the
        // loop body, so the waitcnt state at the back edge is exact); an odd last chunk is peeled
        int c = 0;
        for (; c + 1 < p.nchunks; c += 2) {
            iter(c, ra, rb, sa1, sb1);
            iter(c + 1, sa1, sb1, ra, rb);
        }
        if (c < p.nchunks) iter(c, ra, rb, sa1, sb1);
    } else {
    Dec dc = decode(0);  // decode of the chunk being computed
    read_frags(0, 0, dc, fa0, fb0);
    for (int c = 0; c < p.nchunks; ++c) {
        const int cur = c & 1;
        // Branch-free pipeline: always prefetch; the last iteration re-loads its own (valid) chunk
        // into the idle buffer, which nothing reads.  The next chunk's global loads are spread over
        // the first MFMA groups so their address VALU issues in the MFMA shadow (T14/T19).
        const int cn = c + 1 < p.nchunks ? c + 1 : c;
        const Dec d = decode(cn);
        if constexpr (MODE == 3) read_poff(d);
        read_frags(cur, 1, dc, fa1, fb1);
        load_a(d, cn, 0);
        load_a(d, cn, 1);
        __builtin_amdgcn_sched_barrier(0);
        mfma_group(fa0, fb0);
        __builtin_amdgcn_sched_barrier(0);
        read_frags(cur, 2, dc, fa0, fb0);
        load_a(d, cn, 2);
        load_a(d, cn, 3);
        __builtin_amdgcn_sched_barrier(0);
        mfma_group(fa1, fb1);
        __builtin_amdgcn_sched_barrier(0);
        read_frags(cur, 3, dc, fa1, fb1);
        load_b(cn);
        __builtin_amdgcn_sched_barrier(0);
        mfma_group(fa0, fb0);
        __builtin_amdgcn_sched_barrier(0);
        mfma_group(fa1, fb1);
        store_chunk(cur ^ 1);
        __syncthreads();
        dc = d;
        read_frags(cur ^ 1, 0, dc, fa0, fb0);
    }
    }  // !SPL

    conv_epilogue<NT, SPL, 4>(p, acc, m0, n0, wv, tid, reinterpret_cast<double*>(&As[0][0]));
}

template <int NT>
int launch_nt(const ConvParams& p, int mode, hipStream_t st) {
    const int nm = cdiv(p.M, BM);
    const dim3 grid(nm * p.n_nblk), block(256);
    // chunk-uniform decode + raw-buffer loads (byte extents must fit the 32-bit offsets)
    const bool uni = mode == 0 && p.Cin % BK == 0 && p.C1 % BK == 0 && (p.C2 == 0 || p.C2 == p.C1) &&
                     p.ks * p.ks <= MAXTAP && p.kpad == p.ks * p.ks * p.Cin && p.Hi == p.H && p.Wi == p.W &&
                     p.bytes1 && (p.C2 == 0 || p.bytes2) && p.bytesw;
    const bool pro = p.sc1 || p.sc2;
    if (p.wscale) {  // split path (f16x3, or bf16 single product), validated by the caller: uni
        if (p.bf) {
            if (p.circular) hipLaunchKernelGGL((k_conv<NT, 3, true, false, 2>), grid, block, 0, st, p);
            else hipLaunchKernelGGL((k_conv<NT, 3, false, false, 2>), grid, block, 0, st, p);
        } else {
            if (p.circular) hipLaunchKernelGGL((k_conv<NT, 3, true, false, 1>), grid, block, 0, st, p);
            else hipLaunchKernelGGL((k_conv<NT, 3, false, false, 1>), grid, block, 0, st, p);
        }
        return check_launch("tcx_conv2d_h2");
    }
    if (pro) {  // validated by the caller: uni && circular
        hipLaunchKernelGGL((k_conv<NT, 3, true, true>), grid, block, 0, st, p);
    } else if (p.circular) {
        if (uni) hipLaunchKernelGGL((k_conv<NT, 3, true, false>), grid, block, 0, st, p);
        else if (mode == 0) hipLaunchKernelGGL((k_conv<NT, 0, true, false>), grid, block, 0, st, p);
        else if (mode == 1) hipLaunchKernelGGL((k_conv<NT, 1, true, false>), grid, block, 0, st, p);
        else hipLaunchKernelGGL((k_conv<NT, 2, true, false>), grid, block, 0, st, p);
    } else {
        if (uni) hipLaunchKernelGGL((k_conv<NT, 3, false, false>), grid, block, 0, st, p);
        else if (mode == 0) hipLaunchKernelGGL((k_conv<NT, 0, false, false>), grid, block, 0, st, p);
        else hipLaunchKernelGGL((k_conv<NT, 1, false, false>), grid, block, 0, st, p);
    }
    return check_launch("tcx_conv2d");
}

int launch_conv(ConvParams& p, int cout_pad, int mode, hipStream_t st) {
    // BN choice: 96 when it tiles Cout exactly (96, 192, 576 ...), else 64 / 32.
    int nt = (cout_pad % 96 == 0) ? 3 : (cout_pad % 64 == 0 ? 2 : 1);
    p.n_nblk = cout_pad / (32 * nt);
    if (p.M == 0) return TCX_OK;
    prof_begin(st);
    int rc;
    if (nt == 3) rc = launch_nt<3>(p, mode, st);
    else if (nt == 2) rc = launch_nt<2>(p, mode, st);
    else rc = launch_nt<1>(p, mode, st);
    // algorithmic work of this launch: 2 * pixels * Cout * ks^2 * Cin (no padding counted)
    prof_end(st, 2.0 * (double)p.M * p.Cout * p.ks * p.ks * p.Cin);
    return rc;
}

__global__ void k_pack_conv(const float* __restrict__ w, float* __restrict__ wpk, int Cout, int Cin, int ks,
                            int cout_pad, int kpad) {
    const size_t n = (size_t)cout_pad * kpad;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const int co = (int)(i / kpad);
        const int k = (int)(i - (size_t)co * kpad);
        const int tap = k / Cin, ci = k - (k / Cin) * Cin;
        float v = 0.f;
        if (co < Cout && tap < ks * ks) {
            const int dy = tap / ks, dx = tap - (tap / ks) * ks;
            v = w[(((size_t)co * Cin + ci) * ks + dy) * ks + dx];
        }
        wpk[i] = v;
    }
}

// ConvTranspose2d(k=4, s=2, p=1) as 4 sub-pixel 2x2 convs.  Output row oy = 2a + ry reads
// input rows a - 1 + dy (ry = 0: dy 0 -> ky 3, dy 1 -> ky 1) and a + dy (ry = 1: dy 0 -> ky 2,
// dy 1 -> ky 0); the same along x.  w [Cin][Cout][4][4] -> wpk[phase][cout_pad][kpad].
__global__ void k_pack_convT(const float* __restrict__ w, float* __restrict__ wpk, int Cin, int Cout,
                             int cout_pad, int kpad) {
    const size_t per = (size_t)cout_pad * kpad;
    const size_t n = 4 * per;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const int ph = (int)(i / per);
        const size_t rem = i - (size_t)ph * per;
        const int co = (int)(rem / kpad);
        const int k = (int)(rem - (size_t)co * kpad);
        const int tap = k / Cin, ci = k - (k / Cin) * Cin;
        float v = 0.f;
        if (co < Cout && tap < 4) {
            const int ry = ph >> 1, rx = ph & 1;
            const int dy = tap >> 1, dx = tap & 1;
            const int ky = ry == 0 ? (dy == 0 ? 3 : 1) : (dy == 0 ? 2 : 0);
            const int kx = rx == 0 ? (dx == 0 ? 3 : 1) : (dx == 0 ? 2 : 0);
            v = w[(((size_t)ci * Cout + co) * 4 + ky) * 4 + kx];
        }
        wpk[i] = v;
    }
}

// Data gradient of a stride-1 conv as a forward conv over dY: output channel ci' (= ci_lo + ci'),
// k = (dy*ks + dx)*Cout + co, value w[co][ci][ks-1-dy][ks-1-dx] (flipped taps, swapped channels).
__global__ void k_pack_conv_dgrad(const float* __restrict__ w, float* __restrict__ wpk, int Cout, int Cin, int ks,
                                  int ci_lo, int n_ci, int cout_pad, int kpad) {
    const size_t n = (size_t)cout_pad * kpad;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const int r = (int)(i / kpad);
        const int k = (int)(i - (size_t)r * kpad);
        const int tap = k / Cout, co = k - (k / Cout) * Cout;
        float v = 0.f;
        if (r < n_ci && tap < ks * ks) {
            const int dy = tap / ks, dx = tap - (tap / ks) * ks;
            v = w[(((size_t)co * Cin + ci_lo + r) * ks + (ks - 1 - dy)) * ks + (ks - 1 - dx)];
        }
        wpk[i] = v;
    }
}

// fp32 packed weight [cout_pad][kpad] -> h2 split [cout_pad][kpad/8][2][8] f16 of w * 2^e, with
// e chosen from max|w| so the largest scaled weight lies in [2^13, 2^14) (lo halves normal);
// *wscale = 2^-e.  One workgroup: max-reduce, then split.
// bf != 0: the bf16 single-product form — unscaled (bf16 has the fp32 range), *wscale = 1.
__global__ __launch_bounds__(1024) void k_pack_h2(const float* __restrict__ wpk, char* __restrict__ wh,
                                                  float* __restrict__ wscale, size_t n, int bf) {
    __shared__ float red[16];
    const int tid = threadIdx.x;
    float m = 0.f;
    for (size_t i = tid; i < n; i += 1024) m = fmaxf(m, fabsf(wpk[i]));
    for (int off = 32; off; off >>= 1) m = fmaxf(m, __shfl_xor(m, off));
    if ((tid & 63) == 0) red[tid >> 6] = m;
    __syncthreads();
    if (tid == 0) {
        float mx = 0.f;
        for (int w = 0; w < 16; ++w) mx = fmaxf(mx, red[w]);
        int k = 0;
        if (mx > 0.f && mx < INFINITY) (void)frexpf(mx, &k);  // mx < 2^k
        int e = bf ? 0 : 14 - k;
        e = e < -100 ? -100 : (e > 100 ? 100 : e);
        red[0] = ldexpf(1.f, e);
        wscale[0] = ldexpf(1.f, -e);
    }
    __syncthreads();
    const float sc = red[0];
    for (size_t g = tid; g < n / 4; g += 1024) {
        float4 v = reinterpret_cast<const float4*>(wpk)[g];
        v.x *= sc; v.y *= sc; v.z *= sc; v.w *= sc;
        store4_h2x(wh, (g >> 1) * 32, (int)(g & 1), v, bf != 0);
    }
}

}  // namespace
}  // namespace tcx

using namespace tcx;

extern "C" int tcx_pack_conv_weight_h2(const float* wpk, void* wh, float* wscale, int cout_pad, int kpad,
                                       void* stream) {
    TCX_REQUIRE(wpk && wh && wscale && cout_pad > 0 && kpad > 0 && kpad % BK == 0 && aligned16(wpk) && aligned16(wh),
                "tcx_pack_conv_weight_h2: bad args");
    hipLaunchKernelGGL(k_pack_h2, dim3(1), dim3(1024), 0, (hipStream_t)stream, wpk, (char*)wh, wscale,
                       (size_t)cout_pad * kpad, 0);
    return check_launch("tcx_pack_conv_weight_h2");
}

extern "C" int tcx_pack_conv_weight_bf16(const float* wpk, void* wh, float* wscale, int cout_pad, int kpad,
                                         void* stream) {
    TCX_REQUIRE(wpk && wh && wscale && cout_pad > 0 && kpad > 0 && kpad % BK == 0 && aligned16(wpk) && aligned16(wh),
                "tcx_pack_conv_weight_bf16: bad args");
    hipLaunchKernelGGL(k_pack_h2, dim3(1), dim3(1024), 0, (hipStream_t)stream, wpk, (char*)wh, wscale,
                       (size_t)cout_pad * kpad, 1);
    return check_launch("tcx_pack_conv_weight_bf16");
}

extern "C" int tcx_conv2d_h2_pro(const void* x1, const void* x2, int Bt, int bmod, int H, int W, int C1, int C2,
                                 const void* wh, const void* wfrag, const float* wscale, const float* bias,
                                 const float* bias_b,
                                 const float* resid, void* y, int out_h2, int Cout, int cout_pad, int kpad, int ks,
                                 int stride, int pad, int circular, int act, double* gn_stats, const float* pro_scale1,
                                 const float* pro_shift1, const float* pro_scale2, const float* pro_shift2,
                                 int bf16, unsigned* ovf, void* stream) {
    TCX_REQUIRE(x1 && wh && wscale && y, "tcx_conv2d_h2: null pointer");
    TCX_REQUIRE(Bt >= 0 && H > 0 && W > 0 && C1 > 0 && C2 >= 0 && Cout > 0, "tcx_conv2d_h2: bad shape");
    TCX_REQUIRE((C2 == 0) == (x2 == nullptr), "tcx_conv2d_h2: x2/C2 mismatch");
    TCX_REQUIRE(cout_pad >= Cout && cout_pad % 32 == 0, "tcx_conv2d_h2: cout_pad must be a multiple of 32 >= Cout");
    TCX_REQUIRE(act >= 0 && act <= 3 && ks >= 1 && stride >= 1 && pad >= 0, "tcx_conv2d_h2: bad geometry/act");
    const int Cin = C1 + C2;
    TCX_REQUIRE(C1 % BK == 0 && (C2 == 0 || C2 == C1) && ks * ks <= MAXTAP && kpad == ks * ks * Cin,
                "tcx_conv2d_h2: needs C1 %% 32 == 0, C2 in {0, C1}, ks*ks <= 16 and kpad == ks*ks*Cin");
    TCX_REQUIRE(!out_h2 || Cout % 8 == 0, "tcx_conv2d_h2: h2 output needs Cout %% 8 == 0");
    TCX_REQUIRE(aligned16(x1) && (!x2 || aligned16(x2)) && aligned16(wh) && aligned16(y),
                "tcx_conv2d_h2: pointers must be 16-B aligned");
    ConvParams p{};
    p.x1 = (const float*)x1; p.x2 = (const float*)x2; p.C1 = C1; p.C2 = C2; p.Cin = Cin;
    p.bmod = bmod; p.H = H; p.W = W; p.Hi = H; p.Wi = W;
    p.Ho = (H + 2 * pad - ks) / stride + 1;
    p.Wo = (W + 2 * pad - ks) / stride + 1;
    TCX_REQUIRE(p.Ho > 0 && p.Wo > 0, "tcx_conv2d_h2: empty output");
    p.HoWo = p.Ho * p.Wo;
    p.M = Bt * p.HoWo;
    p.w = (const float*)wh; p.bias = bias; p.bias_b = bias_b; p.resid = resid; p.y = (float*)y;
    p.Cout = Cout; p.kpad = kpad; p.nchunks = kpad / BK;
    p.ks = ks; p.stride = stride; p.pad_y = pad; p.pad_x = pad; p.circular = circular;
    p.Hy = p.Ho; p.Wy = p.Wo; p.osy = 1; p.ooy = 0; p.osx = 1; p.oox = 0; p.act = act;
    p.gn = gn_stats;
    p.nsplit = cdiv(p.HoWo, BM);
    if (gn_stats) TCX_REQUIRE(p.HoWo % BM == 0, "tcx_conv2d_h2: fused GN stats need Ho*Wo %% 128 == 0");
    // bits 4 / 5 of bf16: source 1 / source 2 chunk-major ([C/8][B][H][W][32 B] records, ConvParams::cm1/cm2)
    const int cmf = bf16 >> 4;
    bf16 &= 15;
    TCX_REQUIRE(bf16 >= 0 && bf16 <= 2 && cmf >= 0 && cmf <= 3,
                "tcx_conv2d_h2: bf16 must be 0 (f16x3), 1 (bf16 records) or 2 (2-byte bf16), plus chunk-major bits 16/32");
    const size_t bsrc = bmod > 0 ? (size_t)bmod : (size_t)Bt;
    const size_t lim = (size_t)1 << 31;
    const size_t esz = bf16 == 2 ? 2 : 4;  // bytes per source element (the prologue's fp32 sources: 4)
    const size_t b1 = bsrc * H * W * C1 * (pro_scale1 ? 4 : esz), b2 = bsrc * H * W * C2 * (pro_scale2 ? 4 : esz),
                 bw = (size_t)cout_pad * kpad * 4;
    TCX_REQUIRE(b1 < lim && b2 < lim && bw < lim, "tcx_conv2d_h2: operands must be < 2 GiB (32-bit buffer offsets)");
    p.bytes1 = (unsigned)b1; p.bytes2 = (unsigned)b2; p.bytesw = (unsigned)bw;
    p.wscale = wscale; p.out_h2 = out_h2; p.ovf = ovf;
    TCX_REQUIRE(!pro_scale1 == !pro_shift1 && !pro_scale2 == !pro_shift2 && (C2 > 0 || !pro_scale2),
                "tcx_conv2d_h2: prologue tables come in scale/shift pairs per source");
    p.sc1 = pro_scale1; p.sh1 = pro_shift1; p.sc2 = pro_scale2; p.sh2 = pro_shift2;
    p.wf = wfrag;
    static const int h2pair = [] {
        const char* e = getenv("TCX_H2_PAIR");
        return (e && e[0] == '0') ? 0 : 1;
    }();
    p.h2pair = h2pair;
    static const int epi_static = [] {
        const char* e = getenv("TCX_EPI_STATIC");
        return (e && e[0] == '0') ? 0 : 1;
    }();
    p.epi_static = epi_static;
    p.bf = bf16;  // k_conv3p / k_conv3h have no bf16 form: those shapes take the im2col kernel
    if (bf16 == 2) {
        // 2-byte bf16 tensors (config 5 at 256^2): only the LDS-DMA kernels read them
        TCX_REQUIRE(!pro_scale1 && !pro_scale2, "tcx_conv2d_h2: 2-byte bf16 sources take no prologue");
        ConvParams q = p;
        q.n_nblk = cout_pad / 96;
        const bool ok = (conv3g_applies(p, cout_pad) && conv3lb_takes(q)) || conv4s2g_applies(p, cout_pad) ||
                        lin1x1_applies(p, cout_pad);
        TCX_REQUIRE(ok, "tcx_conv2d_h2: 2-byte bf16 operands need k_conv3lb (3x3, rows of 64/128/256 px), "
                        "k_conv4s2g (4x4/s2) or k_lin1x1 (1x1) shapes");
    }
    if (cmf) {
        // chunk-major sources: the 4x4/s2 LDS-DMA kernel (source 1) or k_conv3m (source 2) for f16x3 records;
        // config 5's 2-byte bf16 planes (round 6): k_conv4s2g's slim form (source 1) or k_conv3lb (source 2)
        p.cm1 = cmf & 1;
        p.cm2 = cmf >> 1;
        TCX_REQUIRE((bf16 == 0 || bf16 == 2) && !pro_scale1 && !pro_scale2 && (!p.cm2 || C2 > 0) && cmf != 3,
                    "tcx_conv2d_h2: chunk-major sources are f16x3 records or 2-byte bf16, without a prologue, on one "
                    "source");
        if (p.cm1) {
            TCX_REQUIRE(conv4s2g_applies(p, cout_pad), "tcx_conv2d_h2: a chunk-major source 1 needs a k_conv4s2g shape");
            return launch_conv4s2g(p, cout_pad, (hipStream_t)stream);
        }
        if (bf16 == 2) {
            ConvParams q = p;
            q.n_nblk = cout_pad / 96;
            TCX_REQUIRE(conv3g_applies(p, cout_pad) && conv3lb_takes(q),
                        "tcx_conv2d_h2: a chunk-major 2-byte bf16 source 2 needs a k_conv3lb shape");
            return launch_conv3g(p, cout_pad, (hipStream_t)stream);
        }
        TCX_REQUIRE(conv3g_applies(p, cout_pad) && conv3m_takes(p),
                    "tcx_conv2d_h2: a chunk-major source 2 needs a k_conv3m shape");
        return launch_conv3g(p, cout_pad, (hipStream_t)stream);
    }
    if (conv3g_applies(p, cout_pad)) return launch_conv3g(p, cout_pad, (hipStream_t)stream);
    TCX_REQUIRE(!pro_scale1 && !pro_scale2,
                "tcx_conv2d_h2: the GroupNorm+SiLU prologue needs k_conv3g: the fragment-ordered weights "
                "(tcx_pack_conv_weight_h2_frag) and a 3x3 stride-1 conv with W in {16, 32, 64, 128}, Cin %% 32 == 0, "
                "Cin <= 384, Cout padded to 96k");
    if (!p.bf && conv3h_applies(p, cout_pad)) return launch_conv3h(p, cout_pad, (hipStream_t)stream);
    if (conv4s2g_applies(p, cout_pad)) return launch_conv4s2g(p, cout_pad, (hipStream_t)stream);
    if (conv4s2h_applies(p, cout_pad)) return launch_conv4s2h(p, cout_pad, (hipStream_t)stream);
    if (lin1x1_applies(p, cout_pad)) return launch_lin1x1(p, cout_pad, (hipStream_t)stream);
    return launch_conv(p, cout_pad, 0, (hipStream_t)stream);
}

extern "C" int tcx_conv2d_h2(const void* x1, const void* x2, int Bt, int bmod, int H, int W, int C1, int C2,
                             const void* wh, const float* wscale, const float* bias, const float* bias_b,
                             const float* resid, void* y, int out_h2, int Cout, int cout_pad, int kpad, int ks,
                             int stride, int pad, int circular, int act, double* gn_stats, unsigned* ovf,
                             void* stream) {
    return tcx_conv2d_h2_pro(x1, x2, Bt, bmod, H, W, C1, C2, wh, nullptr, wscale, bias, bias_b, resid, y, out_h2, Cout,
                             cout_pad, kpad, ks, stride, pad, circular, act, gn_stats, nullptr, nullptr, nullptr,
                             nullptr, 0, ovf, stream);
}

extern "C" int tcx_conv2d(const float* x1, const float* x2, int Bt, int bmod, int H, int W, int C1, int C2,
                          const float* wpk, const float* bias, const float* bias_b, const float* resid,
                          float* y, int Cout, int cout_pad, int kpad, int ks, int stride, int pad,
                          int circular, int upsample, int act, double* gn_stats, const float* pro_scale1,
                          const float* pro_shift1, const float* pro_scale2, const float* pro_shift2,
                          void* stream) {
    TCX_REQUIRE(x1 && wpk && y, "tcx_conv2d: null pointer");
    TCX_REQUIRE(Bt >= 0 && H > 0 && W > 0 && C1 > 0 && C2 >= 0 && Cout > 0, "tcx_conv2d: bad shape");
    TCX_REQUIRE((C2 == 0) == (x2 == nullptr), "tcx_conv2d: x2/C2 mismatch");
    TCX_REQUIRE(cout_pad >= Cout && cout_pad % 32 == 0, "tcx_conv2d: cout_pad must be a multiple of 32 >= Cout");
    const int Cin = C1 + C2;
    TCX_REQUIRE(kpad % BK == 0 && kpad >= ks * ks * Cin, "tcx_conv2d: kpad must be a multiple of 32 >= ks*ks*Cin");
    TCX_REQUIRE(ks >= 1 && stride >= 1 && pad >= 0, "tcx_conv2d: bad geometry");
    ConvParams p{};
    p.x1 = x1; p.x2 = x2; p.C1 = C1; p.C2 = C2; p.Cin = Cin;
    p.bmod = bmod; p.H = H; p.W = W;
    p.Hi = upsample ? 2 * H : H;
    p.Wi = upsample ? 2 * W : W;
    p.Ho = (p.Hi + 2 * pad - ks) / stride + 1;
    p.Wo = (p.Wi + 2 * pad - ks) / stride + 1;
    TCX_REQUIRE(p.Ho > 0 && p.Wo > 0, "tcx_conv2d: empty output");
    p.HoWo = p.Ho * p.Wo;
    p.M = Bt * p.HoWo;
    p.w = wpk; p.bias = bias; p.bias_b = bias_b; p.resid = resid; p.y = y;
    p.Cout = Cout; p.kpad = kpad; p.nchunks = kpad / BK;
    p.ks = ks; p.stride = stride; p.pad_y = pad; p.pad_x = pad; p.circular = circular;
    TCX_REQUIRE(act >= 0 && act <= 3, "tcx_conv2d: bad act");
    p.Hy = p.Ho; p.Wy = p.Wo; p.osy = 1; p.ooy = 0; p.osx = 1; p.oox = 0; p.act = act;
    p.gn = gn_stats;
    p.nsplit = cdiv(p.HoWo, BM);
    int mode = 0;
    const bool vec_ok = (C1 % 4 == 0) && (C2 % 4 == 0) && aligned16(x1) && (!x2 || aligned16(x2));
    if (upsample) {
        TCX_REQUIRE(vec_ok && circular, "tcx_conv2d: upsample needs Cin%4==0, circular padding");
        mode = 2;
    } else if (!vec_ok) {
        TCX_REQUIRE(x2 == nullptr, "tcx_conv2d: scalar path supports a single source");
        mode = 1;
    }
    if (gn_stats) TCX_REQUIRE(p.HoWo % BM == 0, "tcx_conv2d: fused GN stats need Ho*Wo %% 128 == 0");
    p.sc1 = pro_scale1; p.sh1 = pro_shift1; p.sc2 = pro_scale2; p.sh2 = pro_shift2;
    {
        const size_t bsrc = bmod > 0 ? (size_t)bmod : (size_t)Bt;
        const size_t lim = (size_t)1 << 31;
        const size_t b1 = bsrc * H * W * C1 * sizeof(float), b2 = bsrc * H * W * C2 * sizeof(float);
        const size_t bw = (size_t)cout_pad * kpad * sizeof(float);
        p.bytes1 = b1 < lim ? (unsigned)b1 : 0u;
        p.bytes2 = b2 < lim ? (unsigned)b2 : 0u;
        p.bytesw = bw < lim ? (unsigned)bw : 0u;
    }
    if (pro_scale1 || pro_scale2) {
        TCX_REQUIRE((pro_scale1 != nullptr) == (pro_shift1 != nullptr) &&
                    (pro_scale2 != nullptr) == (pro_shift2 != nullptr), "tcx_conv2d: prologue scale/shift pairs");
        TCX_REQUIRE(mode == 0 && Cin % BK == 0 && C1 % BK == 0 && circular && bmod == 0 && p.HoWo % BM == 0 &&
                    C1 <= PRO_MAXC && C2 <= PRO_MAXC && (pro_scale2 == nullptr || x2 != nullptr) &&
                    (C2 == 0 || C2 == C1) && ks * ks <= MAXTAP && kpad == ks * ks * Cin &&
                    p.bytes1 && (C2 == 0 || p.bytes2) && p.bytesw,
                    "tcx_conv2d: fused GN prologue needs Cin,C1 %% 32 == 0, C2 in {0,C1}, kpad == K, circular, "
                    "no bmod/upsample, Ho*Wo %% 128 == 0, C <= 384, extents < 2 GiB");
    }
    TCX_REQUIRE(aligned16(wpk), "tcx_conv2d: packed weight must be 16-B aligned");
    if (!upsample && !gn_stats && !pro_scale1 && !pro_scale2 && bmod == 0 && C2 == 0 && stride == 1) {
        // one-channel side (the score net's first / out convs and the out conv's data gradient): thin.hip
        ThinConv a{x1, wpk, bias, bias_b, resid, y, Bt, H, W, C1, Cout, kpad, ks, pad, circular, p.Ho, p.Wo, act};
        if (thin_conv_takes(a)) return launch_thin_conv(a, (hipStream_t)stream);
    }
    return launch_conv(p, cout_pad, mode, (hipStream_t)stream);
}

extern "C" int tcx_convT2x(const float* x, int Bt, int H, int W, int Cin, const float* wpk4, const float* bias,
                           float* y, int Cout, int cout_pad, int kpad, int act, void* stream) {
    return tcx_conv_transpose2x(x, Bt, H, W, Cin, wpk4, bias, y, Cout, cout_pad, kpad, act, 0, stream);
}

extern "C" int tcx_conv_transpose2x(const float* x, int Bt, int H, int W, int Cin, const float* wpk4,
                                    const float* bias, float* y, int Cout, int cout_pad, int kpad, int act,
                                    int circular, void* stream) {
    TCX_REQUIRE(x && wpk4 && y, "tcx_convT2x: null pointer");
    TCX_REQUIRE(cout_pad >= Cout && cout_pad % 32 == 0 && kpad % BK == 0 && kpad >= 4 * Cin, "tcx_convT2x: bad padding");
    for (int ph = 0; ph < 4; ++ph) {
        const int ry = ph >> 1, rx = ph & 1;
        ConvParams p{};
        p.x1 = x; p.x2 = nullptr; p.C1 = Cin; p.C2 = 0; p.Cin = Cin;
        p.bmod = 0; p.H = H; p.W = W; p.Hi = H; p.Wi = W;
        p.Ho = H; p.Wo = W; p.HoWo = H * W; p.M = Bt * H * W;
        p.w = wpk4 + (size_t)ph * cout_pad * kpad;
        p.bias = bias; p.bias_b = nullptr; p.resid = nullptr; p.y = y;
        p.Cout = Cout; p.kpad = kpad; p.nchunks = kpad / BK;
        p.ks = 2; p.stride = 1; p.pad_y = 1 - ry; p.pad_x = 1 - rx; p.circular = circular;
        p.Hy = 2 * H; p.Wy = 2 * W; p.osy = 2; p.ooy = ry; p.osx = 2; p.oox = rx;
        p.act = act; p.gn = nullptr; p.nsplit = 1;
        const bool vec_ok = (Cin % 4 == 0) && aligned16(x);
        {
            const size_t lim = (size_t)1 << 31;
            const size_t b1 = (size_t)Bt * H * W * Cin * sizeof(float), bw = (size_t)cout_pad * kpad * sizeof(float);
            p.bytes1 = b1 < lim ? (unsigned)b1 : 0u;
            p.bytesw = bw < lim && aligned16(p.w) ? (unsigned)bw : 0u;
        }
        TCX_TRY(launch_conv(p, cout_pad, vec_ok ? 0 : 1, (hipStream_t)stream));
    }
    return TCX_OK;
}

// The same four sub-pixel 2x2 convs on the f16x3 split path (round 6): the training step's data gradient
// of the 4x4/s2 downsamples (the adjoint of sde_score_model.py:215-216's ds1 / ds2) on h2 records of dY
// and of the phase weights (tcx_f32_to_h2_scaled of tcx_pack_convT_weight's [4][cout_pad][kpad]), the
// combined scale *wscale = 1 / (s_w s_dy) applied in k_conv's epilogue (MODE 3 staging, SPL 1)
extern "C" int tcx_conv_transpose2x_h2(const void* xh, int Bt, int H, int W, int Cin, const void* wh4,
                                       const float* wscale, const float* bias, float* y, int Cout, int cout_pad,
                                       int kpad, int act, int circular, void* stream) {
    TCX_REQUIRE(xh && wh4 && wscale && y, "tcx_convT2x_h2: null pointer");
    TCX_REQUIRE(Bt >= 0 && H > 0 && W > 0 && Cin % BK == 0 && Cout > 0 && cout_pad >= Cout && cout_pad % 32 == 0 &&
                    kpad == 4 * Cin && act >= 0 && act <= 3,
                "tcx_convT2x_h2: needs Cin %% 32 == 0, kpad == 4 Cin, cout_pad %% 32 == 0");
    TCX_REQUIRE(aligned16(xh) && aligned16(wh4) && aligned16(y), "tcx_convT2x_h2: pointers must be 16-B aligned");
    const size_t lim = (size_t)1 << 31;
    const size_t b1 = (size_t)Bt * H * W * Cin * 4, bw = (size_t)cout_pad * kpad * 4;
    TCX_REQUIRE(b1 < lim && 4 * bw < lim, "tcx_convT2x_h2: operands must be < 2 GiB (32-bit buffer offsets)");
    for (int ph = 0; ph < 4; ++ph) {
        const int ry = ph >> 1, rx = ph & 1;
        ConvParams p{};
        p.x1 = (const float*)xh; p.x2 = nullptr; p.C1 = Cin; p.C2 = 0; p.Cin = Cin;
        p.bmod = 0; p.H = H; p.W = W; p.Hi = H; p.Wi = W;
        p.Ho = H; p.Wo = W; p.HoWo = H * W; p.M = Bt * H * W;
        p.w = (const float*)((const char*)wh4 + (size_t)ph * bw);
        p.bias = bias; p.bias_b = nullptr; p.resid = nullptr; p.y = y;
        p.Cout = Cout; p.kpad = kpad; p.nchunks = kpad / BK;
        p.ks = 2; p.stride = 1; p.pad_y = 1 - ry; p.pad_x = 1 - rx; p.circular = circular;
        p.Hy = 2 * H; p.Wy = 2 * W; p.osy = 2; p.ooy = ry; p.osx = 2; p.oox = rx;
        p.act = act; p.gn = nullptr; p.nsplit = 1;
        p.bytes1 = (unsigned)b1; p.bytesw = (unsigned)bw;
        p.wscale = wscale; p.out_h2 = 0; p.bf = 0;
        TCX_TRY(launch_conv(p, cout_pad, 0, (hipStream_t)stream));
    }
    return TCX_OK;
}

extern "C" int tcx_pack_conv_weight(const float* w, float* wpk, int Cout, int Cin, int ks, int cout_pad, int kpad,
                                    void* stream) {
    TCX_REQUIRE(w && wpk && cout_pad >= Cout && kpad >= ks * ks * Cin, "tcx_pack_conv_weight: bad args");
    const size_t n = (size_t)cout_pad * kpad;
    const int blocks = (int)std::min<size_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(k_pack_conv, dim3(blocks), dim3(256), 0, (hipStream_t)stream, w, wpk, Cout, Cin, ks, cout_pad, kpad);
    return check_launch("tcx_pack_conv_weight");
}

extern "C" int tcx_pack_convT_weight(const float* w, float* wpk, int Cin, int Cout, int cout_pad, int kpad,
                                     void* stream) {
    TCX_REQUIRE(w && wpk && cout_pad >= Cout && kpad >= 4 * Cin, "tcx_pack_convT_weight: bad args");
    const size_t n = 4 * (size_t)cout_pad * kpad;
    const int blocks = (int)std::min<size_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(k_pack_convT, dim3(blocks), dim3(256), 0, (hipStream_t)stream, w, wpk, Cin, Cout, cout_pad, kpad);
    return check_launch("tcx_pack_convT_weight");
}

extern "C" int tcx_linear(const float* x1, int K1, const float* x2, int K2, const float* wpk, const float* b,
                          const float* resid, float* y, int M, int N, int npad, int kpad, int act, void* stream) {
    const int K = K1 + K2;
    TCX_REQUIRE(x1 && wpk && y && M >= 0 && N > 0 && K1 > 0 && K2 >= 0, "tcx_linear: bad args");
    TCX_REQUIRE((K2 == 0) == (x2 == nullptr), "tcx_linear: x2/K2 mismatch");
    TCX_REQUIRE(npad >= N && npad % 32 == 0 && kpad >= K && kpad % BK == 0, "tcx_linear: bad padding");
    TCX_REQUIRE(act >= 0 && act <= 3, "tcx_linear: bad act");
    ConvParams p{};
    p.x1 = x1; p.x2 = x2; p.C1 = K1; p.C2 = K2; p.Cin = K;
    p.bmod = 0; p.H = 1; p.W = 1; p.Hi = 1; p.Wi = 1; p.Ho = 1; p.Wo = 1; p.HoWo = 1; p.M = M;
    p.w = wpk; p.bias = b; p.bias_b = nullptr; p.resid = resid; p.y = y;
    // chunks cover K only: a caller may pass a column window of a wider packed weight (row stride
    // kpad, e.g. one half of the prior's FiLM projection), whose columns past K are not padding
    p.Cout = N; p.kpad = kpad; p.nchunks = cdiv(K, BK);
    p.ks = 1; p.stride = 1; p.pad_y = 0; p.pad_x = 0; p.circular = 0;
    p.Hy = 1; p.Wy = 1; p.osy = 1; p.ooy = 0; p.osx = 1; p.oox = 0; p.act = act; p.gn = nullptr; p.nsplit = 1;
    const bool vec_ok = (K1 % 4 == 0) && (K2 % 4 == 0) && aligned16(x1) && (!x2 || aligned16(x2));
    TCX_REQUIRE(vec_ok || x2 == nullptr, "tcx_linear: two-source form needs K1,K2 %% 4 == 0 and aligned rows");
    return launch_conv(p, npad, vec_ok ? 0 : 1, (hipStream_t)stream);
}

extern "C" int tcx_pack_conv_dgrad_weight(const float* w, float* wpk, int Cout, int Cin, int ks, int ci_lo, int n_ci,
                                          int cout_pad, int kpad, void* stream) {
    TCX_REQUIRE(w && wpk && ci_lo >= 0 && n_ci > 0 && ci_lo + n_ci <= Cin && cout_pad >= n_ci &&
                kpad >= ks * ks * Cout, "tcx_pack_conv_dgrad_weight: bad args");
    const size_t n = (size_t)cout_pad * kpad;
    const int blocks = (int)std::min<size_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(k_pack_conv_dgrad, dim3(blocks), dim3(256), 0, (hipStream_t)stream, w, wpk, Cout, Cin, ks, ci_lo,
                       n_ci, cout_pad, kpad);
    return check_launch("tcx_pack_conv_dgrad_weight");
}
