// k_lin1x1: the 1x1 convs of SelfAttention2d (qkv and proj, /root/reference/src/toycrystals/models/
// sde_score_model.py:141-160; 16^2 tokens x 192 -> 576 / 192 at the metric's config) on the split
// path as a plain GEMM over h2 records: y[m][n] = sum_k x[m][k] w[n][k] (+ bias, + residual).
//
// They ran on the im2col kernel (k_conv SPL, conv.hip), which writes every A element to LDS with
// ds_write and re-stages per 32-deep chunk: 0.16 of the f16x3 ceiling.  Here a workgroup owns
// 128 rows x 96 output channels, streams K in 32-channel chunks (128 B of h2 per row) by LDS-DMA
// straight from the activation records and the packed h2 weight rows (no fragment-ordered copy
// needed: the B tile is 96 weight rows x 128 B, the same row-major image as the A tile), double-
// buffered, one barrier per chunk.  Both tiles are row-major with 128-B rows, so the 16-B pieces of
// row r are XOR-swizzled by (r >> 1) & 7: every 16-lane group of a ds_read_b128 of 32 consecutive
// rows then covers 16 distinct 16-B slots of the 256-B bank row (MI355X_MICROARCH.md §LDS groups).
// The DMA writes lane-linearly (lane l of an instruction fills row l / 8, physical piece l % 8), so the
// swizzle rides on the per-lane source offset.  f16x3: hi*lo + lo*hi + hi*hi per product (h2.hpp);
// BF: one bf16 MFMA of the hi halves.  Epilogue shared with the conv kernels (conv_common.hpp).
#include "conv_common.hpp"

namespace tcx {
namespace {

constexpr int X_TM = 128;                 // rows (pixels) per tile: 4 waves x 32
constexpr int X_ABYTES = X_TM * 128;      // A chunk: 128 rows x 32 channels h2
constexpr int X_BBYTES = 96 * 128;        // B chunk: 96 weight rows x 32 channels h2
constexpr int X_STAGE = X_ABYTES + X_BBYTES;
constexpr int X_WAIT_VM7 = 0x0F77;        // s_waitcnt vmcnt(7): one stage (4 + 3 DMA per wave) in flight
constexpr int X_WAIT_VM0 = 0x0F70;

__device__ __forceinline__ void x_dma16(__amdgpu_buffer_rsrc_t r, char* lds, int voff, int soff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, voff, soff, 0, 0);
}

template <bool BF>
__global__ __launch_bounds__(256, 2) void k_lin1x1(ConvParams p) {
    constexpr int NT = 3;
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
    const int m0 = mblk * X_TM, n0 = nblk * 96;
    const int nch = p.Cin / 32;
    const __amdgpu_buffer_rsrc_t ra = mk_rsrc(p.x1, p.bytes1);
    const __amdgpu_buffer_rsrc_t rw = mk_rsrc(p.w, p.bytesw);

    // DMA plan: A instructions 4 wv .. 4 wv + 3 (8 rows each), B instructions 3 wv .. 3 wv + 2
    const int lr = lane >> 3, lp = lane & 7;
    int aoff[4], boff[3];
    // b2 source (BF, p.bf == 2, h2.hpp): a 32-channel chunk is 64 B of hi halves; lane lp of a row
    // fills physical piece lp with logical piece L = lp ^ swizzle, whose hi data (L even) sits at 16 (L / 2)
    // (an odd L, a lo piece, is never read by BF: it gets the same bytes)
    const bool b2 = BF && p.bf == 2;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int r = 8 * (4 * wv + q) + lr;
        const int L = lp ^ ((r >> 1) & 7);
        aoff[q] = b2 ? (m0 + r) * p.Cin * 2 + 16 * (L >> 1) : (m0 + r) * p.Cin * 4 + 16 * L;
    }
#pragma unroll
    for (int q = 0; q < 3; ++q) {
        const int r = 8 * (3 * wv + q) + lr;
        boff[q] = (n0 + r) * p.kpad * 4 + 16 * (lp ^ ((r >> 1) & 7));
    }
    auto issue = [&](int c, int buf) {
        char* const d = smd + buf * X_STAGE;
#pragma unroll
        for (int q = 0; q < 4; ++q) x_dma16(ra, d + (4 * wv + q) * 1024, aoff[q], c * (b2 ? 64 : 128));
#pragma unroll
        for (int q = 0; q < 3; ++q) x_dma16(rw, d + X_ABYTES + (3 * wv + q) * 1024, boff[q], c * 128);
    };

    f32x16 acc[NT];
#pragma unroll
    for (int n = 0; n < NT; ++n) acc[n] = (f32x16){};
    const int ra0 = 32 * wv + li;  // this lane's A row in the tile
    auto rd = [&](int buf, int base, int r, int piece) {
        return __builtin_bit_cast(h8, *reinterpret_cast<const float4*>(smc + buf * X_STAGE + base + r * 128 +
                                                                         16 * (piece ^ ((r >> 1) & 7))));
    };

    issue(0, 0);
    if (nch > 1) issue(1, 1);
    for (int c = 0; c < nch; ++c) {
        const int buf = c & 1;
        if (c + 1 < nch) __builtin_amdgcn_s_waitcnt(X_WAIT_VM7);
        else __builtin_amdgcn_s_waitcnt(X_WAIT_VM0);
        __builtin_amdgcn_s_barrier();
        h8 ah[2], al[2], bh[2][NT], bl[2][NT];
#pragma unroll
        for (int s = 0; s < 2; ++s) {  // 16-deep k-step s: h2 group 2 s + lh of the chunk
            const int ph = 4 * s + 2 * lh;
            ah[s] = rd(buf, 0, ra0, ph);
            if (!BF) al[s] = rd(buf, 0, ra0, ph + 1);
#pragma unroll
            for (int n = 0; n < NT; ++n) {
                bh[s][n] = rd(buf, X_ABYTES, 32 * n + li, ph);
                if (!BF) bl[s][n] = rd(buf, X_ABYTES, 32 * n + li, ph + 1);
            }
        }
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            if constexpr (BF) {
#pragma unroll
                for (int n = 0; n < NT; ++n)
                    acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf8, ah[s]),
                                                                     __builtin_bit_cast(bf8, bh[s][n]), acc[n], 0, 0, 0);
            } else {
#pragma unroll
                for (int n = 0; n < NT; ++n)
                    acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[s], bl[s][n], acc[n], 0, 0, 0);
#pragma unroll
                for (int n = 0; n < NT; ++n)
                    acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[s], bh[s][n], acc[n], 0, 0, 0);
#pragma unroll
                for (int n = 0; n < NT; ++n)
                    acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[s], bh[s][n], acc[n], 0, 0, 0);
            }
        }
        if (c + 2 < nch) {
            __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's reads of `buf` are done
            __builtin_amdgcn_s_barrier();        // ... and every other wave's
            issue(c + 2, buf);
        }
    }
    __syncthreads();  // LDS -> the epilogue's reduction scratch
    conv_epilogue<NT, BF ? 2 : 1, 4>(p, acc, m0, n0, wv, tid, reinterpret_cast<double*>(sm));
}

}  // namespace

// Host dispatch (conv.hip): a plain 1x1 stride-1 conv over one h2 source, whole tiles
bool lin1x1_applies(const ConvParams& p, int cout_pad) {
    return p.ks == 1 && p.stride == 1 && p.pad_y == 0 && p.pad_x == 0 && p.Hi == p.H && p.Wi == p.W && p.C2 == 0 &&
           p.x2 == nullptr && p.Cin % 32 == 0 && p.kpad == p.Cin && cout_pad % 96 == 0 && p.M % X_TM == 0 &&
           p.HoWo % X_TM == 0 && p.osy == 1 && p.osx == 1 && p.sc1 == nullptr && p.bmod <= 0;
}

int launch_lin1x1(ConvParams& p, int cout_pad, hipStream_t st) {
    p.n_nblk = cout_pad / 96;
    if (p.M == 0) return TCX_OK;
    prof_begin(st);
    constexpr size_t shm = 2 * (size_t)X_STAGE;
    static bool attr[2] = {false, false};
    auto kc = p.bf ? &k_lin1x1<true> : &k_lin1x1<false>;
    if (!attr[p.bf ? 1 : 0]) {
        if (hipFuncSetAttribute(reinterpret_cast<const void*>(kc), hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)shm) != hipSuccess) {
            set_error("tcx_conv2d_h2: cannot enable %zu B of dynamic LDS", shm);
            return TCX_EHIP;
        }
        attr[p.bf ? 1 : 0] = true;
    }
    hipLaunchKernelGGL(kc, dim3((p.M / X_TM) * p.n_nblk), dim3(256), shm, st, p);
    const int rc = check_launch("tcx_conv2d_h2(1x1)");
    prof_end(st, 2.0 * (double)p.M * p.Cout * p.Cin);
    return rc;
}

}  // namespace tcx
