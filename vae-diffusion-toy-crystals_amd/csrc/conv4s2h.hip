// Halo-staged 4x4 stride-2 conv over h2 (split-f16) operands: the U-Net's downsamples ds1 / ds2
// (/root/reference/src/toycrystals/models/sde_score_model.py:208,210 — Conv2d(C, C, 4, stride 2,
// padding 1, circular)).
//
// The im2col kernel (conv.hip, k_conv SPL) writes every im2col element to LDS once per tap: 16
// writes per input element for a 4x4 kernel, and its ds_write_b128 traffic, not the MFMA, sets
// its pace (0.29 of the split peak on ds1/ds2).  Here, as in k_conv3h, a workgroup owns 128 output
// pixels = TR = 128/Wo whole output rows x 96 output channels and stages the (2TR+2) x (2Wo+2)
// input halo of those rows once per input-channel slice; the 16 taps read their A fragments from
// it at constant offsets.  The halo is stored column-parity deinterleaved (even input columns,
// then odd ones) so the stride-2 reads of consecutive output pixels hit consecutive halo slots:
// tap (dy, dx) of output pixel (r, c) reads slot (2r + dy) * (2Wo+2) + (dx & 1) * (Wo+1) + c + (dx >> 1).
//
// Slices are 16 input channels (one 16-deep MFMA step per tap; 64 B of h2 per halo pixel, slots
// padded to 80 B: 20*p mod 64 is distinct for every 16 consecutive slots, so ds_read_b128 of
// consecutive pixels is conflict free), so the halo (52.8 KB at Wo = 32) + a double-buffered
// weight chunk of two taps (2 x 96 x 144 B) stay under 80 KB and two workgroups share a CU.
// K order: 16-channel slice outer, tap pair inner; one barrier per tap pair (18 MFMAs per wave:
// 2 taps x NT = 3 accumulators x 3 split products).  The next slice's halo is loaded into
// registers during the current slice and stored after its last tap pair (one halo buffer).
// Epilogue shared with k_conv / k_conv3h (conv_common.hpp).
#include "conv_common.hpp"

namespace tcx {
namespace {

constexpr int DS_NW = 4;       // waves per workgroup: 128 output pixels
constexpr int DS_HROW = 20;    // floats per halo slot: 16 (h2 of 16 channels, 64 B) + 16 B pad
constexpr int DS_WROW = 36;    // floats per weight row: 2 taps x 16 (h2 of 16 channels) + 16 B pad

__host__ __device__ constexpr int ds_halo_px(int Wo) { return (2 * (128 / Wo) + 2) * (2 * Wo + 2); }
constexpr size_t ds_lds_bytes(int Wo) {
    return ((size_t)ds_halo_px(Wo) * DS_HROW + 2 * 96 * DS_WROW) * sizeof(float);
}

template <int Wo, bool CIRC, bool BF>  // BF: bf16 records, one product (h2.hpp)
__global__ __launch_bounds__(256, 2) void k_conv4s2h(ConvParams p) {
    constexpr int NT = 3;
    constexpr int NTHR = 64 * DS_NW;
    constexpr int BN = 32 * NT;
    constexpr int TR = 128 / Wo;          // output rows per tile
    constexpr int RS = 2 * Wo + 2;        // halo slots per halo row (both parities)
    constexpr int NPX = ds_halo_px(Wo);
    constexpr int HPI = (NPX * 4 + NTHR - 1) / NTHR;  // 16-B halo pieces per thread
    constexpr int BBUF = BN * DS_WROW;
    static_assert(TR * Wo == 128, "tile = whole output rows");
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float* const Hs = sm;                    // [NPX][DS_HROW]
    float* const Bs = sm + NPX * DS_HROW;    // [2][BN][DS_WROW]

    const int tid = threadIdx.x;
    const int lane = tid & 63, wv = tid >> 6, li = lane & 31, lh = lane >> 5;
    const int tile = xcd_remap(blockIdx.x, gridDim.x);
    const int mblk = tile / p.n_nblk;
    const int nblk = tile - mblk * p.n_nblk;
    const int m0 = mblk * 128, n0 = nblk * BN;
    const int b = m0 / p.HoWo;
    const int r0 = (m0 - b * p.HoWo) / Wo;  // first output row of the tile
    const int bs = p.bmod > 0 ? b % p.bmod : b;
    const int H = p.H, W = p.W;              // input dims (= 2 Ho, 2 Wo)
    const int nsl = p.Cin / 16;              // 16-channel slices
    const int nsteps = 8 * nsl;              // tap pairs

    const __amdgpu_buffer_rsrc_t r1 = mk_rsrc(p.x1, p.bytes1);
    const __amdgpu_buffer_rsrc_t rw = mk_rsrc(p.w, p.bytesw);

    // ---- halo staging plan: piece e = tid + NTHR i -> halo pixel e >> 2, 16-B piece e & 3
    const int rowb = p.C1 * 4;  // bytes per source pixel
    int hoff[HPI];
    int hdst[HPI];
#pragma unroll
    for (int i = 0; i < HPI; ++i) {
        const int e = tid + NTHR * i;
        const int hp = e >> 2;
        hoff[i] = kOOB;
        hdst[i] = -1;
        if (hp < NPX) {
            const int hr = hp / RS, hc = hp - hr * RS;
            int y = 2 * r0 + hr - 1, x = hc - 1;
            bool ok = true;
            if (CIRC) {
                y = wrap_idx(y, H);
                x = wrap_idx(x, W);
            } else {
                ok = y >= 0 && y < H && x >= 0 && x < W;
            }
            hoff[i] = ok ? ((bs * H + y) * W + x) * rowb + (e & 3) * 16 : kOOB;
            hdst[i] = (hr * RS + (hc & 1) * (Wo + 1) + (hc >> 1)) * DS_HROW + (e & 3) * 4;
        }
    }
    float4 hv[HPI];
    auto halo_load = [&](int s) {  // 16-channel slice s (uniform)
#pragma unroll
        for (int i = 0; i < HPI; ++i) hv[i] = bld4(r1, hoff[i], s * 64);
    };
    auto halo_store = [&]() {
#pragma unroll
        for (int i = 0; i < HPI; ++i)
            if ((i + 1) * NTHR <= NPX * 4 || hdst[i] >= 0)
                *reinterpret_cast<float4*>(&Hs[hdst[i]]) = hv[i];
    };
    // ---- weight staging: per tap pair, BN rows x 2 taps x 4 pieces of 16 B (8 per row)
    constexpr int BPI = (BN * 8 + NTHR - 1) / NTHR;
    float4 bv[BPI];
    int boff[BPI];
#pragma unroll
    for (int i = 0; i < BPI; ++i) {
        const int e = tid + NTHR * i;
        const int tk = (e & 7) >> 2;  // tap of the pair
        boff[i] = ((n0 + (e >> 3)) * p.kpad + tk * p.Cin) * 4 + (e & 3) * 16;
    }
    auto w_load = [&](int c) {  // step c = 8 s + u -> taps 2u, 2u+1 of slice s: k = t * Cin + 16 s
        const int s = c >> 3, u = c & 7;
        const int kb = (2 * u * p.Cin + 16 * s) * 4;
#pragma unroll
        for (int i = 0; i < BPI; ++i)
            if ((BN * 8) % NTHR == 0 || tid + NTHR * i < BN * 8) bv[i] = bld4(rw, boff[i], kb);
    };
    auto w_store = [&](int buf) {
#pragma unroll
        for (int i = 0; i < BPI; ++i) {
            const int e = tid + NTHR * i;
            if ((BN * 8) % NTHR == 0 || e < BN * 8)
                *reinterpret_cast<float4*>(&Bs[buf * BBUF + (e >> 3) * DS_WROW + (e & 7) * 4]) = bv[i];
        }
    };

    // ---- fragments
    const int mloc = wv * 32 + li;  // this lane's A row = tile pixel
    const int abase = (2 * (mloc / Wo) * RS + (mloc % Wo)) * DS_HROW + lh * 8;
    const int bbase = li * DS_WROW + lh * 8;
    f32x16 acc[NT];
#pragma unroll
    for (int n = 0; n < NT; ++n) acc[n] = (f32x16){};
    h8 a_h[2], a_l[2], b_h[2][NT], b_l[2][NT];
    auto rd_a = [&](int u) {  // taps 2u, 2u+1
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int t = 2 * u + k;
            const int dy = t >> 2, dx = t & 3;
            const float* A = &Hs[abase + (dy * RS + (dx & 1) * (Wo + 1) + (dx >> 1)) * DS_HROW];
            a_h[k] = __builtin_bit_cast(h8, ld4(A));
            a_l[k] = __builtin_bit_cast(h8, ld4(A + 4));
        }
    };
    auto rd_b = [&](int bb) {
        const float* B = &Bs[bb * BBUF + bbase];
#pragma unroll
        for (int k = 0; k < 2; ++k)
#pragma unroll
            for (int n = 0; n < NT; ++n) {
                b_h[k][n] = __builtin_bit_cast(h8, ld4(B + n * 32 * DS_WROW + 16 * k));
                b_l[k][n] = __builtin_bit_cast(h8, ld4(B + n * 32 * DS_WROW + 16 * k + 4));
            }
    };
    auto mf = [&](int k) {
        if constexpr (BF) {
#pragma unroll
            for (int n = 0; n < NT; ++n)
                acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf8, a_h[k]),
                                                                 __builtin_bit_cast(bf8, b_h[k][n]), acc[n], 0, 0, 0);
            return;
        }
#pragma unroll
        for (int n = 0; n < NT; ++n) acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a_h[k], b_l[k][n], acc[n], 0, 0, 0);
#pragma unroll
        for (int n = 0; n < NT; ++n) acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a_l[k], b_h[k][n], acc[n], 0, 0, 0);
#pragma unroll
        for (int n = 0; n < NT; ++n) acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a_h[k], b_h[k][n], acc[n], 0, 0, 0);
    };

    // ---- prologue: slice 0's halo and tap pair 0 in LDS; slice 1's halo and pair 1 in flight
    halo_load(0);
    w_load(0);
    halo_store();
    w_store(0);
    if (nsl > 1) halo_load(1);
    w_load(nsteps > 1 ? 1 : 0);
    __syncthreads();
    rd_a(0);

    for (int s = 0; s < nsl; ++s) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int c = 8 * s + u;
            const int cur = c & 1;
            rd_b(cur);
            __builtin_amdgcn_sched_barrier(0);
            mf(0);
            mf(1);
            __builtin_amdgcn_sched_barrier(0);
            w_store(cur ^ 1);  // tap pair c + 1
            __syncthreads();
            if (c + 2 < nsteps) w_load(c + 2);
            if (u < 7) {
                rd_a(u + 1);
            } else {
                // every wave is past its reads of slice s: store slice s+1 (loaded during s)
                if (s + 1 < nsl) {
                    halo_store();
                    __syncthreads();
                    if (s + 2 < nsl) halo_load(s + 2);
                }
                rd_a(0);
            }
        }
    }
    __syncthreads();  // the halo buffer becomes the epilogue's reduction scratch
    conv_epilogue<NT, BF ? 2 : 1, DS_NW>(p, acc, m0, n0, wv, tid, reinterpret_cast<double*>(sm));
}

template <int Wo>
int launch_ds(const ConvParams& p, hipStream_t st) {
    constexpr size_t shm = ds_lds_bytes(Wo);
    static bool attr[4] = {false, false, false, false};
    const int ki = (p.circular ? 1 : 0) + (p.bf ? 2 : 0);
    auto kc = p.bf ? (p.circular ? &k_conv4s2h<Wo, true, true> : &k_conv4s2h<Wo, false, true>)
                   : (p.circular ? &k_conv4s2h<Wo, true, false> : &k_conv4s2h<Wo, false, false>);
    if (!attr[ki]) {
        if (hipFuncSetAttribute(reinterpret_cast<const void*>(kc), hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)shm) != hipSuccess) {
            set_error("tcx_conv2d_h2: cannot enable %zu B of dynamic LDS", shm);
            return TCX_EHIP;
        }
        attr[ki] = true;
    }
    const int grid = (p.M / 128) * p.n_nblk;
    hipLaunchKernelGGL(kc, dim3(grid), dim3(64 * DS_NW), shm, st, p);
    return check_launch("tcx_conv2d_h2(halo 4x4/s2)");
}

}  // namespace

// Host dispatch (conv.hip): true when the stride-2 halo kernel covers this conv.
bool conv4s2h_applies(const ConvParams& p, int cout_pad) {
    return p.ks == 4 && p.stride == 2 && p.pad_y == 1 && p.pad_x == 1 && p.Hi == p.H && p.Wi == p.W &&
           (p.Wo == 16 || p.Wo == 32 || p.Wo == 64) && p.H == 2 * p.Ho && p.W == 2 * p.Wo &&
           p.HoWo % 128 == 0 && cout_pad % 96 == 0 && p.Cin % 16 == 0 && p.C2 == 0 && p.x2 == nullptr &&
           p.kpad == 16 * p.Cin && p.osy == 1 && p.osx == 1;
}

int launch_conv4s2h(ConvParams& p, int cout_pad, hipStream_t st) {
    p.n_nblk = cout_pad / 96;
    if (p.M == 0) return TCX_OK;
    prof_begin(st);
    int rc;
    if (p.Wo == 32) rc = launch_ds<32>(p, st);
    else if (p.Wo == 16) rc = launch_ds<16>(p, st);
    else rc = launch_ds<64>(p, st);
    prof_end(st, 2.0 * (double)p.M * p.Cout * 16 * p.Cin);
    return rc;
}

}  // namespace tcx
