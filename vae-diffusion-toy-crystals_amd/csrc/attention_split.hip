// f16x3 split flash attention for the split-precision U-Net evaluator: the bottleneck
// self-attention of SelfAttention2d (/root/reference/src/toycrystals/models/sde_score_model.py:
// 136-167, softmax(q k^T / sqrt(d)) v per (batch, head) over N = H*W tokens) with qkv and the
// output in h2 storage (h2.hpp), both products on v_mfma_f32_32x32x16_f16: 3 MFMAs per fp32
// product (hi*lo + lo*hi + hi*hi, f32 accumulation) at 16x the fp32 MFMA rate.
//
// Same key-tiled online softmax as k_attention_flash (attention.hip):
//   S^T = K Q^T : A = K rows (key = lane, the 8 dims of step s on lane half h) read from LDS as
//                 one hi and one lo b128; B = Q^T fragments held in registers (query on the lane).
//   P           : the S accumulators (query on the lane, keys (r&3)+8(r>>2)+4h of a 32-key
//                 subtile) are exponentiated, scaled by 2^10 (so p >= 2^-24 keeps its lo half out
//                 of the f16 subnormal range) and split; register r = 8s+e of step s is k-slot 8h+e.
//   O^T = V^T P^T: A = V^T, staged TRANSPOSED in LDS as [d][slot] hi / lo f16 rows with keys
//                 permuted into the slot order above (slot 16s+8h+e <-> key 16s+8(e>>2)+4h+(e&3)),
//                 so a lane's 8 k-slots are one b128 read.  D = 48 pads O^T to 64 rows (zero V).
// Per 128-key tile: K rows copied (h2 as is), V transposed with b32 writes (two keys per dword).
// The output is a convex combination of V rows, so |O| <= max|V| < 65504: no range flag.
#include "common.hpp"
#include "h2.hpp"

namespace tcx {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef unsigned u4 __attribute__((ext_vector_type(4)));

// tile load (global -> registers) and store (registers -> LDS stage, V transposed) of the kernel below
#define TCX_ATT_LOAD_R(k0, kreg, vreg) \
    do { \
_Pragma("unroll") \
        for (int u = 0; u < KI; ++u) {  /* BF: the hi pieces only (global piece 2 pc) */ \
            /* PF2: unconditional (ragged threads reload the last piece): no branch, exact vmcnt counts */ \
            const int i = PF2 ? min(tid + 512 * u, KT * KPL - 1) : tid + 512 * u; \
            const int j = i / KPL, pc = i - (i / KPL) * KPL; \
            if (PF2 || KT * KPL % 512 == 0 || i < KT * KPL) \
                kreg[u] = *reinterpret_cast<const f4*>(base + (size_t)(k0 + j) * rs + (size_t)(C + h * D) * ESZ + \
                                                       (B2 ? pc : BF ? 2 * pc : pc) * 16); \
        } \
_Pragma("unroll") \
        for (int u = 0; u < VI; ++u) { \
            const int i = PF2 ? min(tid + 512 * u, (KT / 2) * G - 1) : tid + 512 * u; \
            if (PF2 || i < (KT / 2) * G) { \
                const int g = i / (KT / 2), jp = i - g * (KT / 2);  /* key pair (2 jp, 2 jp + 1), dim group g */ \
                const char* src = base + (size_t)(k0 + 2 * jp) * rs + (size_t)(2 * C + h * D) * ESZ + g * 8 * ESZ; \
                vreg[u][0] = *reinterpret_cast<const u4*>(src); \
                if (!BF) vreg[u][1] = *reinterpret_cast<const u4*>(src + 16); \
                vreg[u][2] = *reinterpret_cast<const u4*>(src + rs); \
                if (!BF) vreg[u][3] = *reinterpret_cast<const u4*>(src + rs + 16); \
            } \
        } \
    } while (0)
#define TCX_ATT_STORE_R(st, kreg, vreg) \
    do { \
        char* Ks = Kb(st); \
        unsigned* Vh = Vhb(st); \
        unsigned* Vl = Vlb(st); \
_Pragma("unroll") \
        for (int u = 0; u < KI; ++u) { \
            const int i = tid + 512 * u; \
            const int j = i / KPL, pc = i - (i / KPL) * KPL; \
            if (KT * KPL % 512 == 0 || i < KT * KPL) *reinterpret_cast<f4*>(Ks + j * KSB + pc * 16) = kreg[u]; \
        } \
_Pragma("unroll") \
        for (int u = 0; u < VI; ++u) { \
            const int i = tid + 512 * u; \
            if (i < (KT / 2) * G) { \
                const int g = i / (KT / 2), jp = i - g * (KT / 2); \
                const int j = 2 * jp; \
                /* slot of key j within its subtile: kk = 16s + 8(e>>2) + 4h + (e&3) -> 16s + 8h + e */ \
                const int kk = j & 31, rem = kk & 15; \
                const int slot = (j & ~31) + (kk & 16) + 8 * ((rem >> 2) & 1) + ((rem & 3) | ((rem >> 3) << 2)); \
                const int col = slot >> 1;  /* j even -> slot even; key j + 1 takes slot + 1 */ \
                const u4 h0 = vreg[u][0], l0 = vreg[u][1], h1 = vreg[u][2], l1 = vreg[u][3]; \
_Pragma("unroll") \
                for (int e = 0; e < 8; ++e) { \
                    const int sh = 16 * (e & 1); \
                    const unsigned a = (h0[e >> 1] >> sh) & 0xffffu, c = (h1[e >> 1] >> sh) & 0xffffu; \
                    const unsigned al = (l0[e >> 1] >> sh) & 0xffffu, cl = (l1[e >> 1] >> sh) & 0xffffu; \
                    Vh[(g * 8 + e) * VSW + col] = a | (c << 16); \
                    if (!BF) Vl[(g * 8 + e) * VSW + col] = al | (cl << 16); \
                } \
            } \
        } \
    } while (0)

#define TCX_ATT_LOAD(k0) TCX_ATT_LOAD_R(k0, kreg, vreg)
#define TCX_ATT_STORE(st) TCX_ATT_STORE_R(st, kreg, vreg)

// staged K row: h2 pieces (D * 4 B), or for BF only the hi pieces (D * 2 B: the lo halves of K and V are
// never loaded), + 16 B pad (both strides an odd number of 16-B units: conflict-free b128 row reads)
__host__ __device__ constexpr int attn_ksb(int D, bool BF) { return (BF ? D * 2 : D * 4) + 16; }

// FMT 0: h2 records; 1 (BF): bf16 records (h2.hpp), one v_mfma_f32_32x32x16_bf16 (hi x hi) per product,
// P in bf16; 2 (BF, B2): the same on 2-byte bf16 qkv and output (h2.hpp "b2": the records' hi halves)
// XCD-aware workgroup order (round 6, TCX_ATTN_XCD=0: off): the hardware deals consecutive workgroups to the
// 8 XCDs round-robin, so the N / 256 query blocks of one (image, head) — which all stream the same K / V
// rows — were spread over every XCD's L2 and each fetched the (image, head)'s K / V from HBM (config 5:
// 1,711 MB read per launch for 302 MB of qkv, profiles/r05_t_cfg5_pmc_traffic.txt).  With xcd_remap the
// query blocks of an (image, head), and the heads of an image (whose K / V share cache lines of the token
// rows), run on one XCD at about the same time.
// PF2 (bf16 forms at N >= 512; TCX_ATTN_PF2=0: off): a second register set, so each key tile's global loads
// are issued two tiles before its LDS store instead of one.  The loop is unrolled by two so both sets are
// static registers and its loads / stores unconditional (the last trip reloads the last tile: no compiler
// vmcnt(0) at control-flow joins), which leaves the previous tile's loads in flight across a whole tile.
template <int D, int FMT, bool PF2 = false>
__global__ __launch_bounds__(512) void k_attention_split(const char* __restrict__ qkv, char* __restrict__ out, int N,
                                                         int C, float scale, int xcd, float defer2) {
    constexpr bool BF = FMT >= 1, B2 = FMT == 2;
    static_assert(!PF2 || BF, "the two-deep prefetch is bf16 only");
    constexpr int ESZ = B2 ? 2 : 4;  // bytes per element of qkv / out
    static_assert(D % 16 == 0 && D <= 64, "split attention: head dim multiple of 16, <= 64");
    constexpr int KT = 128;            // keys per staged tile
    constexpr int NST = KT / 32;       // 32-key subtiles
    constexpr int DS = D / 16;         // 16-deep steps of Q.K
    constexpr int DT = (D + 31) / 32;  // 32-row tiles of O^T
    constexpr int DP = DT * 32;
    constexpr int KSB = attn_ksb(D, BF);  // bytes per staged key row (h2, or BF: hi pieces) + 16 B pad
    constexpr int VSW = KT / 2 + 4;    // dwords per V^T row (two f16 slots each) + 16 B pad
    // two LDS stages (tile t computed from one while tile t+1, loaded into registers during that
    // compute, is written to the other): [2][K | V^T hi | V^T lo]
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int STAGE = KT * KSB + 2 * DP * VSW * 4;
    int b = blockIdx.z, h = blockIdx.y, qb = blockIdx.x;
    if (xcd) {
        const int nq = gridDim.x, nh = gridDim.y;
        const int flat = blockIdx.x + nq * (blockIdx.y + nh * blockIdx.z);
        const int t = xcd_remap(flat, nq * nh * gridDim.z);
        qb = t % nq;
        h = (t / nq) % nh;
        b = t / (nq * nh);
    }
    const int tid = threadIdx.x;
    const size_t rs = 3 * ESZ * (size_t)C;  // bytes per token row of qkv (3C channels)
    const char* base = qkv + (size_t)b * N * rs;
    const int lane = tid & 63, w = tid >> 6;
    const int li = lane & 31, lh = lane >> 5;
    const int q = qb * 256 + w * 32 + li;
    const float scale2 = scale * 1.4426950408889634f;  // log2(e) / sqrt(D)
    h8 qh[DS], ql[DS];
    {
        const char* qr = base + (size_t)q * rs + (size_t)h * D * ESZ;
#pragma unroll
        for (int s = 0; s < DS; ++s) {
            qh[s] = *reinterpret_cast<const h8*>(qr + (2 * s + lh) * 8 * ESZ);
            if constexpr (!BF) ql[s] = *reinterpret_cast<const h8*>(qr + (2 * s + lh) * 32 + 16);
        }
    }
    auto Kb = [&](int st) { return smem + st * STAGE; };
    auto Vhb = [&](int st) { return reinterpret_cast<unsigned*>(smem + st * STAGE + KT * KSB); };
    auto Vlb = [&](int st) { return reinterpret_cast<unsigned*>(smem + st * STAGE + KT * KSB + DP * VSW * 4); };
    // ONES (bf16, D < DP): V^T row D, a padding row of the PV product, is all ones, so
    // O^T row D accumulates the row sum of P on the MFMA, rescaled with O by the online softmax: no
    // VALU adds for l (they were a fifth of the softmax VALU, which bounds this loop)
    constexpr bool ONES = BF && DP > D;  // measured: 256^2 bf16 1390 -> 1313 us; the f16x3 form at N = 256 (two key tiles) lost 7 %
    constexpr unsigned ONE2 = 0x3F803F80u;  // two bf16 ones per dword
    if (DP > D) {
        for (int i = tid; i < (DP - D) * VSW; i += 512) {
#pragma unroll
            for (int st = 0; st < 2; ++st) {
                Vhb(st)[D * VSW + i] = ONES && i < VSW ? ONE2 : 0u;
                Vlb(st)[D * VSW + i] = 0u;
            }
        }
    }
    f32x16 oacc[DT];
#pragma unroll
    for (int t = 0; t < DT; ++t) oacc[t] = (f32x16){};
    float m = -INFINITY, l = 0.f;
    constexpr int KP = D / 4;  // 16-B pieces per K row
    constexpr int KPL = BF ? KP / 2 : KP;  // pieces staged per K row (BF: the hi pieces)
    constexpr int G = D / 8;   // 8-dim groups per V row
    constexpr int KI = (KT * KPL + 511) / 512;       // K pieces per thread (guarded when ragged)
    constexpr int VI = ((KT / 2) * G + 511) / 512;   // V (key pair, dim group) items per thread
    f4 kreg[KI];        // native vectors: arrays of HIP's float4/uint4 structs stayed in scratch here
    u4 vreg[VI][4];
    f4 kreg2[PF2 ? KI : 1];  // PF2: the second set
    u4 vreg2[PF2 ? VI : 1][4];
    const int ntile = N / KT;
    // one key tile's math from LDS stage cur
    auto step = [&](const int cur) {
        const char* Ks = Kb(cur);
        const unsigned* Vh = Vhb(cur);
        const unsigned* Vl = Vlb(cur);
        f32x16 sacc[NST];
#pragma unroll
        for (int n = 0; n < NST; ++n) {
            sacc[n] = (f32x16){};
            const char* kr = Ks + (n * 32 + li) * KSB;
#pragma unroll
            for (int s = 0; s < DS; ++s) {
                const h8 kh = *reinterpret_cast<const h8*>(kr + (2 * s + lh) * (BF ? 16 : 32));
                if constexpr (BF) {
                    sacc[n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf8, kh),
                                                                      __builtin_bit_cast(bf8, qh[s]), sacc[n], 0, 0, 0);
                    continue;
                }
                const h8 kl = *reinterpret_cast<const h8*>(kr + (2 * s + lh) * 32 + 16);
                sacc[n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(kh, ql[s], sacc[n], 0, 0, 0);
                sacc[n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(kl, qh[s], sacc[n], 0, 0, 0);
                sacc[n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(kh, qh[s], sacc[n], 0, 0, 0);
            }
        }
        // row max and row sum as NST independent chains combined at the end (one 64-long dependent
        // chain per lane left the two waves per SIMD stalled on VALU latency)
        float mtn[NST];
#pragma unroll
        for (int n = 0; n < NST; ++n) {
            mtn[n] = sacc[n][0];
#pragma unroll
            for (int r = 1; r < 16; ++r) mtn[n] = fmaxf(mtn[n], sacc[n][r]);
        }
        float mt = mtn[0];
#pragma unroll
        for (int n = 1; n < NST; ++n) mt = fmaxf(mt, mtn[n]);
        mt = fmaxf(mt, __shfl_xor(mt, 32));
        // bf16: the running max is deferred (FA4-style) -- the offset m moves only when the tile's max passes it
        // by more than defer2 in log2 units of p, so p <= 2^(10 + defer2) (2^18: fp32 / bf16 range to spare, the
        // softmax exact for any offset) and the O rescale below runs on a handful of tiles instead of most of
        // them; defer2 = 0 is the exact running max
        const float mn = BF ? ((mt - m) * scale2 > defer2 ? mt : m) : fmaxf(m, mt);
        // exponentials as hardware exp2 of pre-scaled logits (v_exp_f32; the VALU of the
        // softmax, not the MFMA, bounds this loop)
        const float alpha = __builtin_amdgcn_exp2f((m - mn) * scale2);  // 0 on the first tile (m = -inf)
        const float mb = fmaf(-mn, scale2, 10.f);  // + 10: p is produced pre-scaled by 2^10
        m = mn;
        if constexpr (!ONES) l *= alpha;
        // bf16 (N = 4,096: 32 key tiles): rescale only when some lane's running max moved (x 1 is exact;
        // after the first tiles the max rarely moves, and the 32 multiplies per tile are VALU the loop
        // is bound by)
        if (!BF || __builtin_amdgcn_ballot_w64(alpha != 1.f) != 0) {
#pragma unroll
            for (int t = 0; t < DT; ++t)
#pragma unroll
                for (int r = 0; r < 16; ++r) oacc[t][r] *= alpha;
        }
        float ltn[NST];
#pragma unroll
        for (int n = 0; n < NST; ++n) {
            float& lt = ltn[n];
            lt = 0.f;
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                const int c0 = (n * 32 + 16 * s + 8 * lh) >> 1;
                if constexpr (BF) {
                    bf8 pb;
#pragma unroll
                    for (int e = 0; e < 8; ++e) {
                        const float v = __builtin_amdgcn_exp2f(fmaf(sacc[n][8 * s + e], scale2, mb));
                        if constexpr (!ONES) lt += v;
                        pb[e] = (__bf16)v;
                    }
#pragma unroll
                    for (int t = 0; t < DT; ++t) {
                        const h8 vh = *reinterpret_cast<const h8*>(&Vh[(t * 32 + li) * VSW + c0]);
                        oacc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf8, vh), pb, oacc[t], 0,
                                                                          0, 0);
                    }
                    continue;
                }
                h8 ph, pl;
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    const float v = __builtin_amdgcn_exp2f(fmaf(sacc[n][8 * s + e], scale2, mb));
                    if constexpr (!ONES) lt += v;  // l, like the P operand, carries the 2^10 scale
                    const _Float16 hh = (_Float16)v;
                    ph[e] = hh;
                    pl[e] = (_Float16)(v - (float)hh);
                }
#pragma unroll
                for (int t = 0; t < DT; ++t) {
                    const h8 vh = *reinterpret_cast<const h8*>(&Vh[(t * 32 + li) * VSW + c0]);
                    const h8 vl = *reinterpret_cast<const h8*>(&Vl[(t * 32 + li) * VSW + c0]);
                    oacc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(vh, pl, oacc[t], 0, 0, 0);
                    oacc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(vl, ph, oacc[t], 0, 0, 0);
                    oacc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(vh, ph, oacc[t], 0, 0, 0);
                }
            }
        }
        if constexpr (!ONES) {
            float lt = ltn[0];
#pragma unroll
            for (int n = 1; n < NST; ++n) lt += ltn[n];
            lt += __shfl_xor(lt, 32);
            l += lt;
        }
    };
    TCX_ATT_LOAD(0);
    TCX_ATT_STORE(0);
    if constexpr (PF2) {
        // ntile even (N % 256 == 0), >= 4; set A carries even tiles, set B odd ones
        TCX_ATT_LOAD_R(KT, kreg2, vreg2);
        __syncthreads();
        for (int tt = 0; tt < ntile; tt += 2) {
            TCX_ATT_LOAD_R(min(tt + 2, ntile - 1) * KT, kreg, vreg);  // set A was stored at the end of tile tt - 1
            step(0);
            TCX_ATT_STORE_R(1, kreg2, vreg2);  // tile tt + 1 (loaded during tile tt - 1) into the stage tile tt - 1 left
            __syncthreads();
            TCX_ATT_LOAD_R(min(tt + 3, ntile - 1) * KT, kreg2, vreg2);
            step(1);
            TCX_ATT_STORE_R(0, kreg, vreg);  // tile tt + 2 (the last trip: a reload, never read)
            __syncthreads();
        }
    } else {
        __syncthreads();
        for (int tt = 0; tt < ntile; ++tt) {
            const int cur = tt & 1;
            if (tt + 1 < ntile) TCX_ATT_LOAD((tt + 1) * KT);  // in flight during this tile's math
            step(cur);
            if (tt + 1 < ntile) TCX_ATT_STORE(cur ^ 1);  // that stage was last read in tile tt - 1
            __syncthreads();
        }
    }
    if constexpr (ONES) {
        // row D of O^T: tile D / 32, register 4 ((D % 32) / 8) + (D % 4), held by the lanes of half
        // ((D % 8) / 4) (= 0 for D % 8 == 0); the other half takes it across the wave
        constexpr int TD = D / 32, RD = 4 * ((D % 32) / 8) + (D % 4);
        static_assert(D % 8 == 0, "ONES: the sum row must sit in lane half 0");
        const float own = oacc[TD][RD];
        const float other = __shfl_xor(own, 32);
        l = lh == 0 ? own : other;
    }
    const float inv = 1.f / l;
#pragma unroll
    for (int t = 0; t < DT; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int d = t * 32 + 8 * i + 4 * lh;
            if (d < D) {
                const float4 v = make_float4(oacc[t][4 * i] * inv, oacc[t][4 * i + 1] * inv, oacc[t][4 * i + 2] * inv,
                                             oacc[t][4 * i + 3] * inv);
                if constexpr (B2) store4_b2(out, ((size_t)b * N + q) * C, (h * D + d) >> 2, v);
                else store4_h2x(out, ((size_t)b * N + q) * C * 4, (h * D + d) >> 2, v, BF);
            }
        }
}

template <int D, int FMT, bool PF2>
int launch_split_v(const void* qkv, void* out, int Bt, int N, int C, int heads, hipStream_t st) {
    const float scale = (float)(1.0 / std::sqrt((double)D));
    constexpr int DP = (D + 31) / 32 * 32;
    constexpr size_t shm = 2 * ((size_t)128 * attn_ksb(D, FMT >= 1) + 2 * (size_t)DP * (128 / 2 + 4) * 4);
    static bool attr_set = false;
    if (!attr_set) {
        if (hipFuncSetAttribute(reinterpret_cast<const void*>(&k_attention_split<D, FMT, PF2>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm) != hipSuccess) {
            set_error("tcx_attention_split: cannot enable %zu B of dynamic LDS", shm);
            return TCX_EHIP;
        }
        attr_set = true;
    }
    static const int xcd = [] {
        const char* e = getenv("TCX_ATTN_XCD");
        return (e && e[0] == '0') ? 0 : 1;
    }();
    static const float defer2 = [] {  // TCX_ATTN_DEFER: deferred-max threshold (log2 units; 0 = exact running max)
        const char* e = getenv("TCX_ATTN_DEFER");
        return e ? std::max(0.f, std::min(16.f, (float)atof(e))) : 8.f;
    }();
    hipLaunchKernelGGL((k_attention_split<D, FMT, PF2>), dim3(N / 256, heads, Bt), dim3(512), shm, st, (const char*)qkv,
                       (char*)out, N, C, scale, xcd, defer2);
    return check_launch("tcx_attention_split");
}

template <int D, int FMT>
int launch_split(const void* qkv, void* out, int Bt, int N, int C, int heads, hipStream_t st) {
    if constexpr (FMT >= 1) {
        static const bool pf2 = [] {
            const char* e = getenv("TCX_ATTN_PF2");
            return !(e && e[0] == '0');
        }();
        if (pf2 && N >= 4 * 128) return launch_split_v<D, FMT, true>(qkv, out, Bt, N, C, heads, st);
    }
    return launch_split_v<D, FMT, false>(qkv, out, Bt, N, C, heads, st);
}

#undef TCX_ATT_LOAD
#undef TCX_ATT_STORE
#undef TCX_ATT_LOAD_R
#undef TCX_ATT_STORE_R

}  // namespace
}  // namespace tcx

using namespace tcx;

namespace tcx {
int attention_split(const void* qkv, void* out, int Bt, int N, int C, int heads, int bf, hipStream_t st) {
    TCX_REQUIRE(qkv && out && heads > 0 && C % heads == 0, "tcx_attention_split: bad args");
    TCX_REQUIRE(N > 0 && N % 256 == 0, "tcx_attention_split: needs N %% 256 == 0");
    TCX_REQUIRE(aligned16(qkv) && aligned16(out), "tcx_attention_split: pointers must be 16-B aligned");
    if (Bt == 0) return TCX_OK;
#define TCX_ATT_D(D_)                                                                        \
    case D_:                                                                                 \
        return bf == 2 ? launch_split<D_, 2>(qkv, out, Bt, N, C, heads, st)                 \
             : bf ? launch_split<D_, 1>(qkv, out, Bt, N, C, heads, st)                      \
                  : launch_split<D_, 0>(qkv, out, Bt, N, C, heads, st);
    switch (C / heads) {
        TCX_ATT_D(16)
        TCX_ATT_D(32)
        TCX_ATT_D(48)
        TCX_ATT_D(64)
        default:
            set_error("tcx_attention_split: head dim %d unsupported (16, 32, 48, 64)", C / heads);
            return TCX_EUNSUP;
    }
#undef TCX_ATT_D
}
}  // namespace tcx

extern "C" int tcx_attention_split(const void* qkv, void* out, int Bt, int N, int C, int heads, void* stream) {
    return attention_split(qkv, out, Bt, N, C, heads, 0, (hipStream_t)stream);
}

extern "C" int tcx_attention_split_bf16(const void* qkv, void* out, int Bt, int N, int C, int heads, void* stream) {
    return attention_split(qkv, out, Bt, N, C, heads, 1, (hipStream_t)stream);
}

extern "C" int tcx_attention_split_b2(const void* qkv, void* out, int Bt, int N, int C, int heads, void* stream) {
    return attention_split(qkv, out, Bt, N, C, heads, 2, (hipStream_t)stream);
}
