// "h2" split-f16 storage of an fp32 tensor, the operand format of the f16x3 conv path.
//
// A tensor [..][C] (C % 8 == 0) is stored as [..][C/8][2][8] f16: for every 8-channel group,
// 8 "hi" halves then 8 "lo" halves, hi = f16(v), lo = f16(v - hi) (both round-to-nearest-even).
// Four bytes per element, so every byte offset of the fp32 layout that is a multiple of 32
// (a pixel, an 8-channel group) is unchanged and the im2col gather of the conv is the same code.
// hi + lo carries 22 significant bits (f16 subnormals are kept by the gfx950 converts and MFMA,
// measured: tools/probe/mfma_f16_probe.hip), and a product a*b is formed on MFMA as
// hi_a*hi_b + hi_a*lo_b + lo_a*hi_b (three v_mfma_f32_32x32x16_f16, f32 accumulate): the dropped
// lo*lo term and the split residuals are below 2^-21 relative, within the fp32 rounding of the
// K-long accumulation.  Weights are scaled by an exact power of two before the
// split so that their lo halves stay normal; the epilogue multiplies by the inverse.
// Range: |v| must stay below 65504 (f16 max); writers raise a flag word otherwise (the host
// re-runs in fp32: toycrystals_amd/models/sde_score_model.py).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace tcx {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));

constexpr float kH2Max = 65504.f;

__device__ __forceinline__ unsigned short f16_bits(_Float16 h) { return __builtin_bit_cast(unsigned short, h); }

// split one value: returns (lo << 16) | hi
__device__ __forceinline__ unsigned split1(float v) {
    const _Float16 h = (_Float16)v;
    const _Float16 l = (_Float16)(v - (float)h);
    return (unsigned)f16_bits(h) | ((unsigned)f16_bits(l) << 16);
}

// 4 consecutive channels -> 4 hi halves (uint2) and 4 lo halves (uint2)
__device__ __forceinline__ void split4(const float4 v, uint2& hi, uint2& lo) {
    const unsigned a = split1(v.x), b = split1(v.y), c = split1(v.z), d = split1(v.w);
    hi.x = (a & 0xffffu) | (b << 16);
    hi.y = (c & 0xffffu) | (d << 16);
    lo.x = (a >> 16) | (b & 0xffff0000u);
    lo.y = (c >> 16) | (d & 0xffff0000u);
}

// bf16 single-product mode (the "bf16" precision of the score U-Net evaluator, config 5): the same
// record layout with hi = bf16(v) (round to nearest even) and lo = bf16(v - hi); consumers multiply
// the hi halves only (one v_mfma_f32_32x32x16_bf16 per product), weights unscaled.  bf16 has the
// fp32 exponent range, so nothing overflows.
typedef __bf16 bf8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ unsigned short bf16_bits(__bf16 h) { return __builtin_bit_cast(unsigned short, h); }

__device__ __forceinline__ unsigned split1_bf(float v) {
    const __bf16 h = (__bf16)v;
    const __bf16 l = (__bf16)(v - (float)h);
    return (unsigned)bf16_bits(h) | ((unsigned)bf16_bits(l) << 16);
}

// either split, by a uniform flag (writers; HBM-bound, so the branch is free)
__device__ __forceinline__ unsigned split1x(float v, bool bf) { return bf ? split1_bf(v) : split1(v); }

__device__ __forceinline__ void split4x(const float4 v, uint2& hi, uint2& lo, bool bf) {
    const unsigned a = split1x(v.x, bf), b = split1x(v.y, bf), c = split1x(v.z, bf), d = split1x(v.w, bf);
    hi.x = (a & 0xffffu) | (b << 16);
    hi.y = (c & 0xffffu) | (d << 16);
    lo.x = (a >> 16) | (b & 0xffff0000u);
    lo.y = (c >> 16) | (d & 0xffff0000u);
}

__device__ __forceinline__ void store4_h2x(char* base, size_t pix, int q, const float4 v, bool bf) {
    uint2 hi, lo;
    split4x(v, hi, lo, bf);
    char* g = base + pix + 32 * (size_t)(q >> 1) + 8 * (q & 1);
    *reinterpret_cast<uint2*>(g) = hi;
    *reinterpret_cast<uint2*>(g + 16) = lo;
}

// "b2": config 5's 2-byte bf16 tensors (bf = 2 in the conv / writer flags): plain NHWC bf16 (round to
// nearest even), i.e. only the hi halves of the bf16 records above.  A bf16 product never reads the lo
// halves, so every record reader's byte offset of a hi piece is halved: pixel p, 8-channel group g at
// p C 2 + 16 g (records: p C 4 + 32 g).
__device__ __forceinline__ unsigned pack2_bf(float a, float b) {
    return (unsigned)bf16_bits((__bf16)a) | ((unsigned)bf16_bits((__bf16)b) << 16);
}
// channels [4q, 4q+4) of the pixel whose b2 row starts at element `pix_elem` (= pixel * C)
__device__ __forceinline__ void store4_b2(char* base, size_t pix_elem, int q, const float4 v) {
    *reinterpret_cast<uint2*>(base + (pix_elem + 4 * (size_t)q) * 2) = make_uint2(pack2_bf(v.x, v.y), pack2_bf(v.z, v.w));
}
__device__ __forceinline__ float bf_lo(unsigned w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bf_hi(unsigned w) { return __uint_as_float(w & 0xffff0000u); }

__device__ __forceinline__ bool h2_bad(float v) { return !(fabsf(v) < kH2Max); }

// Store channels [4q, 4q+4) of one pixel whose h2 record starts at byte `pix` (= pixel * C * 4).
__device__ __forceinline__ void store4_h2(char* base, size_t pix, int q, const float4 v) {
    uint2 hi, lo;
    split4(v, hi, lo);
    char* g = base + pix + 32 * (size_t)(q >> 1) + 8 * (q & 1);
    *reinterpret_cast<uint2*>(g) = hi;
    *reinterpret_cast<uint2*>(g + 16) = lo;
}

// Raise the overflow flag (rare: a plain per-lane atomic on the taken branch only).  The pointer is
// cast to the global address space so the atomic is one global_atomic_or: on a generic pointer the
// compiler expands it into a run-time LDS / scratch / global address-space switch (whose LDS-aperture
// compare it could not encode inside the k_conv3lg tap loop).
__device__ __forceinline__ void h2_flag(unsigned* ovf, bool bad) {
    if (bad && ovf)
        __hip_atomic_fetch_or((__attribute__((address_space(1))) unsigned*)ovf, 1u, __ATOMIC_RELAXED,
                              __HIP_MEMORY_SCOPE_AGENT);
}

// Decode 4 channels [4q, 4q+4) of one pixel record (tests / conversions).
__device__ __forceinline__ float4 load4_h2(const char* base, size_t pix, int q) {
    const char* g = base + pix + 32 * (size_t)(q >> 1) + 8 * (q & 1);
    const uint2 hi = *reinterpret_cast<const uint2*>(g);
    const uint2 lo = *reinterpret_cast<const uint2*>(g + 16);
    auto f = [](unsigned h, unsigned l) {
        return (float)__builtin_bit_cast(_Float16, (unsigned short)h) + (float)__builtin_bit_cast(_Float16, (unsigned short)l);
    };
    return make_float4(f(hi.x & 0xffffu, lo.x & 0xffffu), f(hi.x >> 16, lo.x >> 16), f(hi.y & 0xffffu, lo.y & 0xffffu),
                       f(hi.y >> 16, lo.y >> 16));
}

}  // namespace tcx
