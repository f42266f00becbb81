// Shared helpers for libtcx (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>

#include "../../include/tcx.h"

namespace tcx {

void set_error(const char* fmt, ...);

// Live kernel timing for the roofline (bench.py): when enabled by tcx_prof_enable, every
// implicit-GEMM conv launch is bracketed by a pair of HIP events on its own stream; elapsed
// times and algorithmic FLOPs are accumulated through a ring of event pairs (the host only waits
// on a pair when the ring wraps, i.e. ~thousands of launches behind the GPU).
void prof_begin(hipStream_t st);
void prof_end(hipStream_t st, double flops);

inline int check_launch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("%s: %s", what, hipGetErrorString(e));
        return TCX_EHIP;
    }
    return TCX_OK;
}

#define TCX_REQUIRE(cond, ...)                \
    do {                                      \
        if (!(cond)) {                        \
            ::tcx::set_error(__VA_ARGS__);    \
            return TCX_EINVAL;                \
        }                                     \
    } while (0)

#define TCX_TRY(expr)                \
    do {                             \
        int _rc = (expr);            \
        if (_rc != TCX_OK) return _rc; \
    } while (0)

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

inline int cdiv(int a, int b) { return (a + b - 1) / b; }
inline size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

// Bijective XCD-aware remap of a linear workgroup id (cdna_hip_programming.md §5.5 T1):
// consecutive logical tiles land on the same XCD (blocks b and b+8 share one), so tiles that
// share input rows / weights share that XCD's L2.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
    const int q = nwg >> 3, r = nwg & 7, xcd = orig & 7;
    const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
    return base + (orig >> 3);
}

__device__ __forceinline__ float silu_f(float v) { return v / (1.0f + expf(-v)); }
// SiLU on the hardware exp2 / reciprocal (a few ulp from silu_f), as the conv prologues, the head and
// the first-conv records compute it: the IEEE expf + division form is ~25 VALU per element
__device__ __forceinline__ float silu_hw(float v) {
    return v * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-1.4426950408889634f * v));
}

__device__ __forceinline__ float absmax4(const float4 v) {
    return fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w)));
}
// Block-reduce a per-thread max |value| (>= 0; 256-thread blocks) and raise *amax (the bit pattern of
// a non-negative float, ordered like the value) with ONE vector-memory atomic per workgroup: same-address
// atomics serialise in one L2 channel, so a launch must keep them to a few thousand (one per wave of a
// 16k-workgroup grid cost milliseconds).  Every thread of the block must call it.
__device__ __forceinline__ void block_amax_publish(float m, unsigned* amax) {
    __shared__ float red[4];
    for (int o = 32; o; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) atomicMax(amax, __float_as_uint(fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]))));
}
// SiLU with the hardware exp2 / reciprocal (a few ulp; used in staged prologues)

// Call first thing in an MFMA kernel: an AGPR reference keeps hipcc from proving the kernel AGPR-free,
// so it selects the AGPR form of the MFMAs (accumulators in AGPRs, fragments in VGPRs).  Round 4 added
// it to k_conv3m while chasing wrong sums under co-run (r04_n), suspecting the all-VGPR form's reuse of
// a moved accumulator's old SrcC register as a load destination; the cause was the store-data hazard
// (conv_common.hpp store_b128_guarded).  k_conv3m runs the all-VGPR form again since round 5 (equal
// speed, co-run / lane tests green without it, profiles/r05_c_*); the skinny prior GEMMs keep it.
// tools/mfma_war_check.py lists the SrcC-reuse sites of a .s.
__device__ __forceinline__ void mfma_agpr_form() { asm volatile("" ::: "a0"); }

__device__ __forceinline__ int wrap_idx(int i, int n) {
    i = i < 0 ? i + n : i;
    return i >= n ? i - n : i;
}

__device__ inline void gn_tables_from_csum(int C, int groups, int HW, const float* __restrict__ gamma,
                                           const float* __restrict__ beta, float eps, float* sc, float* sh,
                                           double* gstat, const double* csum);
// Per-channel scale/shift of batch b into LDS from the partials [b][nsplit][C][2].
// Stage 1: one thread per channel sums its nsplit partials (independent, coalesced loads);
// stage 2: one thread per group sums its cpg channel totals.  (A group-per-thread loop over
// nsplit*cpg dependent loads was ~80 us of serialised latency per block.)
__device__ inline void gn_scale_shift(const double* __restrict__ part, int b, int nsplit, int C, int groups, int HW,
                               const float* __restrict__ gamma, const float* __restrict__ beta, float eps,
                               float* sc, float* sh, double* gstat, double* csum) {
    const int tid = threadIdx.x;
    const double* pb = part + (size_t)b * nsplit * C * 2;
    for (int c = tid; c < C; c += blockDim.x) {
        double a = 0, q = 0;
#pragma unroll 8
        for (int sp = 0; sp < nsplit; ++sp) {
            const double2 v = *reinterpret_cast<const double2*>(pb + ((size_t)sp * C + c) * 2);
            a += v.x;
            q += v.y;
        }
        csum[2 * c] = a;
        csum[2 * c + 1] = q;
    }
    __syncthreads();
    gn_tables_from_csum(C, groups, HW, gamma, beta, eps, sc, sh, gstat, csum);
}

// Stages 2-3 of gn_scale_shift: per-channel totals csum[C][2] (LDS) -> group mean / rstd -> tables.
__device__ inline void gn_tables_from_csum(int C, int groups, int HW, const float* __restrict__ gamma,
                                           const float* __restrict__ beta, float eps, float* sc, float* sh,
                                           double* gstat, const double* csum) {
    const int cpg = C / groups;
    const int tid = threadIdx.x;
    for (int g = tid; g < groups; g += blockDim.x) {
        double a = 0, q = 0;
        for (int c = g * cpg; c < (g + 1) * cpg; ++c) {
            a += csum[2 * c];
            q += csum[2 * c + 1];
        }
        const double n = (double)HW * cpg;
        const double mean = a / n;
        double var = q / n - mean * mean;
        var = var < 0 ? 0 : var;
        gstat[2 * g] = mean;
        gstat[2 * g + 1] = 1.0 / sqrt(var + (double)eps);
    }
    __syncthreads();
    for (int c = tid; c < C; c += blockDim.x) {
        const int g = c / cpg;
        const float rstd = (float)gstat[2 * g + 1];
        const float mean = (float)gstat[2 * g];
        const float gm = gamma ? gamma[c] : 1.f;
        const float bt = beta ? beta[c] : 0.f;
        const float scl = rstd * gm;
        sc[c] = scl;
        sh[c] = bt - mean * scl;
    }
    __syncthreads();
}

// LDS of k_gn_finalize's 1024-thread form: the tables, group stats, channel totals and the per-lane
// channel sums [lanes][C][2] (lanes = 1024 / C)
inline size_t gn_finalize_wide_lds_bytes(int C, int groups) {
    const int lanes = C <= 1024 ? 1024 / C : 1;
    return (size_t)2 * ((C + 3) & ~3) * sizeof(float) + (size_t)2 * groups * sizeof(double) +
           (size_t)2 * C * sizeof(double) * (1 + lanes) + 64;
}

inline size_t gn_fold_lds_bytes(int C, int groups) {
    return (size_t)2 * ((C + 3) & ~3) * sizeof(float) + (size_t)2 * groups * sizeof(double) +
           (size_t)2 * C * sizeof(double) + 64;
}


}  // namespace tcx
