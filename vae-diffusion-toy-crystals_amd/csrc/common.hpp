// Shared helpers for libtcx (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>
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

__device__ __forceinline__ int wrap_idx(int i, int n) {
    i = i < 0 ? i + n : i;
    return i >= n ? i - n : i;
}

}  // namespace tcx
