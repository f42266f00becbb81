// Probe: HBM write rate of the h2-record store pattern.  Every record writer of the split path (apply,
// upsample, first conv, attention prep) has each lane write its 32-B record as two 16-B stores (hi piece,
// lo piece), so ONE store instruction covers 64 x 16 B at a 32-B stride (half of every 64-B segment of a
// 2-KB span) and the next instruction fills the other halves.  Compared here with instructions that each
// write 1 KB contiguous, at the size of the 64^2 apply pass (403 MB), read+write and write-only.
//   hipcc --offload-arch=gfx950 -O3 tools/probe/store_pattern_probe.hip -o tools/probe/store_pattern_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                        \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

// MODE 0: record pattern (lane i: bytes [32 i, 32 i + 16) then [32 i + 16, 32 i + 32))
// MODE 1: contiguous (instruction 0: lane i -> 16 i of a 2-KB block, instruction 1: 1 KB + 16 i)
// RD: also read the same bytes first (an in-place transform)
template <int MODE, bool RD>
__global__ __launch_bounds__(256) void k_rec(uint4* __restrict__ y, size_t n32, int per) {
    const size_t wave = (blockIdx.x * 256 + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    for (int k = 0; k < per; ++k) {
        const size_t blk = (wave * per + k) * 64;  // 64 records = 2 KB per wave and step
        if (blk >= n32) return;
        size_t o0, o1;
        if (MODE == 0) {
            o0 = 2 * (blk + lane);
            o1 = o0 + 1;
        } else {
            o0 = 2 * blk + lane;
            o1 = o0 + 64;
        }
        uint4 a = make_uint4(lane, k, 1, 2), b = make_uint4(3, 4, lane, k);
        if (RD) {
            a = y[o0];
            b = y[o1];
            a.x += 1;
            b.y += 1;
        }
        y[o0] = a;
        y[o1] = b;
    }
}

template <int MODE, bool RD>
float run(uint4* y, size_t n32) {
    const int per = 4;
    const size_t waves = (n32 / 64 + per - 1) / per;
    const dim3 grid((unsigned)((waves * 64 + 255) / 256));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((k_rec<MODE, RD>), grid, dim3(256), 0, 0, y, n32, per);
    CK(hipEventRecord(e0));
    const int reps = 20;
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((k_rec<MODE, RD>), grid, dim3(256), 0, 0, y, n32, per);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms * 1e3f / reps;
}

int main() {
    const size_t bytes = (size_t)256 * 4096 * 96 * 4;  // the 64^2 apply pass: 403 MB
    const size_t n32 = bytes / 32;
    uint4* y;
    CK(hipMalloc(&y, bytes));
    CK(hipMemset(y, 0, bytes));
    const float gb = bytes / 1e9f;
    for (int rep = 0; rep < 2; ++rep) {
        const float a = run<0, false>(y, n32), b = run<1, false>(y, n32);
        const float c = run<0, true>(y, n32), d = run<1, true>(y, n32);
        printf("write-only  record %.1f us (%.2f TB/s)  contiguous %.1f us (%.2f TB/s)\n", a, gb / a * 1e3f,
               b, gb / b * 1e3f);
        printf("read+write  record %.1f us (%.2f TB/s)  contiguous %.1f us (%.2f TB/s)\n", c, 2 * gb / c * 1e3f,
               d, 2 * gb / d * 1e3f);
    }
    CK(hipFree(y));
    return 0;
}
