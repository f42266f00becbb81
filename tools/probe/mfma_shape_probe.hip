// Probe: does the conv's MFMA loop run faster as v_mfma_f32_16x16x32_f16 than as 32x32x16_f16?
// (MI355X_MICROARCH.md "DVFS give-back" item 7 measured 1.12-1.14x for bf16 loops with LDS operands.)
// Both kernels do the same FLOPs per iteration with the same LDS bytes read, on random f16 operands,
// the conv's tile shape per wave (64 pixels x 96 channels, three products per k step as f16x3) at
// two workgroups of 4 waves per CU:
//   K32: per 16-deep step 4 A + 6 B ds_read_b128, 18 x 32x32x16 (acc 2 x 3 tiles)
//   K16: per 32-deep step 8 A + 12 B ds_read_b128, 72 x 16x16x32 (acc 4 x 6 tiles)
// Build: hipcc -O3 --offload-arch=gfx950 -o mfma_shape_probe mfma_shape_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

constexpr int LDSB = 64 * 1024;

__global__ __launch_bounds__(256, 2) void k32(const float4* src, float* out, int iters) {
    extern __shared__ float4 sm[];
    for (int i = threadIdx.x; i < LDSB / 16; i += 256) sm[i] = src[(blockIdx.x * 131 + i) % (LDSB / 16)];
    __syncthreads();
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const char* base = reinterpret_cast<const char*>(sm);
    f32x16 acc[2][3];
    for (int r = 0; r < 2; ++r) for (int n = 0; n < 3; ++n) acc[r][n] = (f32x16){};
    int off = (wv * 4096 + lane * 16) & (LDSB - 1);
    for (int it = 0; it < iters; ++it) {
        h8 ah[2], al[2], bh[3], bl[3];
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            ah[r] = *reinterpret_cast<const h8*>(base + ((off + r * 2048) & (LDSB - 1)));
            al[r] = *reinterpret_cast<const h8*>(base + ((off + r * 2048 + 1024) & (LDSB - 1)));
        }
#pragma unroll
        for (int n = 0; n < 3; ++n) {
            bh[n] = *reinterpret_cast<const h8*>(base + ((off + 8192 + n * 2048) & (LDSB - 1)));
            bl[n] = *reinterpret_cast<const h8*>(base + ((off + 8192 + n * 2048 + 1024) & (LDSB - 1)));
        }
#pragma unroll
        for (int r = 0; r < 2; ++r) {
#pragma unroll
            for (int n = 0; n < 3; ++n) acc[r][n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[r], bl[n], acc[r][n], 0, 0, 0);
#pragma unroll
            for (int n = 0; n < 3; ++n) acc[r][n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[r], bh[n], acc[r][n], 0, 0, 0);
#pragma unroll
            for (int n = 0; n < 3; ++n) acc[r][n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[r], bh[n], acc[r][n], 0, 0, 0);
        }
        off = (off + 16384) & (LDSB - 1);
    }
    float s = 0.f;
    for (int r = 0; r < 2; ++r) for (int n = 0; n < 3; ++n) for (int k = 0; k < 16; ++k) s += acc[r][n][k];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

__global__ __launch_bounds__(256, 2) void k16(const float4* src, float* out, int iters) {
    extern __shared__ float4 sm[];
    for (int i = threadIdx.x; i < LDSB / 16; i += 256) sm[i] = src[(blockIdx.x * 131 + i) % (LDSB / 16)];
    __syncthreads();
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const char* base = reinterpret_cast<const char*>(sm);
    f32x4 acc[4][6];
    for (int r = 0; r < 4; ++r) for (int n = 0; n < 6; ++n) acc[r][n] = (f32x4){};
    int off = (wv * 4096 + lane * 16) & (LDSB - 1);
    for (int it = 0; it < iters / 2; ++it) {  // one 32-deep step = two 16-deep steps of k32
        h8 ah[4], al[4], bh[6], bl[6];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            ah[r] = *reinterpret_cast<const h8*>(base + ((off + r * 2048) & (LDSB - 1)));
            al[r] = *reinterpret_cast<const h8*>(base + ((off + r * 2048 + 1024) & (LDSB - 1)));
        }
#pragma unroll
        for (int n = 0; n < 6; ++n) {
            bh[n] = *reinterpret_cast<const h8*>(base + ((off + 8192 + n * 2048) & (LDSB - 1)));
            bl[n] = *reinterpret_cast<const h8*>(base + ((off + 8192 + n * 2048 + 1024) & (LDSB - 1)));
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
#pragma unroll
            for (int n = 0; n < 6; ++n) acc[r][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[r], bl[n], acc[r][n], 0, 0, 0);
#pragma unroll
            for (int n = 0; n < 6; ++n) acc[r][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[r], bh[n], acc[r][n], 0, 0, 0);
#pragma unroll
            for (int n = 0; n < 6; ++n) acc[r][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[r], bh[n], acc[r][n], 0, 0, 0);
        }
        off = (off + 16384) & (LDSB - 1);
    }
    float s = 0.f;
    for (int r = 0; r < 4; ++r) for (int n = 0; n < 6; ++n) for (int k = 0; k < 4; ++k) s += acc[r][n][k];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 4000;
    const int grid = 256 * 2 * 4;
    std::vector<float> h(LDSB / 4);
    srand(1);
    for (auto& v : h) {
        _Float16 a = (_Float16)((rand() / (float)RAND_MAX - 0.5f) * 2.f), b = (_Float16)((rand() / (float)RAND_MAX - 0.5f));
        unsigned short ua, ub;
        memcpy(&ua, &a, 2); memcpy(&ub, &b, 2);
        unsigned u = ua | ((unsigned)ub << 16);
        memcpy(&v, &u, 4);
    }
    float4* src; float* out;
    CK(hipMalloc(&src, LDSB));
    CK(hipMalloc(&out, grid * 256 * 4));
    CK(hipMemcpy(src, h.data(), LDSB, hipMemcpyHostToDevice));
    CK(hipFuncSetAttribute((const void*)k32, hipFuncAttributeMaxDynamicSharedMemorySize, LDSB));
    CK(hipFuncSetAttribute((const void*)k16, hipFuncAttributeMaxDynamicSharedMemorySize, LDSB));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const double flop = (double)grid * 4 * iters * 18 * 32768.0;
    for (int rep = 0; rep < 3; ++rep) {
        for (int which = 0; which < 2; ++which) {
            for (int w = 0; w < 3; ++w) {  // warm, then timed (the clock settles under load)
                if (which == 0) hipLaunchKernelGGL(k32, dim3(grid), dim3(256), LDSB, 0, src, out, iters);
                else hipLaunchKernelGGL(k16, dim3(grid), dim3(256), LDSB, 0, src, out, iters);
            }
            CK(hipEventRecord(e0));
            for (int w = 0; w < 5; ++w) {
                if (which == 0) hipLaunchKernelGGL(k32, dim3(grid), dim3(256), LDSB, 0, src, out, iters);
                else hipLaunchKernelGGL(k16, dim3(grid), dim3(256), LDSB, 0, src, out, iters);
            }
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            printf("rep %d %s: %.3f ms per launch, %.1f TFLOP/s (f16 MFMA rate)\n", rep,
                   which == 0 ? "32x32x16" : "16x16x32", ms / 5, flop / (ms / 5 * 1e-3) / 1e12);
        }
    }
    return 0;
}
