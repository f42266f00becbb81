// Probe: where a skinny-M f16x3 linear launch of the prior's DDIM goes (k_skinny_h2<3, 4> at fc1's shape:
// M = 36 rows, N = 4096 columns, K = 1024, 16.7 MB of h2 weights), as back-to-back dependent launches on one
// stream (the DDIM's chain).  Variants of the same skeleton (8 waves x 16 columns x a 128-deep K slice per
// wave, all loads up front, 36 MFMAs per wave, wave-order LDS reduce, one record store per 8 columns):
//   full      the product kernel's structure
//   noload    operands from registers (no global loads)
//   noreduce  loads + MFMA, each wave stores its own partial tile (no barrier, no LDS)
//   trivial   one store per workgroup
//   w4        4 waves per workgroup (twice the workgroups, 2 K chunks -> partial planes)
//   ct2       each wave on 2 column tiles (the activations loaded once for 32 columns)
//   hipcc --offload-arch=gfx950 -O3 tools/probe/skinny_probe.hip -o /tmp/skinny_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                               \
    do {                                                                    \
        hipError_t e_ = (x);                                                \
        if (e_ != hipSuccess) {                                             \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));         \
            exit(1);                                                        \
        }                                                                   \
    } while (0)

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int M = 36;
constexpr int MT = 3;

// MODE 0 full, 1 noload, 2 noreduce, 3 trivial; WAVES 8 or 4; CT column tiles per wave
template <int MODE, int WAVES, int CT, int NC, int N, int K>
__global__ __launch_bounds__(64 * WAVES) void k_probe(const char* __restrict__ x, const char* __restrict__ w,
                                                      float* __restrict__ y) {
    constexpr int G = K / 8;
    __shared__ float red[WAVES][16 * MT][16 * CT + 1];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int r = lane & 15, q = lane >> 4;
    if (MODE == 3) {
        if (tid == 0) y[blockIdx.x] = 1.f;
        return;
    }
    const int n0 = blockIdx.x * 16 * CT;
    const int kw0 = blockIdx.y * WAVES * 32 * NC + wv * 32 * NC;
    uint4 wh[CT][NC], wl[CT][NC], xh[NC][MT], xl[NC][MT];
    if (MODE == 1) {
#pragma unroll
        for (int c = 0; c < NC; ++c) {
#pragma unroll
            for (int j = 0; j < CT; ++j) wh[j][c] = wl[j][c] = make_uint4(lane, c, j, 1);
#pragma unroll
            for (int t = 0; t < MT; ++t) xh[c][t] = xl[c][t] = make_uint4(t, c, lane, 2);
        }
    } else {
#pragma unroll
        for (int c = 0; c < NC; ++c)
#pragma unroll
            for (int j = 0; j < CT; ++j) {
                const char* p = w + ((size_t)(n0 + 16 * j + r) * G + (kw0 + 32 * c) / 8 + q) * 32;
                wh[j][c] = *reinterpret_cast<const uint4*>(p);
                wl[j][c] = *reinterpret_cast<const uint4*>(p + 16);
            }
#pragma unroll
        for (int c = 0; c < NC; ++c)
#pragma unroll
            for (int t = 0; t < MT; ++t) {
                const char* p = x + ((size_t)min(16 * t + r, M - 1) * G + (kw0 + 32 * c) / 8 + q) * 32;
                xh[c][t] = *reinterpret_cast<const uint4*>(p);
                xl[c][t] = *reinterpret_cast<const uint4*>(p + 16);
            }
    }
    __builtin_amdgcn_sched_barrier(0);
    f32x4 acc[CT][MT];
#pragma unroll
    for (int j = 0; j < CT; ++j)
#pragma unroll
        for (int t = 0; t < MT; ++t) acc[j][t] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
        for (int j = 0; j < CT; ++j) {
            const h8 bh = __builtin_bit_cast(h8, wh[j][c]), bl = __builtin_bit_cast(h8, wl[j][c]);
#pragma unroll
            for (int t = 0; t < MT; ++t) {
                const h8 ah = __builtin_bit_cast(h8, xh[c][t]), al = __builtin_bit_cast(h8, xl[c][t]);
                acc[j][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl, acc[j][t], 0, 0, 0);
                acc[j][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh, acc[j][t], 0, 0, 0);
                acc[j][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, acc[j][t], 0, 0, 0);
            }
        }
    if (MODE == 2) {
        float* dst = y + ((size_t)blockIdx.y * WAVES + wv) * M * N;
#pragma unroll
        for (int j = 0; j < CT; ++j)
#pragma unroll
            for (int t = 0; t < MT; ++t)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int m = 16 * t + 4 * q + e;
                    if (m < M) dst[(size_t)m * N + n0 + 16 * j + r] = acc[j][t][e];
                }
        return;
    }
#pragma unroll
    for (int j = 0; j < CT; ++j)
#pragma unroll
        for (int t = 0; t < MT; ++t)
#pragma unroll
            for (int e = 0; e < 4; ++e) red[wv][16 * t + 4 * q + e][16 * j + r] = acc[j][t][e];
    __syncthreads();
    // one thread per (row, 8 columns): sum the waves in order, store 8 floats
    for (int o = tid; o < M * 2 * CT; o += 64 * WAVES) {
        const int m = o / (2 * CT), c0 = 8 * (o % (2 * CT));
        float v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            float s = red[0][m][c0 + k];
#pragma unroll
            for (int ww = 1; ww < WAVES; ++ww) s += red[ww][m][c0 + k];
            v[k] = s;
        }
        float* dst = y + (size_t)blockIdx.y * M * N + (size_t)m * N + n0 + c0;
        *reinterpret_cast<float4*>(dst) = make_float4(v[0], v[1], v[2], v[3]);
        *reinterpret_cast<float4*>(dst + 4) = make_float4(v[4], v[5], v[6], v[7]);
    }
}

// launches rotate over `copies` weight copies of `wbytes` (copies = 24: every launch streams from HBM)
template <int MODE, int WAVES, int CT, int NC = 4, int N = 4096, int K = 1024>
float run(const char* x, const char* w, float* y, int iters, int copies, size_t wbytes) {
    const dim3 grid(N / (16 * CT), K / (WAVES * 32 * NC));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int i = 0; i < 20; ++i)
        hipLaunchKernelGGL((k_probe<MODE, WAVES, CT, NC, N, K>), grid, dim3(64 * WAVES), 0, 0, x, w + (size_t)(i % copies) * wbytes, y);
    CK(hipEventRecord(e0));
    for (int i = 0; i < iters; ++i)
        hipLaunchKernelGGL((k_probe<MODE, WAVES, CT, NC, N, K>), grid, dim3(64 * WAVES), 0, 0, x, w + (size_t)(i % copies) * wbytes, y);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms * 1e3f / iters;
}

int main() {
    // weights: 24 copies (400 MB) so that each launch streams from HBM, as the DDIM's 16 trunk linears do
    const size_t wbytes = (size_t)4096 * 1024 * 4;
    const int copies = 24;
    char* w;
    char* x;
    float* y;
    CK(hipMalloc(&w, wbytes * copies));
    CK(hipMalloc(&x, (size_t)M * 4096 * 4));
    CK(hipMalloc(&y, (size_t)16 * M * 4096 * 4));
    CK(hipMemset(w, 0, wbytes * copies));
    CK(hipMemset(x, 0, (size_t)M * 4096 * 4));
    for (int rep = 0; rep < 2; ++rep) {
        for (int cp : {24, 1}) {
            printf("weights %s\n", cp == 24 ? "from HBM (24 rotating copies)" : "one copy (cache-resident)");
            printf("  full      %.2f us\n", run<0, 8, 1>(x, w, y, 240, cp, wbytes));
            printf("  noload    %.2f us\n", run<1, 8, 1>(x, w, y, 240, cp, wbytes));
            printf("  noreduce  %.2f us\n", run<2, 8, 1>(x, w, y, 240, cp, wbytes));
            printf("  trivial   %.2f us\n", run<3, 8, 1>(x, w, y, 240, cp, wbytes));
            printf("  w4        %.2f us\n", run<0, 4, 1>(x, w, y, 240, cp, wbytes));
            printf("  ct2       %.2f us\n", run<0, 8, 2>(x, w, y, 240, cp, wbytes));
            printf("  w4ct2     %.2f us\n", run<0, 4, 2>(x, w, y, 240, cp, wbytes));
            printf("  w4ct4nc2  %.2f us\n", run<0, 4, 4, 2>(x, w, y, 240, cp, wbytes));
            printf("  w8ct4nc2  %.2f us\n", run<0, 8, 4, 2>(x, w, y, 240, cp, wbytes));
            printf("  w4ct8nc1  %.2f us\n", run<0, 4, 8, 1>(x, w, y, 240, cp, wbytes));
            printf("  fc2 (N 1024, K 4096): w8ct1nc4 %.2f  w4ct4nc2 %.2f  w4ct2nc4 %.2f  w4ct8nc1 %.2f us\n",
                   run<0, 8, 1, 4, 1024, 4096>(x, w, y, 240, cp, wbytes), run<0, 4, 4, 2, 1024, 4096>(x, w, y, 240, cp, wbytes),
                   run<0, 4, 2, 4, 1024, 4096>(x, w, y, 240, cp, wbytes), run<0, 4, 8, 1, 1024, 4096>(x, w, y, 240, cp, wbytes));
        }
    }
    return 0;
}
