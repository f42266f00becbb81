// Probe: does v_mfma_f32_32x32x16_f16 keep f16 subnormal inputs, and does the f32->f16
// conversion produce subnormals (default float mode, gfx950)?  Also the exactness of the
// 3-product hi/lo split on random dot products against an fp64 host reference.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include <vector>
#include <random>
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));

__global__ void k_denorm(const float* in, float* out, float* cvt_out) {
    const int l = threadIdx.x;
    h8 a, b;
    for (int j = 0; j < 8; ++j) { a[j] = (_Float16)in[0]; b[j] = (_Float16)1.0f; }
    f16v acc = {};
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc, 0, 0, 0);
    out[l] = acc[0];
    if (l == 0) cvt_out[0] = (float)(_Float16)in[0];
}

// dot products of length K over rows: split-f16 3-product (hi*hi + hi*lo + lo*hi) via MFMA
// A [32][K] rows, B [K][32]; one wave; K multiple of 16.
__global__ void k_dot(const float* A, const float* B, float* C, int K, float wscale) {
    const int l = threadIdx.x, r = l & 31, h = l >> 5;
    f16v acc = {};
    for (int k0 = 0; k0 < K; k0 += 16) {
        h8 ah, al, bh, bl;
        for (int j = 0; j < 8; ++j) {
            float a = A[r * K + k0 + 8 * h + j];
            _Float16 x = (_Float16)a; ah[j] = x; al[j] = (_Float16)(a - (float)x);
            float b = B[(k0 + 8 * h + j) * 32 + r] * wscale;
            _Float16 y = (_Float16)b; bh[j] = y; bl[j] = (_Float16)(b - (float)y);
        }
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, acc, 0, 0, 0);
    }
    for (int i = 0; i < 16; ++i) {
        const int row = (i & 3) + 8 * (i >> 2) + 4 * h;
        C[row * 32 + r] = acc[i] / wscale;
    }
}
// same with the exact fp32 MFMA for comparison
__global__ void k_dot32(const float* A, const float* B, float* C, int K) {
    const int l = threadIdx.x, r = l & 31, h = l >> 5;
    f16v acc = {};
    for (int k0 = 0; k0 < K; k0 += 2) {
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(A[r * K + k0 + h], B[(k0 + h) * 32 + r], acc, 0, 0, 0);
    }
    for (int i = 0; i < 16; ++i) {
        const int row = (i & 3) + 8 * (i >> 2) + 4 * h;
        C[row * 32 + r] = acc[i];
    }
}

int main() {
    float *din, *dout, *dcvt;
    hipMalloc(&din, 4); hipMalloc(&dout, 256); hipMalloc(&dcvt, 4);
    const float vals[3] = {ldexpf(1.f, -20), ldexpf(3.f, -24), ldexpf(1.f, -10)};
    for (float v : vals) {
        hipMemcpy(din, &v, 4, hipMemcpyHostToDevice);
        k_denorm<<<1, 64>>>(din, dout, dcvt);
        float o, c;
        hipMemcpy(&o, dout, 4, hipMemcpyDeviceToHost);
        hipMemcpy(&c, dcvt, 4, hipMemcpyDeviceToHost);
        printf("in %.6e: cvt %.6e  mfma(16 terms) %.6e expect %.6e\n", v, c, o, 16.f * c);
    }
    const int K = 1728;
    std::mt19937 g(1);
    std::normal_distribution<float> nd;
    std::uniform_real_distribution<float> ud(-1.f, 1.f);
    std::vector<float> A(32 * K), B(K * 32), C(32 * 32), C32(32 * 32);
    for (auto& a : A) { float x = nd(g); x = (ud(g) < 0 ? 0.01f : 1.f) * x; a = x > 0 ? x : 0.1f * x; }
    for (auto& b : B) b = ud(g) / sqrtf((float)K);
    float *dA, *dB, *dC;
    hipMalloc(&dA, A.size() * 4); hipMalloc(&dB, B.size() * 4); hipMalloc(&dC, C.size() * 4);
    hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice);
    k_dot<<<1, 64>>>(dA, dB, dC, K, 1024.f);
    hipMemcpy(C.data(), dC, C.size() * 4, hipMemcpyDeviceToHost);
    k_dot32<<<1, 64>>>(dA, dB, dC, K);
    hipMemcpy(C32.data(), dC, C.size() * 4, hipMemcpyDeviceToHost);
    double e16 = 0, e32 = 0;
    for (int i = 0; i < 32; ++i)
        for (int j = 0; j < 32; ++j) {
            double ref = 0, sc = 0;
            for (int k = 0; k < K; ++k) { ref += (double)A[i * K + k] * B[k * 32 + j]; sc += fabs((double)A[i * K + k] * B[k * 32 + j]); }
            e16 = fmax(e16, fabs(C[i * 32 + j] - ref) / sc);
            e32 = fmax(e32, fabs(C32[i * 32 + j] - ref) / sc);
        }
    printf("max |err|/sum|ab|: f16x3 split %.3e   fp32 mfma %.3e\n", e16, e32);
    return 0;
}
