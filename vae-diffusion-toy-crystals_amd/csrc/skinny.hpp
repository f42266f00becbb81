// Skinny-M linears (M <= 64 rows): split-K partial GEMM + fused reduce epilogues (skinny.hip).
// Used by tcx_linear_ws and by the native prior forward / DDIM sampler (prior.hip).
#pragma once
#include "common.hpp"

namespace tcx {

// Per source: chunks of 8 waves x 16*nb k-values (nb in {2,4,8}), s chunks.  Depends on K only, so
// the fp32 summation order of every output element is independent of M and N.
struct SkPlan {
    int nb1, s1, nb2, s2;
};

bool skinny_ok(int M, int N, int K1, int K2);
SkPlan skinny_plan(int K1, int K2);
inline size_t skinny_part_floats(const SkPlan& p, int M, int N) { return (size_t)(p.s1 + p.s2) * M * N; }

// part[s][M][N] = raw partial sums of x W^T over chunk s (source 1 chunks, then source 2 chunks).
// W = w [>= 16*cdiv(N,16) rows][kpad]; source 2 reads weight columns [K1, K1 + K2).
int skinny_partials(const float* x1, int ldx1, int K1, const float* x2, int ldx2, int K2, const float* w, int kpad,
                    int M, int N, const SkPlan& p, float* part, hipStream_t st);

// Epilogue of the fixed-order reduce over the S partial planes.
struct SkEpi {
    const float* b = nullptr;      // [N] bias
    const float* resid = nullptr;  // [M][N] added after the bias (may alias y)
    int act = 0;                   // 0 none, 1 relu, 2 sigmoid, 3 silu
    float* y = nullptr;            // [M][N] result (may be null in DDIM mode)
    // DDIM eta = 0 update (diffusion_prior.py:226-250) with the row as eps_pred: z [M][N] in place
    float* z = nullptr;
    float abar_t = 0.f, abar_prev = 0.f;
    int last = 0;
    // split-f16 ("h2", h2.hpp) output instead of y (k_skinny_h2's one-chunk epilogue): [M][N/8][2][8]
    void* y_h2 = nullptr;
    unsigned* ovf = nullptr;  // raised when a value leaves the f16 range
};
int skinny_reduce(const float* part, int S, int M, int N, const SkEpi& e, hipStream_t st);
// partials + reduce, or (one chunk, one source) the epilogue inside the GEMM kernel
int skinny_linear(const float* x1, int ldx1, int K1, const float* x2, int ldx2, int K2, const float* w, int kpad,
                  int M, int N, float* part, const SkEpi& e, hipStream_t st);

// Reduce + bias (+ resid) into y, then LayerNorm (+ FiLM) of each finished row into yn:
// yn = LN(y) * lw + lb, then (gy != null) yn * (1 + gamma) + beta with
// gamma = gy[m][c] (+ gt[c]), beta = gy[m][N + c] (+ gt[N + c]).  N % 4 == 0, N <= 4096.
struct SkLn {
    const float* lw = nullptr;
    const float* lb = nullptr;
    const float* gy = nullptr;
    int ld_gy = 0;
    const float* gt = nullptr;  // one row broadcast over m (the DDIM's per-step time half)
    float eps = 1e-5f;
    float* yn = nullptr;
    void* yn_h2 = nullptr;    // h2 output instead of yn
    unsigned* ovf = nullptr;
};
bool skinny_ln_ok(int N);
int skinny_reduce_ln(const float* part, int S, int M, int N, const SkEpi& e, const SkLn& ln, hipStream_t st);

// f16x3 skinny linears (K % 32 == 0): x and W in h2 storage (h2.hpp), W rows scaled by exact powers
// of two (winv = the inverse, applied in the epilogue); products hi*hi + hi*lo + lo*hi on
// v_mfma_f32_16x16x32_f16 (16x the f32 MFMA rate), fp32 accumulation.
bool skinny_h2_ok(int M, int N, int K);
size_t skinny_h2_part_floats(int M, int N, int K);
int skinny_h2_chunks(int N, int K);  // partial planes of skinny_h2_partials at this shape
int skinny_h2_partials(const void* xh, int K, const void* wh, const float* winv, int M, int N, float* part,
                       hipStream_t st);
int skinny_h2_linear(const void* xh, int K, const void* wh, const float* winv, int M, int N, float* part,
                     const SkEpi& e, hipStream_t st);

// LayerNorm (+ FiLM with an optional broadcast row gt) of M rows, norm.hip
int launch_layernorm_film(const float* x, float* y, int M, int Wd, const float* lw, const float* lb, const float* gb,
                          int ld_gb, const float* gt, float eps, hipStream_t st);

}  // namespace tcx
