// Toy-crystal Gaussian splatting for the procedural dataset (replaces the per-item CPU render of
// /root/reference/src/toycrystals/data.py:132-153 + the normalisation :204-206 and the uint8
// quantisation of scripts/build_dataset.py:34).
//
// One workgroup (256 threads) per image; a thread owns PPT = ceil(H*W/256) consecutive pixels.
// The image's atom list is read with wave-uniform (scalar) loads; per atom a thread first tests
// the squared distance from the atom to the bounding box of its pixels and skips the atom when
// every term would be exp(arg) with arg < -110 — exactly 0.0f in fp32 (expf underflows to 0
// below -103.98), so the skip changes no bit.  The terms themselves follow the reference's fp32
// operation order: dx = x - px, dy = y - py, d2 = dx*dx + dy*dy (separately rounded products,
// no FMA contraction), arg = -d2 / s2 (IEEE division by the fp32 operand 2 sigma^2), expf, and a
// sequential fp32 sum over the atoms in list order.  Then the image max (workgroup reduction),
// x = v / (max + 1e-8f), clamp to [0, 1], optional uint8 = (uint8)(x * 255.f) (truncation).
// The work is ~N_near x H*W expf per image: ALU-bound, one launch per batch of images.
#include "common.hpp"

namespace tcx {
namespace {

constexpr int RT = 256;

template <int MAXP>  // pixels per thread (ppt rounded up to a power of two)
__global__ __launch_bounds__(RT) void k_render(const float* __restrict__ pts, const int* __restrict__ offs,
                                               const float* __restrict__ s2v, int H, int W, float* __restrict__ xo,
                                               unsigned char* __restrict__ uo) {
    __shared__ float red[RT / 64];
    const int img = blockIdx.x;
    const int tid = threadIdx.x;
    const int HW = H * W;
    const int ppt = (HW + RT - 1) / RT;
    const int q0 = tid * ppt;
    const int p0 = offs[img], p1 = offs[img + 1];
    const float s2 = s2v[img];
    const float cut = 110.f * s2 * 1.0001f;
    float acc[MAXP];
    float px[MAXP], py[MAXP];
    float bx0 = 3.4e38f, bx1 = -3.4e38f, by0 = 3.4e38f, by1 = -3.4e38f;
#pragma unroll
    for (int k = 0; k < MAXP; ++k) {
        acc[k] = 0.f;
        const int q = q0 + k;
        const bool v = k < ppt && q < HW;
        const int qq = v ? q : 0;
        px[k] = (float)(qq % W);
        py[k] = (float)(qq / W);
        if (v) {
            bx0 = fminf(bx0, px[k]); bx1 = fmaxf(bx1, px[k]);
            by0 = fminf(by0, py[k]); by1 = fmaxf(by1, py[k]);
        }
    }
    for (int i = p0; i < p1; ++i) {
        const float ax = pts[2 * i], ay = pts[2 * i + 1];
        const float ex = fmaxf(fmaxf(bx0 - ax, ax - bx1), 0.f);
        const float ey = fmaxf(fmaxf(by0 - ay, ay - by1), 0.f);
        if (ex * ex + ey * ey > cut) continue;  // every term of this atom is exactly 0.0f
#pragma unroll
        for (int k = 0; k < MAXP; ++k) {
            if (k < ppt) {
                const float dx = __fsub_rn(px[k], ax), dy = __fsub_rn(py[k], ay);
                const float d2 = __fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy));
                acc[k] = __fadd_rn(acc[k], expf(__fdiv_rn(-d2, s2)));
            }
        }
    }
    float m = -3.4e38f;
#pragma unroll
    for (int k = 0; k < MAXP; ++k)
        if (k < ppt && q0 + k < HW) m = fmaxf(m, acc[k]);
    for (int o = 32; o; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    if ((tid & 63) == 0) red[tid >> 6] = m;
    __syncthreads();
    m = red[0];
#pragma unroll
    for (int w = 1; w < RT / 64; ++w) m = fmaxf(m, red[w]);
    const float den = __fadd_rn(m, 1e-8f);
    const size_t base = (size_t)img * HW;
#pragma unroll
    for (int k = 0; k < MAXP; ++k) {
        const int q = q0 + k;
        if (k < ppt && q < HW) {
            float x = __fdiv_rn(acc[k], den);
            x = fminf(fmaxf(x, 0.f), 1.f);
            if (xo) xo[base + q] = x;
            if (uo) uo[base + q] = (unsigned char)(int)__fmul_rn(x, 255.f);
        }
    }
}

}  // namespace
}  // namespace tcx

using namespace tcx;

extern "C" int tcx_render_crystals(const float* pts, const int* offsets, const float* s2, int n_img, int H, int W,
                                   float* x_out, unsigned char* u8_out, void* stream) {
    TCX_REQUIRE(offsets && s2 && (x_out || u8_out) && n_img >= 0 && H > 0 && W > 0,
                "tcx_render_crystals: bad args");
    TCX_REQUIRE((H * W + RT - 1) / RT <= 64, "tcx_render_crystals: at most 16384 pixels per image");
    if (n_img == 0) return TCX_OK;
    TCX_REQUIRE(pts, "tcx_render_crystals: null points");
    const int ppt = (H * W + RT - 1) / RT;
    const dim3 g(n_img), b(RT);
    hipStream_t st = (hipStream_t)stream;
    if (ppt <= 1) hipLaunchKernelGGL(k_render<1>, g, b, 0, st, pts, offsets, s2, H, W, x_out, u8_out);
    else if (ppt <= 2) hipLaunchKernelGGL(k_render<2>, g, b, 0, st, pts, offsets, s2, H, W, x_out, u8_out);
    else if (ppt <= 4) hipLaunchKernelGGL(k_render<4>, g, b, 0, st, pts, offsets, s2, H, W, x_out, u8_out);
    else if (ppt <= 8) hipLaunchKernelGGL(k_render<8>, g, b, 0, st, pts, offsets, s2, H, W, x_out, u8_out);
    else if (ppt <= 16) hipLaunchKernelGGL(k_render<16>, g, b, 0, st, pts, offsets, s2, H, W, x_out, u8_out);
    else if (ppt <= 32) hipLaunchKernelGGL(k_render<32>, g, b, 0, st, pts, offsets, s2, H, W, x_out, u8_out);
    else hipLaunchKernelGGL(k_render<64>, g, b, 0, st, pts, offsets, s2, H, W, x_out, u8_out);
    return check_launch("tcx_render_crystals");
}
