// One-channel convolutions (thin.hip): the first / out convs of the score net and their gradients.
#pragma once
#include "common.hpp"

namespace tcx {

struct ThinConv {
    const float* x;  // [B][H][W][Cin]
    const float* w;  // packed weight row-major [cout_pad][kpad], k = tap * Cin + ci
    const float *bias, *bias_b, *resid;
    float* y;        // [B][Ho][Wo][Cout]
    int B, H, W, Cin, Cout, kpad, ks, pad, circular, Ho, Wo, act;
};

// tcx_conv2d (conv.hip): true when this shape runs on the one-channel kernels; the launch
bool thin_conv_takes(const ThinConv& a);
int launch_thin_conv(const ThinConv& a, hipStream_t st);

struct ThinWgrad {
    const float* wide;  // Cout == 1: x [P][C];  Cin == 1: dY [P][C]
    const float* thin;  // Cout == 1: dY [P];    Cin == 1: x [P]
    int B, H, W, C, ks, pad, circular;  // 3 x 3, pad 1
    int sign;           // thin operand at pixel p - off(tap) (Cout == 1: -1) or p + off(tap) (Cin == 1: +1)
    int segw, nseg;     // work unit: a segment of segw pixels of one image row (nseg per row)
    int units, upw, S;  // B H nseg units, units per workgroup, pixel streams per workgroup
    float* part;        // [nsplit][T][C] (Cout == 1 / Cin == 1 alike: k = tap C + c resp. tap, co = c)
};

// tcx_conv_wgrad (gemm.hip): fills *a's plan (caller sets wide / thin / pad / circular / sign / part) and
// returns the partial-plane count (<= max_split), or 0 when the shape does not run here
int thin_wgrad_plan(int B, int H, int W, int Cin, int Cout, int ks, int stride, int max_split, ThinWgrad* a);
int launch_thin_wgrad(const ThinWgrad& a, int nsplit, hipStream_t st);

}  // namespace tcx
