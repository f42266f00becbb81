// One-channel convolutions of the training step (round 6): the score net's first conv (x_t, 1 channel
// -> 96, sde_score_model.py:246 down1.net[0]), its out conv (96 -> 1, :264 self.out), their data
// gradients (the out conv's is a 1 -> 96 conv over dY) and their weight gradients.
//
// The implicit-GEMM kernels tile Cout by 32 and K by 32, so a 1-channel side wastes 31 of every 32
// MFMA columns (out conv forward 331 us, its weight gradient 429 us per B = 128 step on k_conv /
// k_wgrad, profiles/r06_d_train_kernel_breakdown.txt) on a layer whose floor is one pass over the
// 96-channel tensor (201 MB: ~40 us).  These are HBM-bound reductions, so they run on the VALU in
// fp32 with coalesced 16-B loads — no MFMA:
//   k_thin_cin1   y[o][co]  = bias + bias_b + sum_tap w[co][tap] x[o + off(tap)]   (+ resid, act)
//   k_thin_cout1  y[o]      = bias + sum_tap sum_ci w[tap][ci] x[o + off(tap)][ci] (+ resid, act)
//   k_thin_wgrad  part[s][tap Cin + ci][co] = sum over split s's pixels of the same products
//                 (Cout == 1: x shifted, dY one channel; Cin == 1: x one channel shifted, dY wide),
//                 folded by tcx_conv_wgrad's k_wgrad_reduce (fixed split order: deterministic).
// Stride 1 only; circular or zero padding.  Every sum runs in a fixed order (no atomics).
#include "thin.hpp"

#include <algorithm>

namespace tcx {

namespace {

__device__ __forceinline__ float thin_act(float v, int act) {
    if (act == 1) return fmaxf(v, 0.f);
    if (act == 2) return 1.f / (1.f + expf(-v));
    if (act == 3) return silu_f(v);
    return v;
}

// workgroups stride over the output rows (weights transposed into LDS as [tap][Cout] and the bias staged once
// per workgroup: staging them per row cost more than the row's arithmetic); per row the ks input rows (with
// their wrapped / zero halo columns) are staged in LDS and one thread takes (output pixel, 4 output channels)
// in turn; 32-bit index math
__global__ __launch_bounds__(256) void k_thin_cin1(ThinConv a) {
    extern __shared__ __attribute__((aligned(16))) float wT[];
    const int T = a.ks * a.ks, Q = a.Cout / 4, XW = a.Wo + a.ks - 1;  // staged row width
    float* bsh = wT + T * a.Cout;                                     // [Cout] bias
    float* xs = bsh + a.Cout;                                         // [ks][XW]
    for (int i = threadIdx.x; i < T * a.Cout; i += 256) {
        const int co = i / T, tap = i - co * T;  // consecutive lanes read one packed row's taps
        wT[tap * a.Cout + co] = a.w[(size_t)co * a.kpad + tap];
    }
    for (int i = threadIdx.x; i < a.Cout; i += 256) bsh[i] = a.bias ? a.bias[i] : 0.f;
    for (int row = blockIdx.x; row < a.B * a.Ho; row += gridDim.x) {
        const int b = row / a.Ho, oy = row - b * a.Ho;
        const float* xb = a.x + (size_t)b * a.H * a.W;
        __syncthreads();  // the previous row's reads of xs are done (and the weights staged)
        for (int i = threadIdx.x; i < a.ks * XW; i += 256) {
            const int dy = i / XW, c = i - dy * XW;  // staged column c = input column c - pad
            const int iy = oy + dy - a.pad, ix = c - a.pad;
            float v = 0.f;
            if (a.circular) v = xb[wrap_idx(iy, a.H) * a.W + wrap_idx(ix, a.W)];
            else if (iy >= 0 && iy < a.H && ix >= 0 && ix < a.W) v = xb[iy * a.W + ix];
            xs[i] = v;
        }
        __syncthreads();
        for (int it = threadIdx.x; it < a.Wo * Q; it += 256) {
            const int ox = it / Q, cq = it - ox * Q;
            float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
            for (int dy = 0; dy < a.ks; ++dy)
                for (int dx = 0; dx < a.ks; ++dx) {
                    const float v = xs[dy * XW + ox + dx];
                    const float4 w4 = *reinterpret_cast<const float4*>(wT + (dy * a.ks + dx) * a.Cout + 4 * cq);
                    acc.x = fmaf(v, w4.x, acc.x); acc.y = fmaf(v, w4.y, acc.y);
                    acc.z = fmaf(v, w4.z, acc.z); acc.w = fmaf(v, w4.w, acc.w);
                }
            float4 add = *reinterpret_cast<const float4*>(bsh + 4 * cq);
            if (a.bias_b) {
                const float4 bb = *reinterpret_cast<const float4*>(a.bias_b + (size_t)b * a.Cout + 4 * cq);
                add.x += bb.x; add.y += bb.y; add.z += bb.z; add.w += bb.w;
            }
            const size_t oi = ((size_t)row * a.Wo + ox) * a.Cout + 4 * cq;
            if (a.resid) {
                const float4 rr = *reinterpret_cast<const float4*>(a.resid + oi);
                add.x += rr.x; add.y += rr.y; add.z += rr.z; add.w += rr.w;
            }
            const float4 out = make_float4(thin_act(acc.x + add.x, a.act), thin_act(acc.y + add.y, a.act),
                                           thin_act(acc.z + add.z, a.act), thin_act(acc.w + add.w, a.act));
            *reinterpret_cast<float4*>(a.y + oi) = out;
        }
    }
}

// workgroups stride over the output rows; per row the ks input rows are read as contiguous [x][c] float4 streams (lane =
// 4 channels of one pixel, coalesced), each float4 dotted with the ks weight quads of its tap row per dx
// and the ks partials per (dx, x, quad) left in LDS; the row's outputs then sum them in a fixed order
// (4 lanes per pixel over quads, then dx).  Row stride QP = Q | 1 floats keeps those reads free of bank
// conflicts.
__global__ __launch_bounds__(256) void k_thin_cout1(ThinConv a) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int ks = a.ks, C = a.Cin, Q = C / 4, QP = Q | 1;
    float* wk = sm;                      // [ks ks C]
    float* part = sm + ks * ks * C;      // [ks][W][QP]
    for (int i = threadIdx.x; i < ks * ks * C; i += 256) wk[i] = a.w[i];
    for (int row = blockIdx.x; row < a.B * a.Ho; row += gridDim.x) {
        const int b = row / a.Ho, oy = row - b * a.Ho;
        const float* xb = a.x + (size_t)b * a.H * a.W * C;
        __syncthreads();  // the weights staged; the previous row's partials read
        for (int it = threadIdx.x; it < a.W * Q; it += 256) {
            const int x = it / Q, cq = it - x * Q;
            float acc[7] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
            for (int dy = 0; dy < ks; ++dy) {
                int iy = oy + dy - a.pad;
                if (a.circular) iy = wrap_idx(iy, a.H);
                else if (iy < 0 || iy >= a.H) continue;
                const float4 v = *reinterpret_cast<const float4*>(xb + ((size_t)iy * a.W + x) * C + 4 * cq);
                for (int dx = 0; dx < ks; ++dx) {
                    const float4 w4 = *reinterpret_cast<const float4*>(wk + (dy * ks + dx) * C + 4 * cq);
                    acc[dx] = fmaf(v.w, w4.w, fmaf(v.z, w4.z, fmaf(v.y, w4.y, fmaf(v.x, w4.x, acc[dx]))));
                }
            }
            for (int dx = 0; dx < ks; ++dx) part[(dx * a.W + x) * QP + cq] = acc[dx];
        }
        __syncthreads();
        // 4 lanes per output pixel, each summing every 4th quad over the ks dx taps, then two xor shuffles
        // (a fixed order); all 256 lanes reach the shuffles
        const int sub = threadIdx.x & 3;
        for (int o0 = 0; o0 < a.Wo; o0 += 64) {
            const int ox = o0 + (threadIdx.x >> 2);
            const bool live = ox < a.Wo;
            float s = 0.f;
            for (int dx = 0; dx < ks && live; ++dx) {
                int ix = ox + dx - a.pad;
                if (a.circular) ix = wrap_idx(ix, a.W);
                else if (ix < 0 || ix >= a.W) continue;
                const float* pp = part + (dx * a.W + ix) * QP;
                for (int q = sub; q < Q; q += 4) s += pp[q];
            }
            s += __shfl_xor(s, 1);
            s += __shfl_xor(s, 2);
            if (!live || sub != 0) continue;
            const size_t o = (size_t)row * a.Wo + ox;
            float v = s + (a.bias ? a.bias[0] : 0.f);
            if (a.bias_b) v += a.bias_b[b];
            if (a.resid) v += a.resid[o];
            a.y[o] = thin_act(v, a.act);
        }
    }
}

size_t cout1_lds(const ThinConv& a) {
    return ((size_t)a.ks * a.ks * a.Cin + (size_t)a.ks * a.W * ((a.Cin / 4) | 1)) * sizeof(float);
}

}  // namespace

// tcx_conv2d's one-channel forms (conv.hip): true when this shape runs here
bool thin_conv_takes(const ThinConv& a) {
    static const bool off = getenv("TCX_THIN") && getenv("TCX_THIN")[0] == '0';  // A/B: the MFMA kernels
    if (off || a.ks < 1 || a.ks > 7 || a.B <= 0 || (size_t)a.B * a.Ho >= (1u << 31)) return false;
    if (a.Cin == 1 && a.Cout % 4 == 0 && a.ks * a.ks * a.Cout <= 8192 && a.Wo + a.ks - 1 <= 4096 && aligned16(a.y) &&
        (!a.resid || aligned16(a.resid)) && (!a.bias_b || aligned16(a.bias_b)))
        return true;
    return a.Cout == 1 && a.Cin % 4 == 0 && cout1_lds(a) <= 48 * 1024 && aligned16(a.x) && aligned16(a.w);
}

int launch_thin_conv(const ThinConv& a, hipStream_t st) {
    if (a.Cin == 1) {
        hipLaunchKernelGGL(k_thin_cin1, dim3(std::min(a.B * a.Ho, 2048)), dim3(256),
                           ((size_t)a.ks * a.ks * a.Cout + a.Cout + (size_t)a.ks * (a.Wo + a.ks - 1)) * sizeof(float), st,
                           a);
    } else {
        hipLaunchKernelGGL(k_thin_cout1, dim3(std::min(a.B * a.Ho, 2048)), dim3(256), cout1_lds(a), st, a);
    }
    return check_launch("thin conv");
}

// ---------------------------------------------------------------- weight gradient
namespace {

// Work unit = one segment of segw pixels of one image row; a workgroup takes upw consecutive units as S
// streams x Q = C/4 channel quads (stream s: units s, s + S, ...).  Thread (s, q) walks its segment's
// pixels x with the thin operand's 3 x 3 neighbourhood in a sliding register window (3 new values per
// pixel) and keeps 9 float4 sums: acc[tap] += wide[p][4q..4q+3] * thin[p -/+ off(tap)].  The streams
// are then summed through LDS tap by tap in stream order (deterministic) into the workgroup's plane.
constexpr int TW_THREADS = 512;

__global__ __launch_bounds__(TW_THREADS) void k_thin_wgrad(ThinWgrad a) {
    __shared__ float4 red[TW_THREADS];  // [S][Q]
    const int Q = a.C / 4;
    const int s = threadIdx.x / Q, q = threadIdx.x - (threadIdx.x / Q) * Q;
    float4 acc[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[t] = make_float4(0.f, 0.f, 0.f, 0.f);
    const int u0 = blockIdx.x * a.upw;
    const int u1 = min(u0 + a.upw, a.units);
    const int H = a.H, W = a.W;
    auto tv = [&](const float* tb, int ty, int tx) -> float {  // thin value at (ty, tx) of this image
        if (ty < 0) return 0.f;
        if (a.circular) tx = wrap_idx(tx, W);
        else if (tx < 0 || tx >= W) return 0.f;
        return tb[ty * W + tx];
    };
    if (s < a.S) {
        for (int u = u0 + s; u < u1; u += a.S) {
            const int row = u / a.nseg, x0 = (u - row * a.nseg) * a.segw;
            const int b = row / H, y = row - b * H;
            const float* tb = a.thin + (size_t)b * H * W;
            const float* wp = a.wide + ((size_t)row * W + x0) * a.C + 4 * q;
            int trow[3];
            float win[3][3];
#pragma unroll
            for (int dy = 0; dy < 3; ++dy) {
                int ty = y + a.sign * (dy - 1);
                if (a.circular) ty = wrap_idx(ty, H);
                else if (ty < 0 || ty >= H) ty = -1;
                trow[dy] = ty;
#pragma unroll
                for (int j = 0; j < 3; ++j) win[dy][j] = tv(tb, ty, x0 - 1 + j);
            }
            for (int i = 0; i < a.segw; ++i) {
                const float4 v = *reinterpret_cast<const float4*>(wp + (size_t)i * a.C);
#pragma unroll
                for (int dy = 0; dy < 3; ++dy)
#pragma unroll
                    for (int dx = 0; dx < 3; ++dx) {
                        const float g = a.sign > 0 ? win[dy][dx] : win[dy][2 - dx];
                        float4& c = acc[dy * 3 + dx];
                        c.x = fmaf(v.x, g, c.x); c.y = fmaf(v.y, g, c.y);
                        c.z = fmaf(v.z, g, c.z); c.w = fmaf(v.w, g, c.w);
                    }
#pragma unroll
                for (int dy = 0; dy < 3; ++dy) {
                    win[dy][0] = win[dy][1];
                    win[dy][1] = win[dy][2];
                    win[dy][2] = tv(tb, trow[dy], x0 + i + 2);
                }
            }
        }
    }
    float4* out = reinterpret_cast<float4*>(a.part + (size_t)blockIdx.x * 9 * a.C);
#pragma unroll
    for (int t = 0; t < 9; ++t) {
        if (s < a.S) red[s * Q + q] = acc[t];
        __syncthreads();
        if ((int)threadIdx.x < Q) {
            float4 v = red[threadIdx.x];
            for (int k = 1; k < a.S; ++k) {
                const float4 w = red[k * Q + threadIdx.x];
                v.x += w.x; v.y += w.y; v.z += w.z; v.w += w.w;
            }
            out[t * Q + threadIdx.x] = v;  // k index tap C + 4 q (.. + 3)
        }
        __syncthreads();
    }
}

}  // namespace

// tcx_conv_wgrad's one-channel forms (gemm.hip): the split plan for at most max_split partial planes
// of T x C floats, or 0 when this shape does not run here
int thin_wgrad_plan(int B, int H, int W, int Cin, int Cout, int ks, int stride, int max_split, ThinWgrad* a) {
    static const bool off = getenv("TCX_THIN") && getenv("TCX_THIN")[0] == '0';
    const int C = Cin == 1 ? Cout : Cin;
    if (off || stride != 1 || ks != 3 || !(Cin == 1 || Cout == 1) || C % 4 != 0 || C / 4 > TW_THREADS || B <= 0 ||
        max_split < 1 || (long long)B * H * W >= (1ll << 31))
        return 0;
    const int segw = W % 16 == 0 ? 16 : W;
    a->B = B; a->H = H; a->W = W; a->C = C; a->ks = ks;
    a->segw = segw; a->nseg = W / segw;
    a->units = B * H * a->nseg;
    a->S = TW_THREADS / (C / 4);
    const int ns = std::max(1, std::min(std::min(max_split, 256), cdiv(a->units, a->S)));
    a->upw = cdiv(a->units, ns);
    return cdiv(a->units, a->upw);
}

int launch_thin_wgrad(const ThinWgrad& a, int nsplit, hipStream_t st) {
    hipLaunchKernelGGL(k_thin_wgrad, dim3(nsplit), dim3(TW_THREADS), 0, st, a);
    return check_launch("thin conv weight gradient");
}

}  // namespace tcx
