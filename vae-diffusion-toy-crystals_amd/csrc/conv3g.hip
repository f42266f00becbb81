// conv3g.hip — dispatch of k_conv3g (kernel and launcher in conv3g.hpp, compiled per row width in
// conv3g_w{16,32,64,128}.hip) and the fragment-ordered weight pack it reads.
#include "conv3g.hpp"

namespace tcx {
int launch3g_w16(const ConvParams& p, hipStream_t st);
int launch3g_w32(const ConvParams& p, hipStream_t st);
int launch3g_w64(const ConvParams& p, hipStream_t st);
int launch3g_w128(const ConvParams& p, hipStream_t st);
int launch3g_w256(const ConvParams& p, hipStream_t st);
namespace {

// Fragment-ordered copy of h2 conv weights for k_conv3g: wf[nblk][c = 9 j + t][n][hi, lo][lane][16 B]
// = the 8 hi (or lo) halves of weight row 96 nblk + 32 n + (lane & 31), packed k = t Cin + 16 j +
// 8 (lane >> 5) (h2 group of 8 channels: [8 hi][8 lo] = 32 B at byte 4 k of the row).
__global__ void k_pack_frag(const char* __restrict__ wh, char* __restrict__ wf, int kpad, int Cin, int nblk_n) {
    const int cpt = Cin / G_KC, nch = 9 * cpt;
    const size_t n16 = (size_t)nblk_n * nch * G_NT * 2 * 64;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
        const int lane = (int)(i & 63);
        size_t q = i >> 6;
        const int hl = (int)(q & 1);
        q >>= 1;
        const int n = (int)(q % G_NT);
        q /= G_NT;
        const int c = (int)(q % nch);
        const int nb = (int)(q / nch);
        const int j = c / 9, t = c - 9 * j;
        const int row = nb * 96 + n * 32 + (lane & 31);
        const int k = t * Cin + j * G_KC + 8 * (lane >> 5);
        *reinterpret_cast<float4*>(wf + i * 16) =
            *reinterpret_cast<const float4*>(wh + ((size_t)row * kpad + k) * 4 + hl * 16);
    }
}

}  // namespace

// TCX_CONV3G=0 keeps k_conv3p on every row width (A/B measurements; no GroupNorm prologue then)
bool conv3g_enabled() {
    static const bool on = [] {
        const char* e = getenv("TCX_CONV3G");
        return !(e && e[0] == '0');
    }();
    return on;
}

bool conv3g_covers(int H, int W, int Cin, int cout_pad, bool bf) {
    if (!conv3g_enabled() || !(W == 16 || W == 32 || W == 64 || W == 128 || (W == 256 && bf))) return false;
    const int tp = g_tp(g_nw(W));
    return H % (tp / W) == 0 && (H * W) % tp == 0 && Cin % 32 == 0 && Cin <= 384 && cout_pad % 96 == 0;
}

bool conv3g_applies(const ConvParams& p, int cout_pad) {
    return p.wf != nullptr && conv3g_covers(p.H, p.W, p.Cin, cout_pad, p.bf) && p.ks == 3 && p.stride == 1 && p.pad_y == 1 && p.pad_x == 1 &&
           p.Hi == p.H && p.Wi == p.W && p.C1 % G_KC == 0 && (p.C2 == 0 || p.C2 == p.C1) && p.kpad == 9 * p.Cin &&
           p.osy == 1 && p.osx == 1;
}

// conv3l.hip: the same conv with the B fragments staged once per workgroup in an LDS ring
bool conv3l_takes(const ConvParams& p);
int launch_conv3l(const ConvParams& p, hipStream_t st);
int launch_conv3m(const ConvParams& p, hipStream_t st);
// conv3lb.hip: the bf16 LDS-DMA form for rows of 64 / 128 / 256 pixels (h2 / bf16 record sources)
bool conv3lb_takes(const ConvParams& p);
int launch_conv3lb(const ConvParams& p, hipStream_t st);
// conv3mb.hip (round 6): config 5's b2 3x3 convs on 16x16x32 bf16 tap pairs, three-slot weight ring
bool conv3mb_takes(const ConvParams& p);
int launch_conv3mb(const ConvParams& p, hipStream_t st);

int launch_conv3g(ConvParams& p, int cout_pad, hipStream_t st) {
    p.n_nblk = cout_pad / 96;
    if (p.M == 0) return TCX_OK;
    prof_begin(st);
    int rc;
    if (p.bf == 2 && conv3mb_takes(p)) rc = launch_conv3mb(p, st);  // b2 sources (chunk-major source 2 too)
    else if (p.cm2 && p.bf == 2) rc = launch_conv3lb(p, st);  // chunk-major b2 source 2 (conv3lb_takes checked)
    else if (p.cm2) rc = launch_conv3m(p, st);  // chunk-major source 2 (tcx_conv2d_h2_pro checked conv3m_takes)
    else if (conv3lb_takes(p)) rc = launch_conv3lb(p, st);
    else if (conv3l_takes(p)) rc = launch_conv3l(p, st);
    else if (p.W == 64) rc = launch3g_w64(p, st);
    else if (p.W == 32) rc = launch3g_w32(p, st);
    else if (p.W == 16) rc = launch3g_w16(p, st);
    else if (p.W == 128) rc = launch3g_w128(p, st);
    else rc = launch3g_w256(p, st);
    prof_end(st, 2.0 * (double)p.M * p.Cout * 9 * p.Cin);
    return rc;
}

}  // namespace tcx

using namespace tcx;

extern "C" size_t tcx_conv_weight_h2_frag_bytes(int cout_pad, int Cin) {
    return (cout_pad % 96 == 0 && Cin % 32 == 0) ? (size_t)cout_pad * 9 * Cin * 4 : 0;
}

extern "C" int tcx_pack_conv_weight_h2_frag(const void* wh, void* wf, int cout_pad, int kpad, int Cin, void* stream) {
    TCX_REQUIRE(wh && wf && cout_pad > 0 && cout_pad % 96 == 0 && Cin > 0 && Cin % 32 == 0 && kpad == 9 * Cin,
                "tcx_pack_conv_weight_h2_frag: needs a 3x3 h2 weight with cout_pad %% 96 == 0, Cin %% 32 == 0");
    TCX_REQUIRE(aligned16(wh) && aligned16(wf), "tcx_pack_conv_weight_h2_frag: 16-B alignment");
    const size_t n16 = (size_t)cout_pad * 9 * Cin * 4 / 16;
    const int blocks = (int)std::min<size_t>((n16 + 255) / 256, 4096);
    hipLaunchKernelGGL(k_pack_frag, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const char*)wh, (char*)wf, kpad,
                       Cin, cout_pad / 96);
    return check_launch("tcx_pack_conv_weight_h2_frag");
}
