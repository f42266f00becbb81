// k_conv3g instantiated for rows of 256 pixels, bf16 (slim halo) only (conv3g.hpp; config 5's 256^2 level).
// 8 waves / 512-px tiles measured equal to 4 waves / 256-px tiles (profiles/r03_w_nw*: 5.53 vs 5.54 img/s).
#include "conv3g.hpp"

namespace tcx {
int launch3g_w256(const ConvParams& p, hipStream_t st) { return launch3g<256, 4>(p, st); }
}  // namespace tcx
