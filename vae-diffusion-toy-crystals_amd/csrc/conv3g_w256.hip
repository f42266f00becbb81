// k_conv3g instantiated for rows of 256 pixels, bf16 (slim halo) only (conv3g.hpp; config 5's 256^2 level)
#include "conv3g.hpp"

namespace tcx {
int launch3g_w256(const ConvParams& p, hipStream_t st) { return launch3g<256>(p, st); }
}  // namespace tcx
