// k_conv3g instantiated for rows of 16 pixels (conv3g.hpp; split per width for parallel builds)
#include "conv3g.hpp"

namespace tcx {
int launch3g_w16(const ConvParams& p, hipStream_t st) { return launch3g<16>(p, st); }
}  // namespace tcx
