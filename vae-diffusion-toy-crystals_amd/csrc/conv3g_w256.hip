// k_conv3g instantiated for rows of 256 pixels, bf16 (slim halo) only (conv3g.hpp; config 5's 256^2 level)
#include "conv3g.hpp"

#include <cstdlib>

namespace tcx {
int launch3g_w256(const ConvParams& p, hipStream_t st) {
    static const bool nw8 = [] {  // TCX_G256NW (temporary A/B): 8 waves, 512-px tiles, one workgroup per CU
        const char* e = getenv("TCX_G256NW");
        return e && atoi(e) == 8;
    }();
    return nw8 ? launch3g<256, 8>(p, st) : launch3g<256, 4>(p, st);
}
}  // namespace tcx
