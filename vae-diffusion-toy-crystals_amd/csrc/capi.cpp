// libtcx C-ABI plumbing: thread-local error string and version.
#include <cstdarg>
#include <cstdio>

#include "common.hpp"

namespace tcx {
static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    std::vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}
}  // namespace tcx

namespace tcx {
namespace {
constexpr int kRing = 4096;
struct Prof {
    bool on = false;
    bool created = false;
    hipEvent_t ev[2 * kRing];
    double flops[kRing];
    bool pending[kRing];
    int head = 0;
    long long launches = 0;
    double ms = 0.0, fl = 0.0;
} g_prof;

void retire(int slot) {
    if (!g_prof.pending[slot]) return;
    (void)hipEventSynchronize(g_prof.ev[2 * slot + 1]);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, g_prof.ev[2 * slot], g_prof.ev[2 * slot + 1]);
    g_prof.ms += ms;
    g_prof.fl += g_prof.flops[slot];
    g_prof.launches += 1;
    g_prof.pending[slot] = false;
}
}  // namespace

void prof_begin(hipStream_t st) {
    if (!g_prof.on) return;
    const int slot = g_prof.head;
    retire(slot);
    (void)hipEventRecord(g_prof.ev[2 * slot], st);
}

void prof_end(hipStream_t st, double flops) {
    if (!g_prof.on) return;
    const int slot = g_prof.head;
    (void)hipEventRecord(g_prof.ev[2 * slot + 1], st);
    g_prof.flops[slot] = flops;
    g_prof.pending[slot] = true;
    g_prof.head = (slot + 1) % kRing;
}
}  // namespace tcx

extern "C" const char* tcx_last_error(void) { return tcx::g_err; }

extern "C" int tcx_prof_enable(int on) {
    using tcx::g_prof;
    if (on && !g_prof.created) {
        for (int i = 0; i < 2 * tcx::kRing; ++i) {
            if (hipEventCreate(&g_prof.ev[i]) != hipSuccess) {
                tcx::set_error("tcx_prof_enable: hipEventCreate failed");
                return TCX_EHIP;
            }
        }
        g_prof.created = true;
    }
    for (int i = 0; i < tcx::kRing; ++i) g_prof.pending[i] = false;
    g_prof.head = 0;
    g_prof.launches = 0;
    g_prof.ms = g_prof.fl = 0.0;
    g_prof.on = on != 0;
    return TCX_OK;
}

extern "C" int tcx_prof_read(double* total_ms, long long* launches, double* flops) {
    using tcx::g_prof;
    if (g_prof.created)
        for (int i = 0; i < tcx::kRing; ++i) tcx::retire(i);
    if (total_ms) *total_ms = g_prof.ms;
    if (launches) *launches = g_prof.launches;
    if (flops) *flops = g_prof.fl;
    return TCX_OK;
}
extern "C" int tcx_version(void) { return 1; }
