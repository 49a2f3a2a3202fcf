// Host-side runtime state of libc2d_hip.so, all of it here ("no global
// mutable state beyond a per-device kernel table that is initialised once under
// std::call_once"):
//   * the timing-ablation masks, read from the environment in the ablation build only (the
//     tuning constants are compile-time, common.h: the production library reads no environment);
//   * the per-(kernel, device) LDS attribute table (common.h ensure_lds): one
//     std::once_flag per device and kernel instantiation;
//   * the explicit plan override of c2d_set_plan_override (tests / tuning sweeps only;
//     the production library never reads a plan from the environment).
#include <atomic>
#include <mutex>
#include <stdlib.h>
#include "common.h"

namespace c2d {

thread_local int g_last_hip_error = 0;

#ifdef C2D_ENABLE_ABLATION
static int env_int(const char* name, int dflt) {
    const char* e = getenv(name);
    return e ? atoi(e) : dflt;
}
int ablation_gemm() {
    static const int v = env_int("C2D_GEMM_ABL", 0);
    return v;
}
int ablation_attn() {
    static const int v = env_int("C2D_ATTN_ABL", 0);
    return v;
}
#else
int ablation_gemm() { return 0; }
int ablation_attn() { return 0; }
#endif

static std::atomic<int> g_force_tile{0}, g_force_split{0};

int plan_override_tile() { return g_force_tile.load(std::memory_order_relaxed); }
int plan_override_split() { return g_force_split.load(std::memory_order_relaxed); }

int current_device() {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) dev = 0;
    return dev;
}

}  // namespace c2d

extern "C" int c2d_set_plan_override(int tile_id, int ksplit) {
    if (tile_id < 0 || ksplit < 0 || ksplit > 64) return C2D_E_ARG;
    c2d::g_force_tile.store(tile_id, std::memory_order_relaxed);
    c2d::g_force_split.store(ksplit, std::memory_order_relaxed);
    return C2D_OK;
}

extern "C" int c2d_get_plan_override(int* tile_id, int* ksplit) {
    if (!tile_id || !ksplit) return C2D_E_ARG;
    *tile_id = c2d::g_force_tile.load(std::memory_order_relaxed);
    *ksplit = c2d::g_force_split.load(std::memory_order_relaxed);
    return C2D_OK;
}

extern "C" int c2d_last_hip_error(void) { return c2d::g_last_hip_error; }
