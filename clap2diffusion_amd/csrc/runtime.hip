// Host-side runtime state of libc2d_hip.so, all of it here ("no global
// mutable state beyond a per-device kernel table that is initialised once under
// std::call_once"):
//   * the tuning switches (A/B-only environment variables), read once per process under
//     std::call_once into an immutable struct;
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

static int env_int(const char* name, int dflt) {
    const char* e = getenv(name);
    return e ? atoi(e) : dflt;
}

const Tuning& tuning() {
    static Tuning t;
    static std::once_flag once;
    std::call_once(once, [] {
        t.gemm_mode = env_int("C2D_GEMM_MODE", 0);        // 2: register-staged kernels only (A/B)
        t.gemm_korder = env_int("C2D_GEMM_KORDER", 1);    // 3x3 K order: channel-block outer (1) / tap outer (0)
        t.gemm_lds_epi = env_int("C2D_GEMM_LDSEPI", 1);   // 0: direct 32x32 GEGLU epilogue (A/B)
        t.splitk_f16 = env_int("C2D_SPLITK_F16", 0) != 0;  // 1: split-K partials in fp16 (A/B only: cancelling partials lose range / precision)
        t.tail_split = env_int("C2D_TAIL_SPLIT", 1);   // 0: no image split of a quantisation tail (A/B)
        t.gemm_sp = env_int("C2D_GEMM_SP", 0);         // 1: tiles 40 / 41 run their software-pipelined twins 60 / 61
        t.panel_regb = env_int("C2D_PANEL_REGB", 0);   // 1: the K = 320 panel GEMM loads its weights into registers (A/B)
        t.panel_stagger = env_int("C2D_PANEL_STAGGER", 2);   // panel GEMM: late start of waves 4-7, x 2048 cycles
        t.attn_negc = env_int("C2D_ATTN_NEGC", 1);
        t.attn_res = env_int("C2D_ATTN_RES", 1);
        t.attn_w8 = env_int("C2D_ATTN_W8", 1);
        t.attn_pp = env_int("C2D_ATTN_PP", 0);
        t.gn_blocks = env_int("C2D_GN_BLOCKS", 512);
        if (t.gn_blocks < 64) t.gn_blocks = 512;
        t.gn_apply_blocks = env_int("C2D_GN_APPLY_BLOCKS", 2048);
        if (t.gn_apply_blocks < 64) t.gn_apply_blocks = 2048;
        t.gn_fused_hw = env_int("C2D_GN_FUSED_HW", 256);
        t.gn_fold = env_int("C2D_GN_FOLD", 1);   // 0: partial + finalize + apply (A/B)
        t.gn_fold_cap = env_int("C2D_GN_FOLD_CAP", 32);   // most partial blocks per image on the fold path
        if (t.gn_fold_cap < 1) t.gn_fold_cap = 32;
        t.gn_fold_apply_blocks = env_int("C2D_GN_FOLD_APPLY_BLOCKS", 1024);   // apply workgroups per launch (fold path, batches below 8 images)
        if (t.gn_fold_apply_blocks < 64) t.gn_fold_apply_blocks = 1024;
#ifdef C2D_ENABLE_ABLATION
        t.gemm_abl = env_int("C2D_GEMM_ABL", 0);
        t.attn_abl = env_int("C2D_ATTN_ABL", 0);
#else
        t.gemm_abl = 0;
        t.attn_abl = 0;
#endif
    });
    return t;
}

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
