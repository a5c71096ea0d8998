// grid.h — launch-size guard shared by the kernel launchers.  Internal.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace hbg {

// One launch's grid: at most 2^31 - 1 workgroups and 2^32 - 1 work-items (the
// AQL dispatch packet's 32-bit grid size).  Launchers return
// hipErrorInvalidConfiguration for a larger batch (the C ABI: HBG_E_ARG, the
// caller splits the batch) instead of truncating the grid.
inline bool grid_fits(uint64_t blocks, uint32_t threads) {
    return blocks <= 0x7FFFFFFFull && blocks * threads <= 0xFFFFFFFFull;
}

// Set by HBG_GRID_CHECK when it refuses a grid, consumed by the C ABI's error
// mapping: only a refusal of this guard is an argument error (HBG_E_ARG); a
// hipErrorInvalidConfiguration from the runtime itself stays HBG_E_DEVICE.
inline thread_local bool g_grid_refused = false;
inline bool take_grid_refused() {
    const bool r = g_grid_refused;
    g_grid_refused = false;
    return r;
}

}  // namespace hbg

#define HBG_GRID_CHECK(blocks, threads)                      \
    do {                                                     \
        if (!::hbg::grid_fits((blocks), (threads))) {        \
            ::hbg::g_grid_refused = true;                    \
            return hipErrorInvalidConfiguration;             \
        }                                                    \
    } while (0)
