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

}  // namespace hbg

#define HBG_GRID_CHECK(blocks, threads)                                                  \
    do {                                                                                 \
        if (!::hbg::grid_fits((blocks), (threads))) return hipErrorInvalidConfiguration; \
    } while (0)
