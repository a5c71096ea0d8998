// dev_err.h — device-side argument errors of the C ABI.
//
// A call made with HBG_DEVICE | HBG_ASYNC returns before its kernels run, so
// an argument the kernels find invalid (an out-of-range index, a payload
// length that does not map to shard_len, an oversized frame) cannot be its
// return value.  Kernels record the FIRST such code in the context's device
// word (atomicCAS from 0, a vector atomic); the next synchronous call or
// hbg_sync() returns it and clears it (api.hip take_error).  The per-item
// outputs of the offending items carry their own invalid values (ok = 0,
// status = HBG_E_ARG, an unwritten message ...).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace hbg {

__device__ __forceinline__ void flag_error(int32_t* err, int32_t code) {
    if (err) atomicCAS(err, 0, code);
}

}  // namespace hbg
