// tdec_kernels.h — launch interface of the ThresholdDecrypt kernels (internal).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/hbgpu.h"

namespace hbg {
namespace bls {

constexpr uint32_t kLineWordsPerPoint = 72 * 68;  // G2Prepared: 68 x (3 Fp2) x 12 u32
constexpr uint32_t kAffWords = 32;                // affine record: x[12] y[12] flags

hipError_t launch_tdec_ct_prepare(uint32_t n, const uint8_t* U48, const uint8_t* V, const uint64_t* V_off,
                                  const uint8_t* W96, uint32_t* ct_u, int32_t* ct_status, uint32_t* coefH,
                                  uint32_t* coefW, hipStream_t st);
hipError_t launch_tdec_pk_prepare(uint32_t n, const uint8_t* pk48, uint32_t* pk_aff, int32_t* pk_status,
                                  hipStream_t st);
hipError_t launch_tdec_verify_shares(uint64_t n, const uint8_t* share48, const uint32_t* share_ct,
                                     const uint32_t* share_pk, const uint32_t* ct_u, const int32_t* ct_status,
                                     const uint32_t* coefH, const uint32_t* coefW, const uint32_t* pk_aff,
                                     const int32_t* pk_status, uint8_t* ok, hipStream_t st);
hipError_t launch_tdec_ct_verify(uint32_t n, const uint32_t* ct_u, const int32_t* ct_status, const uint32_t* coefH,
                                 const uint32_t* coefW, uint8_t* ok, hipStream_t st);
hipError_t launch_tdec_combine(uint32_t n, uint32_t t, const uint8_t* share48, const uint32_t* idx,
                               const uint8_t* V, const uint64_t* V_off, uint8_t* out, int32_t* status,
                               uint32_t* scratch, hipStream_t st);
hipError_t launch_tdec_test(int op, uint32_t n, const uint32_t* in, uint32_t* out, uint32_t in_words,
                            uint32_t out_words, uint32_t* lines, hipStream_t st);

}  // namespace bls
}  // namespace hbg
