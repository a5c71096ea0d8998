// rbc_kernels.h — launch interface between the C ABI (api.hip) and the
// gfx950 kernels (rbc_kernels.hip).  Internal; not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/hbgpu.h"
#include "dev_err.h"
#include "grid.h"

namespace hbg {

// send_shards' layout precondition of hbg_rbc_encode_merkle: payload k maps to
// shard_len L (hbg_shard_len(D + Q, P) == L) and fits its row (P <= stride,
// the u32 length prefix).  Checked on the host in host mode and by
// rbc_check_plen (+ every encode kernel, which skips such an instance) in
// device mode.
__host__ __device__ inline bool payload_fits(uint64_t P, uint64_t pstride, uint32_t D, uint64_t L) {
    return P <= pstride && P <= 0xFFFFFFFFull && (P + 4 + D - 1) / D == L;
}

// Per-instance coding plan consumed by rs_code_generic:
// out_row[out_idx[o]] = XOR_j coef[o][j] * row[in_idx[j]],  coef follows the
// struct as [n_out][D] bytes; then (16-B aligned, plan_offs_at) the same
// coefficients as split-nibble LDS byte offsets, u32 [D][plan_qpad][2] =
// {(c & 15) * 256, (16 + (c >> 4)) * 256} — read by scalar loads; rows
// o >= n_out are {0, 16 * 256} (the zero entries), so whole output tiles
// run unguarded.
struct CodePlan {
    int32_t status;  // 0 or HBG_E_*
    uint32_t n_out;
    uint8_t in_idx[256];
    uint8_t out_idx[256];
};

__host__ __device__ constexpr uint32_t merkle_nodes(uint32_t n) {
    uint32_t t = 0;
    while (n > 1) {
        t += n;
        n = (n + 1) / 2;
    }
    return t + 1;
}

__host__ __device__ constexpr uint32_t merkle_depth(uint32_t n) {
    uint32_t d = 0;
    while (n > 1) {
        n = (n + 1) / 2;
        ++d;
    }
    return d;
}

__host__ __device__ constexpr uint64_t plan_offs_at(uint32_t D, uint32_t max_out) {
    return (sizeof(CodePlan) + (uint64_t)max_out * D + 15) & ~uint64_t(15);
}

__host__ __device__ constexpr uint32_t nib_off_lo(uint32_t c) { return (c & 15u) * 256u; }
__host__ __device__ constexpr uint32_t nib_off_hi(uint32_t c) { return (16u + (c >> 4)) * 256u; }

constexpr uint32_t kGenericTile = 48;  // output rows per rs_code_generic register tile
__host__ __device__ constexpr uint32_t plan_qpad(uint32_t max_out) {
    return (max_out + kGenericTile - 1) / kGenericTile * kGenericTile;
}

// Compact form of the same coefficients for the fused decoder (data-only
// plans, n_out <= D): per (input j, output o < D2 = round_up(D, 2)) one u16 at
// [j * D2 + o] = lo-nibble table index | (16 + hi nibble) << 8 (its 32-entry
// register table), dense, so a column's indices are D2 / 2 scalar dwords and
// an instance's whole table (22 x 11 dwords at N = 64) stays in the scalar cache.
__host__ __device__ constexpr uint32_t plan_nidx_rows(uint32_t D) { return (D + 1) & ~1u; }
__host__ __device__ constexpr uint64_t plan_nidx_at(uint32_t D, uint32_t max_out) {
    return plan_offs_at(D, max_out) + 8ull * D * plan_qpad(max_out);
}
__host__ __device__ constexpr uint32_t nib_idx_pair(uint32_t c) { return (c & 15u) | ((16u + (c >> 4)) << 8); }

inline uint64_t plan_stride(uint32_t D, uint32_t max_out) {
    return (plan_nidx_at(D, max_out) + 2ull * D * plan_nidx_rows(D) + 15) & ~uint64_t(15);
}

bool has_const_encoder(uint32_t D, uint32_t Q);
bool const_encoder_fits(uint32_t D, uint32_t Q, uint64_t S, uint64_t pstride, bool fused);
hipError_t launch_rs_encode_const(uint32_t D, uint32_t Q, uint8_t* shards, uint64_t S, uint64_t L, uint64_t n,
                                  const uint8_t* payloads, uint64_t pstride, const uint64_t* plen, hipStream_t st);
// Fused send_shards (prefix/pad/chunk + Coding::encode + MerkleTree::from_vec)
// for the (D, Q) with a compile-time coding matrix (has_const_encoder).
// clk / clk_cap: the clock probe (hbg_test_set_clock_probe): 4 u64 stamps per
// workgroup when the grid has at most clk_cap workgroups, else none
hipError_t launch_rbc_encode_merkle(uint32_t D, uint32_t Q, uint8_t* shards, uint64_t S, uint64_t L, uint64_t n,
                                    const uint8_t* payloads, uint64_t pstride, const uint64_t* plen, uint8_t* levels,
                                    hipStream_t st, uint64_t* clk = nullptr, uint64_t clk_cap = 0);
hipError_t launch_pack_rows(uint8_t* shards, uint64_t S, uint64_t L, uint32_t N, uint32_t rows, uint64_t n,
                            const uint8_t* payloads, uint64_t pstride, const uint64_t* plen, hipStream_t st);
hipError_t launch_rbc_check_plen(uint64_t n, const uint64_t* plen, uint64_t pstride, uint32_t D, uint64_t L,
                                 int32_t* err, hipStream_t st);
hipError_t launch_rbc_trivial_status(uint64_t n, uint32_t N, const uint8_t* present, int32_t* status,
                                     hipStream_t st);
hipError_t launch_rs_code_generic(uint8_t* shards, uint64_t S, uint64_t L, uint32_t N, uint32_t D, uint64_t n,
                                  const uint8_t* plans, uint64_t plan_stride, hipStream_t st);
// max_row: plan the missing rows below it (N: all, D: data rows only).
hipError_t launch_rs_plan(const uint8_t* present, uint32_t D, uint32_t Q, uint32_t max_row, uint64_t n,
                          const uint8_t* matrix, uint8_t* plans, uint64_t plan_stride, hipStream_t st);
// After a data-only plan: encode the missing parity rows from the data rows
// (has_const_encoder(D, Q) and const_encoder_fits(D, Q, S, 0, false)).
hipError_t launch_rs_encode_missing(uint32_t D, uint32_t Q, uint8_t* shards, uint64_t S, uint64_t L, uint64_t n,
                                    const uint8_t* present, const uint8_t* plans, uint64_t plan_stride,
                                    hipStream_t st);
// Fused reconstruct + Merkle rebuild after a data-only plan (rs_plan max_row =
// D): missing data rows, missing parity rows, the levels and (out != null) the
// glued payload bytes [0, D*L - 4) of every decodable instance in one launch;
// rbc_glue's status pass then needs no copy pass (launch_rbc_glue copy=false).
bool has_fused_decoder(uint32_t D, uint32_t Q);
hipError_t launch_rbc_decode_merkle(uint32_t D, uint32_t Q, uint8_t* shards, uint64_t S, uint64_t L, uint64_t n,
                                    const uint8_t* present, const uint8_t* plans, uint64_t plan_stride,
                                    uint8_t* levels, uint8_t* out, uint64_t ostride, hipStream_t st);
// split: -1 lane-pair blocks for a partial last generation (<= half the CUs),
// 0 one-lane blocks only, 1 lane-pair blocks only (hbg_test_set_merkle_pairs)
hipError_t launch_merkle_build(const uint8_t* shards, uint64_t S, uint64_t L, uint32_t N, uint64_t n,
                               uint8_t* levels, hipStream_t st, int split = -1);
hipError_t launch_merkle_validate(uint32_t N, uint64_t len, const uint8_t* values, uint64_t vstride,
                                  const uint32_t* index, const uint8_t* digests, uint32_t depth,
                                  const uint32_t* ndig, const uint8_t* roots, uint8_t* ok, uint64_t n,
                                  hipStream_t st, uint32_t views = 1);  // ok: [views][n], every view validates all n
hipError_t launch_rbc_glue(const uint8_t* shards, uint64_t S, uint64_t L, uint32_t N, uint32_t D, uint64_t n,
                           const uint8_t* levels, const uint8_t* roots, const int32_t* rstatus, uint64_t* plen,
                           uint8_t* status, uint8_t* out, uint64_t ostride, hipStream_t st, bool copy = true);
hipError_t launch_rbc_write_proof_msgs(uint32_t N, uint64_t L, const uint8_t* shards, uint64_t S,
                                       const uint8_t* levels, uint64_t n, uint32_t tag, uint64_t m,
                                       const uint64_t* inst, const uint32_t* index, uint8_t* out,
                                       const uint64_t* out_off, int32_t* err, hipStream_t st);
hipError_t launch_rbc_read_msgs(uint32_t N, uint64_t L, const uint8_t* msgs, const uint64_t* msg_off, uint64_t m,
                                uint32_t* tag, uint8_t* values, uint64_t vstride, uint32_t* index,
                                uint8_t* digests, uint32_t* ndig, uint8_t* roots, int32_t* status, hipStream_t st);
uint32_t host_proof_digests(uint32_t N, uint32_t i);
hipError_t launch_wire_frame_pack(uint64_t n, const uint8_t* msg, const uint64_t* msg_off, const uint8_t* sig96,
                                  uint8_t* frames, const uint64_t* frame_off, int32_t* err, hipStream_t st);
hipError_t launch_synth(uint32_t tag, uint64_t first, uint64_t nbytes, uint8_t* out, uint64_t ostride, uint64_t n,
                        hipStream_t st);

}  // namespace hbg
