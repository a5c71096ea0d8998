/* hbgpu_testing.h — unit-test hook of libhbgpu.so (not part of the drop-in
 * surface): runs one BLS12-381 building block per item on the device so the
 * parity tests can pin each layer against the oracle.
 * op: 0 fp_mul  1 fp_inv  2 fp2_sqrt  3 g1_decompress  4 g2_decompress
 *     5 pairing  6 hash_g2(seed)  7 miller_loop  8 final_exponentiation
 * in/out: [n][in_words] / [n][out_words] u32, field values canonical LE limbs. */
#ifndef HBGPU_TESTING_H
#define HBGPU_TESTING_H
#include <stdint.h>
#include "hbgpu.h"
#ifdef __cplusplus
extern "C" {
#endif
/* Choose the share-verification schedule of hbg_tdec_verify_shares /
 * hbg_tdec_threshold_decrypt / hbg_sig_verify_shares: 1 (the default) the
 * batched small-exponent test with per-share fallback from 393,216 shares up
 * and one independent pairing check per share below (public-key fixed-base
 * tables when each key verifies >= 2048 shares), 2 batched at every size with
 * the tables always built, 3 batched at every size, 0 one independent pairing
 * check per share.  All return identical bits. */
int hbg_test_set_tdec_batched(hbg_ctx *ctx, int on);
/* Choose the schedule of hbg_rbc_encode_merkle for the (D, Q) with a
 * compile-time coding matrix: 0 rs_encode_const then merkle_build (two
 * launches), 1 the single-launch rbc_encode_merkle kernel (encode pass +
 * LDS transpose + SHA3 leaves + tree), -1 (the default) the fused kernel
 * where it measured faster on MI355X — (D, Q) = (22, 42), N = 64 — and two
 * launches elsewhere.  Both write identical shards and levels. */
int hbg_test_set_rbc_fused(hbg_ctx *ctx, int on);
/* Choose the reconstruct schedule of hbg_rs_reconstruct / hbg_rbc_decode for
 * the (D, Q) with a compile-time coding matrix: 1 rebuild the missing data
 * rows from the first D present rows, then encode the missing parity rows
 * from the data rows (rse's reconstruct order); 0 rebuild every missing row in
 * one pass of the run-time coder; -1 (the default) 1 where Q > 16, where it
 * measured faster on MI355X.  Identical shards. */
int hbg_test_set_rs_split(hbg_ctx *ctx, int on);
/* Choose the schedule of hbg_rbc_decode: 0 rs_plan -> run-time coder (->
 * constant parity encoder, per hbg_test_set_rs_split) -> merkle_build; 1 or
 * -1 (the default) the single-launch rbc_decode_merkle kernel (reconstruct +
 * Merkle rebuild, the missing rows transposed through LDS) where it exists —
 * (D, Q) = (22, 42), N = 64 — and the three-launch schedule elsewhere.
 * Identical shards, levels, statuses and payloads. */
int hbg_test_set_rbc_decode_fused(hbg_ctx *ctx, int on);
/* Choose merkle_build's leaf hashing (hbg_merkle_build, the two-launch
 * hbg_rbc_encode_merkle / hbg_rbc_decode schedules): 0 one lane a leaf; 1 a
 * lane pair a leaf (each lane half of every Keccak word) in every block; -1
 * (the default) lane pairs for the blocks past the launch's last whole
 * generation (one block a CU) when they would fill at most half the CUs, one
 * lane elsewhere.  Identical levels. */
int hbg_test_set_merkle_pairs(hbg_ctx *ctx, int on);
/* Clock probe of the fused send_shards kernel (rbc_encode_merkle): while set,
 * every hbg_rbc_encode_merkle launch of at most cap_workgroups workgroups
 * (one per instance at N = 64) writes 4 u64 per workgroup to dev_buf
 * (device memory): s_memtime (shader clock) at entry and exit, then
 * s_memrealtime (constant 100 MHz) at entry and exit.  cap_workgroups = 0
 * turns it off (the default; the product path never sets it). */
int hbg_test_set_clock_probe(hbg_ctx *ctx, uint64_t *dev_buf, uint64_t cap_workgroups);
/* The BLS12-381 kernels exist in two builds with identical results: the
 * throughput build (G1 kernels at two waves per SIMD, pairing / G2 kernels at
 * one) and the latency build (every kernel at one wave per SIMD's register
 * budget: fewer dependent stalls and spills for a lone wave).  Launches of at most `lanes` work-items take the latency
 * build (default 65,536 = one wave per SIMD; 0: never; UINT64_MAX: always).
 * Process-wide; returns the previous value. */
uint64_t hbg_test_set_latency_lanes(uint64_t lanes);
int hbg_test_bls(hbg_ctx *ctx, int op, uint32_t n, const uint32_t *in, uint32_t in_words, uint32_t *out,
                 uint32_t out_words);
#ifdef __cplusplus
}
#endif
#endif
