// tdec_kernels.h — launch interface of the ThresholdDecrypt kernels (internal).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/hbgpu.h"

namespace hbg {
namespace bls {

constexpr uint32_t kLineWordsPerPoint = 72 * 68;  // G2Prepared: 68 x (3 Fp2) x 12 u32
constexpr uint32_t kAffWords = 32;                // affine record: x[12] y[12] flags
constexpr uint32_t kBatchShares = 64;             // batched verification: shares per batch (8 x 8)

struct BatchDesc;
struct CheckItem;
// Secret key of the batch weights: 32 bytes drawn from getrandom(2) once per
// context (hbg_init) and never exposed, so a sender cannot predict the weight
// its share gets, nor grind shares offline against them.
struct BatchKey {
    uint32_t w[8];
};
constexpr uint32_t kBatchDescBytes = 16, kCheckItemBytes = 8, kBinItemBytes = 16;
constexpr uint32_t kBatchSumBytes = 64 * 2 * 36 * 4;  // per batch: the binary tree's root + left nodes (2 G1 sums each)
constexpr uint32_t kGtBytes = 144 * 4;                // a GT value (Fp12)
constexpr int kBinRounds = 6;                          // binary group-testing rounds after the batch check
constexpr uint32_t kSigBatchSumBytes = 21 * (36 + 72) * 4;  // per batch: G1 + G2 Jacobian sums of 21 tree nodes
// The sig_* check rounds run in launches of at most kResidentBlocks 64-lane
// blocks (2 waves per SIMD x 1,024 SIMDs: the TDec kernels' resident limit);
// their per-lane scratch (G2Prepared lines) is sized for kResidentBlocks * 64.
constexpr uint32_t kResidentBlocks = 2048;

// Ciphertext table: tdec_ct_decode (U + subgroup check -> ct_u, u_status:
// what the share leaves read), tdec_ct_prepare (H = hash_g1_g2(U, V) and its
// lines for U-valid ciphertexts; vdig [n][32] scratch for SHA3(V) of the
// items with |V| > 64) and, on a second stream, tdec_ct_prepare_w (W +
// subgroup check -> the final ct_status, W's G2Prepared lines).
hipError_t launch_tdec_ct_decode(uint32_t n, const uint8_t* U48, uint32_t* ct_u, int32_t* u_status, hipStream_t st);
hipError_t launch_tdec_ct_prepare(uint32_t n, const uint8_t* U48, const uint8_t* V, const uint64_t* V_off,
                                  const int32_t* ct_status, uint32_t* coefH, uint8_t* vdig, hipStream_t st);
hipError_t launch_tdec_ct_prepare_w(uint32_t n, const uint8_t* W96, uint32_t* ct_u, const int32_t* u_status,
                                    int32_t* ct_status, uint32_t* coefW, hipStream_t st);
// H (sponge inline) and W's preparation in one grid (the two above, concurrent)
hipError_t launch_tdec_ct_prepare_hw(uint32_t n, const uint8_t* U48, const uint8_t* V, const uint64_t* V_off,
                                     const uint8_t* W96, uint32_t* ct_u, const int32_t* u_status, int32_t* ct_status,
                                     uint32_t* coefH, uint32_t* coefW, hipStream_t st);
// xor_with_hash's keystream: out = in ^ keystream(seeds[k]) per item (status[k] != 0: skipped; nullable)
hipError_t launch_tdec_keystream_xor(uint64_t n, const uint8_t* seeds, const uint8_t* in, const uint64_t* off,
                                     uint8_t* out, const int32_t* status, hipStream_t st);
hipError_t launch_tdec_v_digest(uint64_t n, const uint8_t* V, const uint64_t* V_off, uint8_t* dig, hipStream_t st);
hipError_t launch_tdec_pk_prepare(uint32_t n, const uint8_t* pk48, uint32_t* pk_aff, int32_t* pk_status,
                                  hipStream_t st);
// cap: items the grid is sized for; n_dev (nullable): the device word holding
// the actual count (<= cap) — the group-testing rounds never round-trip a
// count through the host.
hipError_t launch_tdec_verify_shares(uint64_t cap, const uint32_t* n_dev, const uint8_t* share48,
                                     const uint32_t* share_ct, const uint32_t* share_pk, const uint32_t* ct_u,
                                     const int32_t* ct_status, const uint32_t* coefH, const uint32_t* coefW,
                                     const uint32_t* pk_aff, const int32_t* pk_status, uint8_t* ok, hipStream_t st,
                                     const uint32_t* sel = nullptr, uint32_t* share_aff = nullptr);
hipError_t launch_tdec_index_sanitize(uint64_t n, const uint32_t* a, uint32_t a_bound, const uint32_t* b,
                                      uint32_t b_bound, uint32_t* a_out, uint32_t* b_out, int32_t* err,
                                      hipStream_t st);
size_t tdec_batch_temp_bytes(uint32_t n);
hipError_t launch_tdec_batch_plan(uint32_t n, uint32_t n_keys, const uint32_t* share_ct, uint32_t* keys,
                                  uint32_t* perm, uint32_t* tmp_a, uint32_t* tmp_b, BatchDesc* desc, void* temp,
                                  size_t temp_bytes, uint32_t* nb_dev, hipStream_t st);
uint32_t tdec_batch_bound(uint32_t n, uint32_t n_keys);  // upper bound of the batch count
void tdec_debug_bounds(uint64_t n, uint64_t nb_max, uint64_t n_ct1, uint64_t n_pk1);  // -DHBG_DEBUG_CHECKS only
hipError_t launch_tdec_batch_leaves(uint32_t nb_max, const uint32_t* nb_dev, uint32_t n_ct, const BatchDesc* desc,
                                    const uint32_t* perm, const uint8_t* share48, const uint32_t* share_pk,
                                    const uint8_t* U48, const int32_t* ct_status, const uint32_t* pk_aff,
                                    const int32_t* pk_status, const uint32_t* pk_tbl, uint32_t* sums,
                                    uint8_t* leaf_ok, const BatchKey& key, hipStream_t st,
                                    uint32_t* share_aff = nullptr);
size_t tdec_pk_table_bytes(uint32_t n_pk);
// layout 0: the coin shares' 64-bit-half weights; 1: the decryption shares'
// four 32-bit quarters (windows 4..7 hold [|x|] PK)
hipError_t launch_tdec_pk_table(uint32_t n_pk, const uint32_t* pk_aff, uint32_t* tbl, hipStream_t st,
                                uint32_t layout);
// Binary group testing (tdec_kernels.hip "batched share verification"):
// round 0 over the batches, then kBinRounds rounds over BinItem lists (count:
// a device word; items past next_cap hand their leaves to the per-share list).
// gt_out / gt_in: 2 GT values per item of the writing / previous round.
struct BinItem;
hipError_t launch_tdec_bin_root(uint32_t cap, const uint32_t* nb_dev, const BatchDesc* desc, const uint32_t* perm,
                                const uint32_t* sums, const uint8_t* leaf_ok, const int32_t* ct_status,
                                const uint32_t* ct_u, const uint32_t* coefH, const uint32_t* coefW, uint8_t* ok,
                                uint32_t* gt_out, BinItem* next, uint32_t* next_n, uint32_t next_cap,
                                uint32_t* fail_list, uint32_t* fail_n, hipStream_t st);
hipError_t launch_tdec_bin_step(uint32_t cap, const uint32_t* n_dev, const BinItem* items, const BatchDesc* desc,
                                const uint32_t* perm, const uint32_t* sums, const uint8_t* leaf_ok,
                                const uint32_t* ct_u, const uint32_t* coefH, const uint32_t* coefW, uint8_t* ok,
                                const uint32_t* gt_in, uint32_t* gt_out, BinItem* next, uint32_t* next_n,
                                uint32_t next_cap, uint32_t* fail_list, uint32_t* fail_n, hipStream_t st);
hipError_t launch_bls_sign(uint64_t n, uint32_t n_sk, const uint8_t* sk32, const uint32_t* msg_sk,
                           const uint8_t* msg, const uint64_t* off, uint8_t* sig96, int32_t* err, hipStream_t st);
hipError_t launch_wire_verify_frames(uint64_t n, const uint32_t* pk_aff, const int32_t* pk_status, uint32_t n_pk,
                                     const uint32_t* frame_pk, const uint8_t* frames, const uint64_t* off,
                                     uint32_t* lines, int32_t* status, hipStream_t st);
hipError_t launch_bls_verify(uint64_t n, uint32_t n_pk, const uint32_t* pk_aff, const int32_t* pk_status,
                             const uint32_t* msg_pk, const uint8_t* msg, const uint64_t* off, const uint8_t* sig96,
                             uint32_t* lines, uint8_t* ok, int32_t* err, hipStream_t st);
// seeds / vdig: [n][32] scratch; est: [n] int32 scratch
hipError_t launch_tdec_encrypt(uint64_t n, const uint32_t* pk_aff, const int32_t* pk_status, const uint8_t* r32,
                               const uint8_t* msg, const uint64_t* off, uint8_t* U48, uint8_t* V, uint8_t* W96,
                               uint8_t* seeds, uint8_t* vdig, int32_t* est, int32_t* err, hipStream_t st);
hipError_t launch_tdec_decrypt_share(uint64_t n, uint32_t n_ct, uint32_t n_sk, const uint32_t* u_aff,
                                     const int32_t* u_status, const uint8_t* sk32, const uint32_t* share_ct,
                                     const uint32_t* share_sk, uint8_t* share48, int32_t* status, int32_t* err,
                                     hipStream_t st);
hipError_t launch_coin_combine(uint32_t n, uint32_t t, const uint8_t* share96, const uint32_t* idx, uint8_t* sig96,
                               uint8_t* parity, int32_t* status, hipStream_t st);
hipError_t launch_sig_doc_prepare(uint32_t n, const uint8_t* doc, const uint64_t* off, uint32_t* coefH,
                                  uint8_t* seeds, hipStream_t st);
hipError_t launch_sig_batch_leaves(uint32_t nb_max, const uint32_t* nb_dev, uint32_t n_doc, const BatchDesc* desc,
                                   const uint32_t* perm, const uint8_t* share96, const uint32_t* share_pk,
                                   const uint8_t* seeds, const uint32_t* pk_aff, const int32_t* pk_status,
                                   const uint32_t* pk_tbl, uint32_t* sums, uint8_t* leaf_ok, const BatchKey& key,
                                   hipStream_t st);
hipError_t launch_sig_batch_check(uint32_t cap, const uint32_t* n_dev, uint32_t spec, const CheckItem* items,
                                  const BatchDesc* desc, const uint32_t* perm, const uint32_t* sums,
                                  const uint8_t* leaf_ok, const uint32_t* coefH, uint32_t* lines, uint8_t* ok,
                                  CheckItem* next, uint32_t* next_n, uint32_t* fail_list, uint32_t* fail_n,
                                  hipStream_t st);
hipError_t launch_sig_verify_shares(uint64_t cap, const uint32_t* n_dev, const uint32_t* sel, const uint8_t* share96,
                                    const uint32_t* share_doc, const uint32_t* share_pk, const uint32_t* pk_aff,
                                    const int32_t* pk_status, const uint32_t* coefH, uint32_t* lines, uint8_t* ok,
                                    hipStream_t st);
hipError_t launch_tdec_ct_verify(uint32_t n, const uint32_t* ct_u, const int32_t* ct_status, const uint32_t* coefH,
                                 const uint32_t* coefW, uint8_t* ok, hipStream_t st);
hipError_t launch_tdec_select(uint32_t n_ct, uint32_t N, uint32_t t, const uint8_t* ct_ok, const uint8_t* ok,
                              const uint32_t* arrival, uint32_t arrival_len, const uint8_t* share48,
                              uint32_t* sel_idx, uint8_t* sel48, uint8_t* outcome, int32_t* sel_status,
                              hipStream_t st);
hipError_t launch_tdec_pair_index(uint64_t n, uint32_t N, uint32_t* sct, uint32_t* spk, hipStream_t st);
hipError_t launch_tdec_status_merge(uint32_t n, const int32_t* sel_status, int32_t* status, hipStream_t st);
// seeds: [n][32] scratch (xor_with_hash keys, consumed by tdec_keystream_xor).
// share_aff (nullable): the verified shares' affine points [n][n_nodes][kAffWords]
// written by the share verification (leaves / verify_shares): the combine
// reads share idx[i] of ciphertext g there instead of decompressing share48;
// pre_status (nullable, with share_aff): a ciphertext whose selection failed
// is skipped (its status is the selection's); share_ok (nullable, with
// share_aff): the verification's bits [n][n_nodes] — a selected share whose
// bit is 0 (a validator's own share, inserted unverified) has no share_aff
// entry and is decompressed from share48 (undecodable: HBG_E_INVALID_POINT).
hipError_t launch_tdec_combine(uint32_t n, uint32_t t, const uint8_t* share48, const uint32_t* idx,
                               const uint8_t* V, const uint64_t* V_off, uint8_t* out, int32_t* status,
                               uint32_t* scratch, uint8_t* seeds, hipStream_t st, const uint32_t* share_aff = nullptr,
                               uint32_t n_nodes = 0, const int32_t* pre_status = nullptr,
                               const uint8_t* share_ok = nullptr);
hipError_t launch_tdec_test(int op, uint32_t n, const uint32_t* in, uint32_t* out, uint32_t in_words,
                            uint32_t out_words, uint32_t* lines, hipStream_t st);

}  // namespace bls
}  // namespace hbg
