/* hbgpu.h — C ABI of the MI355X (gfx950) batch engine for hbbft's RBC coding,
 * Merkle and ThresholdDecrypt hot path, as driven by hydrabadger.
 *
 * The reference (VegeBun-csj/hydrabadger) reaches this path only through hbbft:
 *   propose         /root/reference/src/hydrabadger/state.rs:484  dhb.propose(contrib, rng)
 *   handle_message  /root/reference/src/hydrabadger/state.rs:486-487 dhb.handle_message(src, msg, rng)
 * and, inside hbbft [EXT, VegeBun-csj/hbbft master, unvendored], through the
 * call surfaces each entry point below replaces.  Every
 * entry point is batch-first: a single hbbft call is n = 1.
 *
 * Conventions
 *  - Return 0 (HBG_OK) or a negative HBG_E_* code.  Per-instance outcomes
 *    (hbbft's `None` / `false`) go to per-item status/ok arrays.
 *  - flags & HBG_DEVICE: every buffer argument (including small metadata
 *    arrays) is a device pointer on the context's device; otherwise all are
 *    host pointers and the engine stages them through device memory.
 *  - flags & HBG_ASYNC (device mode only): return after enqueueing on the
 *    context stream, with no host synchronisation inside the call (only the
 *    one-time growth of an internal scratch buffer waits for the stream);
 *    call hbg_sync().  Without it calls are synchronous.
 *  - Device-side argument errors: in device mode the index / length
 *    arguments live in device memory, so the kernels check them.  An
 *    offending item gets its invalid per-item output (ok = 0, status =
 *    HBG_E_ARG, an all-zero point encoding, a message or frame left
 *    unwritten) and the context records the FIRST such code; the next
 *    synchronous call or hbg_sync() returns it (and clears it).  Host mode
 *    rejects the same arguments up front with the same code.
 *  - Shard batches: instance k's shard i starts at
 *        shards + (k * N + i) * shard_stride
 *    and holds shard_len (L) meaningful bytes.  Host mode accepts any
 *    shard_stride >= L (shard_stride == L is the reference's own contiguous
 *    `send_shards` buffer).  Device mode needs shard_stride % 16 == 0 and a
 *    16-byte-aligned base; bytes [L, shard_stride) of each row are engine
 *    scratch (they may be overwritten; they are never hashed).
 *  - Merkle trees are returned as the flat digest array of hbbft's
 *    `MerkleTree.levels` followed by the root: [nodes][32] per instance with
 *    nodes = hbg_merkle_nodes(N); level l (size n_l, n_0 = N,
 *    n_{l+1} = ceil(n_l/2)) starts at sum_{m<l} n_m; the root is the last
 *    digest.  `MerkleTree::proof(i)` is a pure index walk over this array.
 *  - One call is one set of kernel launches: a batch whose launch grid would
 *    exceed a single dispatch (2^31 workgroups or 2^32 work-items, e.g. ~16 M
 *    tiny-payload instances) returns HBG_E_ARG before anything runs; split it.
 *  - No callbacks; no allocation is returned to the caller.
 */
#ifndef HBGPU_H
#define HBGPU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- error codes (mirror rse::Error / threshold_crypto::Error variants) ---- */
#define HBG_OK 0
#define HBG_E_ARG (-1)                    /* bad argument / alignment / layout        */
#define HBG_E_DEVICE (-2)                 /* HIP runtime failure                      */
#define HBG_E_NOMEM (-3)                  /* device allocation failed                 */
#define HBG_E_TOO_FEW_DATA_SHARDS (-10)   /* rse::Error::TooFewDataShards             */
#define HBG_E_TOO_FEW_PARITY_SHARDS (-11) /* rse::Error::TooFewParityShards           */
#define HBG_E_TOO_MANY_SHARDS (-12)       /* rse::Error::TooManyShards                */
#define HBG_E_TOO_FEW_SHARDS (-13)        /* rse::Error::TooFewShards                 */
#define HBG_E_TOO_FEW_SHARDS_PRESENT (-14)/* rse::Error::TooFewShardsPresent          */
#define HBG_E_EMPTY_SHARD (-15)           /* rse::Error::EmptyShard                   */
#define HBG_E_INCORRECT_SHARD_SIZE (-16)  /* rse::Error::IncorrectShardSize           */
#define HBG_E_SINGULAR_MATRIX (-17)       /* rse::Error::SingularMatrix (internal)    */
#define HBG_E_NOT_ENOUGH_SHARES (-20)     /* threshold_crypto::Error::NotEnoughShares */
#define HBG_E_DUPLICATE_ENTRY (-21)       /* threshold_crypto::Error::DuplicateEntry  */
#define HBG_E_INVALID_POINT (-22)         /* bad compressed G1/G2 encoding            */
#define HBG_E_INVALID_CIPHERTEXT (-23)    /* Ciphertext::verify false: set_ciphertext rejects it */
#define HBG_E_WIRE_EOF (-30)              /* bincode::ErrorKind::Io(UnexpectedEof)    */
#define HBG_E_WIRE_TAG (-31)              /* bincode: unknown enum variant index      */
#define HBG_E_WIRE_FRAME (-32)            /* length-delimited prefix != frame body    */
#define HBG_E_INVALID_SIGNATURE (-33)     /* hydrabadger Error::InvalidSignature      */
#define HBG_E_UNKNOWN_PEER (-34)          /* Error::VerificationMessageReceivedUnknownPeer */
#define HBG_E_WIRE_VALUE (-35)            /* bincode / serde: a field value is invalid (uuid length != 16) */

#define HBG_DEVICE 1u
#define HBG_ASYNC 2u

/* per-instance decode status (hbg_rbc_decode) */
#define HBG_DECODE_OK 1          /* Some(payload)                                  */
#define HBG_DECODE_NONE 0        /* None: too few shards, root mismatch or < 4 B   */

typedef struct hbg_ctx hbg_ctx;

/* ---- context ----
 * One context binds ONE device (device < 0: the current HIP device).
 * Deviation from SURVEY.md §8(b)'s hbg_init(ctx, const int *device_ids, int n):
 * the engine runs one process per GPU (torch.distributed, RCCL over xGMI),
 * and instances are sharded across processes, never across the devices of
 * one context; a multi-device caller opens one context per device. */
/* The first hbg_init of a process also runs a known-answer self-test of the
 * BLS12-381 kernels (Ciphertext::verify and verify_decryption_share on a
 * committed fixture, both kernel builds, per-share and batched schedules,
 * ~tens of ms once); if any bit differs from the known answers, that and
 * every later hbg_init of the process return HBG_E_DEVICE. */
int hbg_init(hbg_ctx **out, int device);
void hbg_free(hbg_ctx *ctx);
int hbg_ctx_device(const hbg_ctx *ctx);  /* the device the context binds (< 0: ctx is NULL) */
/* Enqueue on an external hipStream_t from now on (e.g.
 * torch.cuda.current_stream().cuda_stream); the handle is used verbatim, so
 * NULL selects the HIP null stream.  hbg_reset_stream() returns to the
 * context's own non-blocking stream.  A switch is ordered: work enqueued on
 * the old stream completes before work enqueued on the new one (an event,
 * no host synchronisation).  An external stream must outlive the switch away
 * from it; if it was destroyed first, hbg_reset_stream falls back to a
 * device-wide synchronisation and still returns to the context's stream. */
int hbg_set_stream(hbg_ctx *ctx, void *hip_stream);
int hbg_reset_stream(hbg_ctx *ctx);
int hbg_sync(hbg_ctx *ctx);
const char *hbg_strerror(int code);
const char *hbg_version(void);

/* ---- shape helpers (pure host functions) ---- */
uint32_t hbg_merkle_nodes(uint32_t n);                /* digests in a flat tree    */
uint32_t hbg_merkle_depth(uint32_t n);                /* max digests in a proof    */
uint32_t hbg_num_faulty(uint32_t n);                  /* hbbft NetworkInfo: (N-1)/3 */
uint64_t hbg_shard_len(uint32_t n, uint64_t payload_len); /* ceil((P+4)/(N-2f))     */

/* Coding::new(data, parity) (hbbft broadcast.rs [EXT]) -> rse ReedSolomon::new:
 * validates the shard counts and writes the (data+parity) x data coding matrix
 * M = V * inv(V[0..data]) (row-major) when out != NULL. */
int hbg_coding_matrix(uint32_t data, uint32_t parity, uint8_t *out);

/* Coding::encode(&mut [&mut [u8]]) -> rse encode: parity rows of every
 * instance are (re)computed in place from the data rows. */
int hbg_rs_encode(hbg_ctx *ctx, uint32_t data, uint32_t parity, uint64_t shard_len,
                  uint8_t *shards, uint64_t shard_stride, uint64_t n, uint32_t flags);

/* Coding::reconstruct_shards(&mut [Option<Box<[u8]>>]) -> rse reconstruct:
 * present[k*N+i] != 0 marks shard i of instance k as present; missing rows are
 * rebuilt in place from the FIRST `data` present rows (index order), present
 * rows are left as received.  status[k] = 0 or a (negative) HBG_E_* code,
 * e.g. HBG_E_TOO_FEW_SHARDS_PRESENT. */
int hbg_rs_reconstruct(hbg_ctx *ctx, uint32_t data, uint32_t parity, uint64_t shard_len,
                       uint8_t *shards, uint64_t shard_stride, const uint8_t *present,
                       int32_t *status, uint64_t n, uint32_t flags);

/* MerkleTree::from_vec(shards) (+ root_hash): SHA3-256 leaves, pair hashes,
 * odd-node promotion.  levels: [n][hbg_merkle_nodes(N)][32]. */
int hbg_merkle_build(hbg_ctx *ctx, uint32_t N, uint64_t shard_len, const uint8_t *shards,
                     uint64_t shard_stride, uint8_t *levels, uint64_t n, uint32_t flags);

/* Proof::validate(n) for n_proofs proofs of one tree size N.
 * values: [n_proofs] rows of value_len bytes at value_stride;
 * digests: [n_proofs][hbg_merkle_depth(N)][32], ndigests[k] of them used;
 * roots: [n_proofs][32];  ok[k] = 1 valid / 0 invalid. */
int hbg_merkle_validate(hbg_ctx *ctx, uint32_t N, uint64_t value_len, const uint8_t *values,
                        uint64_t value_stride, const uint32_t *index, const uint8_t *digests,
                        const uint32_t *ndigests, const uint8_t *roots, uint8_t *ok,
                        uint64_t n_proofs, uint32_t flags);

/* The same n_proofs proofs validated by each of n_views nodes on its own
 * (hbbft handle_echo at every node: the N^3 of an epoch):
 * ok[v * n_proofs + k] is view v's Proof::validate of proof k.  Every view
 * hashes the proofs itself; the views read one table (no per-view copies).
 * n_views = 1 is hbg_merkle_validate. */
int hbg_merkle_validate_views(hbg_ctx *ctx, uint32_t N, uint64_t value_len, const uint8_t *values,
                              uint64_t value_stride, const uint32_t *index, const uint8_t *digests,
                              const uint32_t *ndigests, const uint8_t *roots, uint8_t *ok,
                              uint64_t n_proofs, uint32_t n_views, uint32_t flags);

/* Broadcast::send_shards fused (a2+a3+a4): payload k (payload_len[k] bytes at
 * payloads + k*payload_stride) -> BE u32 length prefix, zero pad, chunk into N
 * shards of shard_len, RS-encode, Merkle-tree.  Every payload_len[k] must give
 * hbg_shard_len(N, payload_len[k]) == shard_len and payload_len[k] <=
 * payload_stride (else HBG_E_ARG; in device mode such an instance is skipped
 * and the error is device-side).  Device mode additionally needs
 * payload_stride % 4 == 0. */
int hbg_rbc_encode_merkle(hbg_ctx *ctx, uint32_t N, const uint8_t *payloads,
                          uint64_t payload_stride, const uint64_t *payload_len,
                          uint64_t shard_len, uint8_t *shards, uint64_t shard_stride,
                          uint8_t *levels, uint64_t n, uint32_t flags);

/* decode_from_shards + glue_shards (a7+a8): reconstruct in place, rebuild the
 * tree over all N shards, compare with roots[k]; on match glue the first
 * data shards: payload_out + k*payload_stride gets payload_len[k] bytes and
 * status[k] = HBG_DECODE_OK, else status[k] = HBG_DECODE_NONE.
 * payload_stride >= D * shard_len (D = N - 2f data shards).  Bytes of an
 * OK row past payload_len[k] are unspecified (the fused N = 64 decoder writes
 * the glued bytes while it rebuilds, before the root comparison); the first
 * D * shard_len bytes of a NONE instance's row are zeroed (both schedules), so
 * no unauthenticated byte is ever left in payload_out. */
int hbg_rbc_decode(hbg_ctx *ctx, uint32_t N, uint64_t shard_len, uint8_t *shards,
                   uint64_t shard_stride, const uint8_t *present, const uint8_t *roots,
                   uint8_t *payload_out, uint64_t payload_stride, uint64_t *payload_len,
                   uint8_t *status, uint64_t n, uint32_t flags);

/* ---- ThresholdDecrypt (family 3): threshold_crypto surfaces ----------------
 * Points cross the boundary in the zcash compressed encoding the crate
 * serialises (G1 48 B, G2 96 B).  A ciphertext table of n_ct entries is
 * U48 [n_ct][48], W96 [n_ct][96] and the V byte strings concatenated in V with
 * V_off[n_ct + 1] offsets (entry k = V[V_off[k] .. V_off[k+1])).
 */

/* Share-verification schedule of hbg_tdec_verify_shares,
 * hbg_tdec_threshold_decrypt and hbg_sig_verify_shares (per context):
 *  - HBG_VERIFY_PER_SHARE: one independent pairing equation per share, the
 *    crate's own check — every bit is deterministic and identical to the
 *    crate's bool.
 *  - HBG_VERIFY_BATCHED (the default): from 393,216 shares per call up, the
 *    shares of one ciphertext (document) are checked in weighted batches of
 *    <= 64 by a small-exponent test with binary splitting down to single
 *    shares; smaller calls run per share.  Every 0 bit is the crate's per-share
 *    verdict.  A 1 bit comes from a passing (sub)batch and equals the crate's
 *    bool except with probability <= 2^-127 per (sub)batch check that holds an
 *    invalid share: the weights take 2^127 distinct values (decryption shares:
 *    a + b|x| + c x^2 + d|x|^3, a..d 32-bit; coin shares: a + b x^2, a and b
 *    64-bit; a odd) and are derived from a secret 32-byte key drawn from
 *    getrandom(2) at hbg_init
 *    and never exposed, so a sender can neither predict nor grind them.
 * Returns HBG_E_ARG for any other mode. */
#define HBG_VERIFY_BATCHED 0
#define HBG_VERIFY_PER_SHARE 1
int hbg_set_share_verify(hbg_ctx *ctx, int mode);

/* PublicKeyShare::verify_decryption_share for n_shares shares:
 * share k (share48[k]) claims to decrypt ciphertext share_ct[k] under public
 * key share pk48[share_pk[k]] (PublicKeySet::public_key_share(i) values).
 * ok[k] = 1 iff every point decodes (in its subgroup), the ciphertext decodes,
 * and e(share, hash_g1_g2(U, V)) == e(pk, W), for points the crate would
 * deserialise: identical to the crate's bool under HBG_VERIFY_PER_SHARE, and
 * under the default HBG_VERIFY_BATCHED up to the 2^-127 bound stated at
 * hbg_set_share_verify (a 0 is always the crate's verdict).  share_ct[k] >=
 * n_ct or share_pk[k] >= n_pk: HBG_E_ARG (device mode: ok[k] = 0,
 * device-side). */
int hbg_tdec_verify_shares(hbg_ctx *ctx, uint32_t n_ct, const uint8_t *U48, const uint8_t *V,
                           const uint64_t *V_off, const uint8_t *W96, uint32_t n_pk,
                           const uint8_t *pk48, uint64_t n_shares, const uint8_t *share48,
                           const uint32_t *share_ct, const uint32_t *share_pk, uint8_t *ok,
                           uint32_t flags);

/* Ciphertext::verify for n_ct ciphertexts: ok[k] = e(G1, W) == e(U, hash_g1_g2(U, V)). */
int hbg_ct_verify(hbg_ctx *ctx, uint32_t n_ct, const uint8_t *U48, const uint8_t *V,
                  const uint64_t *V_off, const uint8_t *W96, uint8_t *ok, uint32_t flags);

/* PublicKeySet::decrypt for n_ct ciphertexts with threshold t: shares48
 * [n_ct][t+1][48] and share_index [n_ct][t+1] are the FIRST t+1 (node index,
 * share) items in the caller's iterator order (hbbft: BTreeMap by node id);
 * x = index + 1.  plaintext gets xor_with_hash(interpolate(...), V) at the V
 * layout (same V_off).  status[k] = 0, HBG_E_DUPLICATE_ENTRY or
 * HBG_E_INVALID_POINT.  Fewer than t+1 shares is the caller's
 * NotEnoughShares (not representable in this layout). */
int hbg_tdec_combine(hbg_ctx *ctx, uint32_t t, uint32_t n_ct, const uint8_t *share48,
                     const uint32_t *share_index, const uint8_t *V, const uint64_t *V_off,
                     uint8_t *plaintext, int32_t *status, uint32_t flags);

/* ---- hbbft ThresholdDecrypt, batched over an epoch ----
 * One node's ThresholdDecrypt instances for n_ct ciphertexts (one per
 * accepted proposal of the epoch), N = n_nodes senders each.  Per ciphertext
 * k (hbbft threshold_decrypt.rs [EXT, recalled from upstream], reached from
 * src/hydrabadger/state.rs:486-487) the arrival list arrival[k][0 ..
 * arrival_len) is replayed; it ends at the first entry >= n_nodes other than
 * a ciphertext marker — HBG_ARRIVAL_CIPHERTEXT (an observer) or
 * HBG_ARRIVAL_OWN | i (validator node i, i < n_nodes) — (arrival == NULL: every
 * sender once, in node order, after the ciphertext):
 *  - entries before HBG_ARRIVAL_CIPHERTEXT arrived before HoneyBadger output
 *    the ciphertext: handle_message holds the share unverified; a sender
 *    already held is faulted (FaultKind::MultipleDecryptionShares ->
 *    HBG_SHARE_REPEAT flag);
 *  - at the marker (no marker: before the first entry): set_ciphertext runs
 *    Ciphertext::verify — false -> status[k] = HBG_E_INVALID_CIPHERTEXT and
 *    nothing else happens for k; then start_decryption drops the held shares
 *    that fail PublicKeyShare::verify_decryption_share
 *    (FaultKind::UnverifiedDecryptionShareSender -> HBG_SHARE_FAULTY; the
 *    rest HBG_SHARE_ACCEPTED), a validator (HBG_ARRIVAL_OWN | i) inserts its
 *    own share share48[k][i] (decrypt_share_no_verify: trusted, never
 *    verified; HBG_SHARE_ACCEPTED) and try_output runs;
 *  - later entries, until the instance terminates: an invalid share is a
 *    fault (HBG_SHARE_FAULTY), a valid one is held (HBG_SHARE_ACCEPTED), a
 *    valid one from a sender already held is a repeat fault
 *    (HBG_SHARE_REPEAT flag);
 *  - try_output: once t+1 shares are held the instance terminates and
 *    PublicKeySet::decrypt interpolates the first t+1 held (node-id order)
 *    into plaintext (the V layout); later arrivals are ignored
 *    (HBG_SHARE_IGNORED, never checked by hbbft); with fewer than t+1 valid
 *    shares status HBG_E_NOT_ENOUGH_SHARES (no output).
 * share48 [n_ct][n_nodes][48] holds sender i's share of ciphertext k at
 * [k][i] (a repeated message carries the same share; slots of senders that
 * never arrive are not read for the output); pk48 [n_nodes][48] the public
 * key shares; outcome [n_ct][n_nodes] (one HBG_SHARE_* code, optionally |
 * HBG_SHARE_REPEAT).  Every share is verified on the device (batched, as
 * hbg_tdec_verify_shares, under the context's hbg_set_share_verify schedule);
 * a validator's own share is never verified: it is decompressed for the
 * combination, and one that does not decode gives HBG_E_INVALID_POINT.
 * Plaintext bytes of a ciphertext with status != 0 are unspecified. */
#define HBG_SHARE_NONE 0u     /* no message from this sender (or not processed)        */
#define HBG_SHARE_ACCEPTED 1u /* valid, held before termination                         */
#define HBG_SHARE_FAULTY 2u   /* invalid before termination: UnverifiedDecryptionShareSender */
#define HBG_SHARE_IGNORED 3u  /* arrived after termination                              */
#define HBG_SHARE_REPEAT 4u   /* flag: MultipleDecryptionShares logged for the sender   */
#define HBG_ARRIVAL_CIPHERTEXT 0xFFFFFFFEu /* arrival entry: set_ciphertext + start_decryption */
#define HBG_ARRIVAL_OWN 0x80000000u        /* HBG_ARRIVAL_OWN | i: the same at validator node i,
                                              whose own share is inserted before try_output */
int hbg_tdec_threshold_decrypt(hbg_ctx *ctx, uint32_t t, uint32_t n_nodes, uint32_t n_ct,
                               const uint8_t *U48, const uint8_t *V, const uint64_t *V_off,
                               const uint8_t *W96, const uint8_t *pk48, const uint8_t *share48,
                               const uint32_t *arrival, uint32_t arrival_len, uint8_t *plaintext,
                               int32_t *status, uint8_t *outcome, uint32_t flags);

/* ---- the proposer / node side of ThresholdDecrypt ------
 * Scalars cross the boundary as 32-byte little-endian integers (an Fr value:
 * the crate's FrRepr limbs in order); [k]P == [k mod r]P for the prime-order
 * points involved, so no range check is needed. */

/* PublicKey::encrypt_with_rng (threshold_crypto) with the randomness explicit:
 * for message k (msg[msg_off[k] .. msg_off[k+1]]) and scalar r32[k]:
 * U48[k] = r G1, V (at the message's offsets) = xor_with_hash(r PK, msg),
 * W96[k] = r hash_g1_g2(U, V).  HBG_E_INVALID_POINT if pk48 does not decode
 * (device-side: U48 / W96 are then all-zero).
 * Replaces the reference call inside hbbft HoneyBadger::propose
 * (reached from src/hydrabadger/state.rs:484). */
int hbg_tdec_encrypt(hbg_ctx *ctx, const uint8_t *pk48, uint64_t n, const uint8_t *r32,
                     const uint8_t *msg, const uint64_t *msg_off, uint8_t *U48, uint8_t *V,
                     uint8_t *W96, uint32_t flags);

/* SecretKeyShare::decrypt_share_no_verify for n (ciphertext, key) pairs:
 * share48[k] = U48[share_ct[k]] * sk32[share_sk[k]].  status[k] = 0, or
 * HBG_E_INVALID_POINT when that U does not decode (share48[k] is then the
 * identity encoding), or HBG_E_ARG for an out-of-range index (device mode).
 * Reached from hbbft ThresholdDecrypt::start_decryption
 * (src/hydrabadger/state.rs:487). */
int hbg_tdec_decrypt_shares(hbg_ctx *ctx, uint32_t n_ct, const uint8_t *U48, uint32_t n_sk,
                            const uint8_t *sk32, uint64_t n, const uint32_t *share_ct,
                            const uint32_t *share_sk, uint8_t *share48, int32_t *status,
                            uint32_t flags);

/* ---- wire-message signatures --------------------------
 * SecretKey::sign(msg) for n messages: sig96[k] = hash_g2(msg_k) * sk32[msg_sk[k]]
 * (replaces src/lib.rs:434, WireMessages::start_send).  msg_sk[k] >= n_sk:
 * HBG_E_ARG (device mode: sig96[k] all-zero, device-side). */
int hbg_bls_sign(hbg_ctx *ctx, uint32_t n_sk, const uint8_t *sk32, uint64_t n,
                 const uint32_t *msg_sk, const uint8_t *msg, const uint64_t *msg_off,
                 uint8_t *sig96, uint32_t flags);

/* PublicKey::verify(sig, msg) for n messages: ok[k] = 1 iff pk48[msg_pk[k]]
 * and sig96[k] decode (the crate's subgroup checks) and
 * e(pk, hash_g2(msg_k)) == e(G1, sig) (replaces src/lib.rs:405-416,
 * WireMessages::poll).  msg_pk[k] >= n_pk: HBG_E_ARG (device mode: ok[k] = 0,
 * device-side). */
int hbg_bls_verify(hbg_ctx *ctx, uint32_t n_pk, const uint8_t *pk48, uint64_t n,
                   const uint32_t *msg_pk, const uint8_t *msg, const uint64_t *msg_off,
                   const uint8_t *sig96, uint8_t *ok, uint32_t flags);

/* ---- threshold_sign common coin -----------------------
 * Signature shares are SecretKeyShare::sign(doc) = hbg_bls_sign with the key
 * shares; PublicKeyShare::verify(share, doc) = hbg_bls_verify with the public
 * key shares.  This combines them: for coin k, the FIRST t+1 (node index,
 * share) items in iterator order (share96 [n][t+1][96], share_index
 * [n][t+1]; x = index + 1) -> sig96[k] = PublicKeySet::combine_signatures,
 * parity[k] = Signature::parity() (the coin value).  status[k] = 0,
 * HBG_E_DUPLICATE_ENTRY or HBG_E_INVALID_POINT.  t + 1 <= 64 (HBG_E_ARG
 * otherwise: one wave per coin, lane = share).  Replaces hbbft ThresholdSign::try_output (reached from
 * src/hydrabadger/state.rs:487 via BinaryAgreement's coin). */
int hbg_sig_combine(hbg_ctx *ctx, uint32_t t, uint64_t n, const uint8_t *share96,
                    const uint32_t *share_index, uint8_t *sig96, uint8_t *parity,
                    int32_t *status, uint32_t flags);

/* PublicKeyShare::verify(share, doc) for n signature shares grouped by
 * document (the coin nonce every node signs): share k (share96[k]) claims to
 * sign doc share_doc[k] (doc[doc_off[d] .. doc_off[d+1]]) under public key
 * share pk48[share_pk[k]].  ok[k] = 1 iff the key and the share decode
 * (subgroup checks) and e(pk, hash_g2(doc)) == e(G1, share): identical to
 * hbg_bls_verify on the same (pk, doc, share) under HBG_VERIFY_PER_SHARE, and
 * under the default HBG_VERIFY_BATCHED up to the 2^-127 bound stated at
 * hbg_set_share_verify.  hash_g2 runs once per document; from 393,216 shares
 * up the shares of one document are checked in weighted batches (a failing
 * batch is split down to the per-share equation).  Out-of-range indices as in
 * hbg_tdec_verify_shares.  Replaces
 * hbbft ThresholdSign::handle_message's PublicKeyShare::verify (reached from
 * src/hydrabadger/state.rs:487). */
int hbg_sig_verify_shares(hbg_ctx *ctx, uint32_t n_doc, const uint8_t *doc, const uint64_t *doc_off,
                          uint32_t n_pk, const uint8_t *pk48, uint64_t n, const uint8_t *share96,
                          const uint32_t *share_doc, const uint32_t *share_pk, uint8_t *ok, uint32_t flags);

/* ---- hbbft broadcast wire format -----------------------
 * bincode 1.x (default config: little-endian fixed-width integers, u64
 * sequence lengths, u32 enum variant index, trailing bytes ignored) of hbbft
 * broadcast::Message [EXT, src/broadcast/message.rs] — Value(Proof) = 0,
 * Echo(Proof) = 1, Ready(Digest) = 2, CanDecode(Digest) = 3,
 * EchoHash(Digest) = 4 — with Proof<Vec<u8>> {value, index: usize,
 * digests: Vec<Digest>, root_hash} [EXT, src/broadcast/merkle.rs] and
 * Digest = [u8; 32] (a tuple: no length).  A Value/Echo message for leaf i of
 * an N-leaf tree is
 *     u32 tag | u64 L | value[L] | u64 i | u64 k | k x [32] digests | [32] root
 * with k = hbg_proof_digests(N, i).  The reference serialises / parses these
 * one frame at a time in WireMessages::start_send / poll (src/lib.rs:432-446,
 * src/lib.rs:397-404). */
#define HBG_MSG_VALUE 0u
#define HBG_MSG_ECHO 1u
#define HBG_MSG_READY 2u
#define HBG_MSG_CAN_DECODE 3u
#define HBG_MSG_ECHO_HASH 4u

uint32_t hbg_proof_digests(uint32_t N, uint32_t index);           /* k of proof(index); 0 if index >= N */
uint64_t hbg_proof_msg_len(uint32_t N, uint32_t index, uint64_t value_len); /* bytes of Value/Echo(proof) */

/* Message::{Value,Echo}(MerkleTree::proof(index[j])) of tree inst[j] for
 * j < m, from a shard batch of n instances (the hbg_rbc_encode_merkle /
 * hbg_merkle_build layout: shards, shard_stride, levels).  Message j is
 * written to out[out_off[j] .. out_off[j+1]), which must be exactly
 * hbg_proof_msg_len(N, index[j], shard_len) bytes, with index[j] < N and
 * inst[j] < n (HBG_E_ARG otherwise; device mode leaves such a message
 * unwritten and the error is device-side).  tag is
 * HBG_MSG_VALUE or HBG_MSG_ECHO.  Device mode needs shard_stride % 16 == 0 and
 * 16-byte-aligned shards and out. */
int hbg_rbc_write_proof_msgs(hbg_ctx *ctx, uint32_t N, uint64_t shard_len, const uint8_t *shards,
                             uint64_t shard_stride, const uint8_t *levels, uint64_t n, uint32_t tag,
                             uint64_t m, const uint64_t *inst, const uint32_t *index, uint8_t *out,
                             const uint64_t *out_off, uint32_t flags);

/* bincode::deserialize::<Message>(msgs[msg_off[j] .. msg_off[j+1])) for j < m
 * into the hbg_merkle_validate layout: tag[j]; for Value/Echo the value row
 * (values + j*value_stride, shard_len bytes), index[j] (usize clamped to
 * 0xFFFFFFFF), digests [m][hbg_merkle_depth(N)][32], ndigests[j] (0xFFFFFFFF
 * when the proof carries more digests than any N-leaf proof: validate is then
 * false, as in hbbft) and roots[j]; for Ready/CanDecode/EchoHash the digest in
 * roots[j].  status[j] = 0, HBG_E_WIRE_EOF (truncated), HBG_E_WIRE_TAG
 * (variant > 4) or HBG_E_INCORRECT_SHARD_SIZE (a well-formed proof whose value
 * is not shard_len bytes: header fields are filled).  A value row is
 * unspecified unless status[j] == 0 and tag[j] <= HBG_MSG_ECHO.
 * Device mode needs value_stride % 16 == 0 and 16-byte-aligned values. */
int hbg_rbc_read_msgs(hbg_ctx *ctx, uint32_t N, uint64_t shard_len, const uint8_t *msgs,
                      const uint64_t *msg_off, uint64_t m, uint32_t *tag, uint8_t *values,
                      uint64_t value_stride, uint32_t *index, uint8_t *digests, uint32_t *ndigests,
                      uint8_t *roots, int32_t *status, uint32_t flags);

/* ---- §8(f4) + §8(f2): hydrabadger's signed, length-delimited frames -------
 * WireMessages (src/lib.rs:358-447) sends every serialised WireMessage as
 *     u32 BE body_len | bincode SignedWireMessage { message: Vec<u8>, sig }
 *   = u32 BE (8 + len + 96) | u64 LE len | message[len] | sig[96]
 * (tokio LengthDelimitedCodec default: 4-byte big-endian length; Signature =
 * 96-byte compressed G2 tuple) and, on receipt, verifies the signature only
 * for WireMessageKind::Message and ::KeyGen (bincode variants 7 and 9 of the
 * 11 at src/lib.rs:250-270: the message's first 4 bytes, u32 LE). */
#define HBG_WIRE_KIND_MESSAGE 7u
#define HBG_WIRE_KIND_KEYGEN 9u
#define HBG_WIRE_KIND_MAX 10u
/* LengthDelimitedCodec::new()'s default max_frame_length (tokio-io 0.1,
 * src/lib.rs:369): a frame body (= 8 + len + 96) above it is an error on both
 * sides — HBG_E_WIRE_FRAME from hbg_wire_verify_frames, and
 * hbg_wire_sign_frames refuses it (HBG_E_WIRE_FRAME). */
#define HBG_WIRE_MAX_FRAME (8u * 1024u * 1024u)

uint64_t hbg_wire_frame_len(uint64_t msg_len); /* 4 + 8 + msg_len + 96 */

/* WireMessages::start_send for n serialised WireMessages: message k
 * (msg[msg_off[k] .. msg_off[k+1]]) signed with sk32[msg_sk[k]]
 * (SecretKey::sign, src/lib.rs:434) and framed into
 * frames[frame_off[k] .. frame_off[k+1]] (exactly hbg_wire_frame_len bytes:
 * HBG_E_ARG otherwise; a body over HBG_WIRE_MAX_FRAME: HBG_E_WIRE_FRAME, as
 * FramedWrite refuses it; device mode leaves such a frame unwritten and the
 * error is device-side). */
int hbg_wire_sign_frames(hbg_ctx *ctx, uint32_t n_sk, const uint8_t *sk32, uint64_t n,
                         const uint32_t *msg_sk, const uint8_t *msg, const uint64_t *msg_off,
                         uint8_t *frames, const uint64_t *frame_off, uint32_t flags);

/* WireMessages::poll for n received frames (frames[frame_off[k] ..
 * frame_off[k+1]], each one codec frame incl. its 4-byte prefix) from peers
 * whose public keys are pk48[frame_pk[k]] (frame_pk[k] >= n_pk: peer key
 * unknown).  status[k] = 0 (the frame yields its WireMessage: verified, or a
 * kind the reference does not verify), HBG_E_WIRE_FRAME, HBG_E_WIRE_EOF,
 * HBG_E_INVALID_POINT (sig does not deserialise), HBG_E_WIRE_TAG (kind > 10,
 * or an InstanceId / key_gen::MessageKind index > 1), HBG_E_WIRE_VALUE (a
 * uuid of length != 16), HBG_E_UNKNOWN_PEER or HBG_E_INVALID_SIGNATURE.  The
 * message of frame k is frames[frame_off[k] + 12 ..][..len].  As poll
 * (src/lib.rs:400-416) the WireMessage is deserialised BEFORE the signature
 * check: for the two verified kinds the body fields the reference tree
 * defines are checked — Message(Uid, ..): the Uid (serde bytes: u64 length,
 * which must be 16, then the 16 bytes, src/lib.rs:149) and the variant index
 * of the hbbft message that follows; KeyGen(InstanceId, key_gen::Message):
 * InstanceId {BuiltIn, User(Uid)} and key_gen::MessageKind {Part, Ack}
 * (src/hydrabadger/key_gen.rs:18-33) with its Part / Ack index.  The bodies
 * inside the unvendored hbbft types (the DHB message, Part, Ack) and the
 * unverified kinds' bodies (control plane) are the caller's to deserialise. */
int hbg_wire_verify_frames(hbg_ctx *ctx, uint32_t n_pk, const uint8_t *pk48, uint64_t n,
                           const uint32_t *frame_pk, const uint8_t *frames, const uint64_t *frame_off,
                           int32_t *status, uint32_t flags);

/* Device-side seeded generator: row k of out gets nbytes of
 * SplitMix64 stream (tag, first_instance + k); bench inputs never cross PCIe. */
int hbg_synth_bytes(hbg_ctx *ctx, uint32_t tag, uint64_t first_instance, uint64_t nbytes,
                    uint8_t *out, uint64_t out_stride, uint64_t n, uint32_t flags);

#ifdef __cplusplus
}
#endif
#endif /* HBGPU_H */
