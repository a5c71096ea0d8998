"""CPU oracle for the hydrabadger RBC-coding + ThresholdDecrypt hot path.

TEST INFRASTRUCTURE ONLY.  Nothing under ``oracle/`` is part of the product:
only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import, link or execute it, and only as the checker
(or the timed CPU baseline), never as the thing measured or shipped.

The reference (VegeBun-csj/hydrabadger) drives hbbft's ``Broadcast`` and
``ThresholdDecrypt`` from ``src/hydrabadger/state.rs:484-487``; every
arithmetic routine on that path lives in third-party crates that are not in
``/root/reference`` (hbbft git master of VegeBun-csj/hbbft, reed-solomon-erasure,
tiny-keccak, threshold_crypto, pairing, rand_chacha — versions unpinned, no
Cargo.lock, ``.gitignore:14-15``).  This package restates their published
algorithms and is pinned by the known-answer tests listed in
SURVEY.md §8(c) (Backblaze RS vector, FIPS-202 via hashlib, RFC 8439 ChaCha20,
BLS12-381 standard constants).  Rows with no external known answer (Merkle
tree shape, ``hash_g2``) are "parity unpinned" — see DESIGN.md §Oracle.

Modules
  gf256     GF(2^8) tables, Vandermonde·inv(top) coding matrix, encode/reconstruct
  merkle    hbbft MerkleTree / Proof (SHA3-256 via hashlib)
  rbc       hbbft Broadcast glue: send_shards / decode_from_shards / glue_shards
  chacha    ChaCha20 keystream as rand_chacha emits it
  bls12_381 field tower, G1/G2, optimal-ate pairing, zcash compression
  tcrypto   threshold_crypto Ciphertext / shares / interpolate / xor_with_hash
  synth     the seeded synthetic-input generator shared with the GPU harness
"""
