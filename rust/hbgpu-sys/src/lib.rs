//! Raw FFI to `include/hbgpu.h` (one declaration per prototype; checked
//! against the header by `tests/test_rust_ffi.py`) plus the safe wrappers a
//! patched hbbft calls (`safe`).
//!
//! The reference (VegeBun-csj/hydrabadger) reaches this path only through
//! hbbft: `src/hydrabadger/state.rs:484` (`dhb.propose`) and
//! `src/hydrabadger/state.rs:486-487` (`dhb.handle_message`).
#![allow(non_camel_case_types)]

use std::os::raw::{c_char, c_int, c_void};

pub mod safe;

#[repr(C)]
pub struct hbg_ctx {
    _private: [u8; 0],
}

pub const HBG_OK: c_int = 0;
pub const HBG_E_ARG: c_int = -1;
pub const HBG_E_DEVICE: c_int = -2;
pub const HBG_E_NOMEM: c_int = -3;
pub const HBG_E_TOO_FEW_DATA_SHARDS: c_int = -10;
pub const HBG_E_TOO_FEW_PARITY_SHARDS: c_int = -11;
pub const HBG_E_TOO_MANY_SHARDS: c_int = -12;
pub const HBG_E_TOO_FEW_SHARDS: c_int = -13;
pub const HBG_E_TOO_FEW_SHARDS_PRESENT: c_int = -14;
pub const HBG_E_EMPTY_SHARD: c_int = -15;
pub const HBG_E_INCORRECT_SHARD_SIZE: c_int = -16;
pub const HBG_E_SINGULAR_MATRIX: c_int = -17;
pub const HBG_E_NOT_ENOUGH_SHARES: c_int = -20;
pub const HBG_E_DUPLICATE_ENTRY: c_int = -21;
pub const HBG_E_INVALID_POINT: c_int = -22;
pub const HBG_E_INVALID_CIPHERTEXT: c_int = -23;
pub const HBG_E_WIRE_EOF: c_int = -30;
pub const HBG_E_WIRE_TAG: c_int = -31;
pub const HBG_E_WIRE_FRAME: c_int = -32;
pub const HBG_E_INVALID_SIGNATURE: c_int = -33;
pub const HBG_E_UNKNOWN_PEER: c_int = -34;
pub const HBG_E_WIRE_VALUE: c_int = -35;

pub const HBG_DEVICE: u32 = 1;
pub const HBG_ASYNC: u32 = 2;
pub const HBG_DECODE_OK: u8 = 1;
pub const HBG_DECODE_NONE: u8 = 0;
pub const HBG_SHARE_NONE: u8 = 0;
pub const HBG_SHARE_ACCEPTED: u8 = 1;
pub const HBG_SHARE_FAULTY: u8 = 2;
pub const HBG_SHARE_IGNORED: u8 = 3;
pub const HBG_SHARE_REPEAT: u8 = 4;
pub const HBG_ARRIVAL_CIPHERTEXT: u32 = 0xFFFF_FFFE;
pub const HBG_ARRIVAL_OWN: u32 = 0x8000_0000;
pub const HBG_MSG_VALUE: u32 = 0;
pub const HBG_MSG_ECHO: u32 = 1;
pub const HBG_MSG_READY: u32 = 2;
pub const HBG_MSG_CAN_DECODE: u32 = 3;
pub const HBG_MSG_ECHO_HASH: u32 = 4;
pub const HBG_WIRE_KIND_MESSAGE: u32 = 7;
pub const HBG_WIRE_KIND_KEYGEN: u32 = 9;
pub const HBG_WIRE_KIND_MAX: u32 = 10;
pub const HBG_WIRE_MAX_FRAME: u32 = 8 * 1024 * 1024;
pub const HBG_VERIFY_BATCHED: c_int = 0;
pub const HBG_VERIFY_PER_SHARE: c_int = 1;

extern "C" {
    pub fn hbg_init(out: *mut *mut hbg_ctx, device: c_int) -> c_int;
    pub fn hbg_free(ctx: *mut hbg_ctx);
    pub fn hbg_ctx_device(ctx: *const hbg_ctx) -> c_int;
    pub fn hbg_set_stream(ctx: *mut hbg_ctx, hip_stream: *mut c_void) -> c_int;
    pub fn hbg_reset_stream(ctx: *mut hbg_ctx) -> c_int;
    pub fn hbg_sync(ctx: *mut hbg_ctx) -> c_int;
    pub fn hbg_strerror(code: c_int) -> *const c_char;
    pub fn hbg_version() -> *const c_char;
    pub fn hbg_merkle_nodes(n: u32) -> u32;
    pub fn hbg_merkle_depth(n: u32) -> u32;
    pub fn hbg_num_faulty(n: u32) -> u32;
    pub fn hbg_shard_len(n: u32, payload_len: u64) -> u64;
    pub fn hbg_coding_matrix(data: u32, parity: u32, out: *mut u8) -> c_int;
    pub fn hbg_rs_encode(ctx: *mut hbg_ctx, data: u32, parity: u32, shard_len: u64, shards: *mut u8,
                         shard_stride: u64, n: u64, flags: u32) -> c_int;
    pub fn hbg_rs_reconstruct(ctx: *mut hbg_ctx, data: u32, parity: u32, shard_len: u64, shards: *mut u8,
                              shard_stride: u64, present: *const u8, status: *mut i32, n: u64,
                              flags: u32) -> c_int;
    pub fn hbg_merkle_build(ctx: *mut hbg_ctx, n_nodes: u32, shard_len: u64, shards: *const u8,
                            shard_stride: u64, levels: *mut u8, n: u64, flags: u32) -> c_int;
    pub fn hbg_merkle_validate(ctx: *mut hbg_ctx, n_nodes: u32, value_len: u64, values: *const u8,
                               value_stride: u64, index: *const u32, digests: *const u8,
                               ndigests: *const u32, roots: *const u8, ok: *mut u8, n_proofs: u64,
                               flags: u32) -> c_int;
    pub fn hbg_merkle_validate_views(ctx: *mut hbg_ctx, n_nodes: u32, value_len: u64, values: *const u8,
                                     value_stride: u64, index: *const u32, digests: *const u8,
                                     ndigests: *const u32, roots: *const u8, ok: *mut u8, n_proofs: u64,
                                     n_views: u32, flags: u32) -> c_int;
    pub fn hbg_rbc_encode_merkle(ctx: *mut hbg_ctx, n_nodes: u32, payloads: *const u8, payload_stride: u64,
                                 payload_len: *const u64, shard_len: u64, shards: *mut u8, shard_stride: u64,
                                 levels: *mut u8, n: u64, flags: u32) -> c_int;
    pub fn hbg_rbc_decode(ctx: *mut hbg_ctx, n_nodes: u32, shard_len: u64, shards: *mut u8, shard_stride: u64,
                          present: *const u8, roots: *const u8, payload_out: *mut u8, payload_stride: u64,
                          payload_len: *mut u64, status: *mut u8, n: u64, flags: u32) -> c_int;
    pub fn hbg_set_share_verify(ctx: *mut hbg_ctx, mode: c_int) -> c_int;
    pub fn hbg_tdec_verify_shares(ctx: *mut hbg_ctx, n_ct: u32, u48: *const u8, v: *const u8, v_off: *const u64,
                                  w96: *const u8, n_pk: u32, pk48: *const u8, n_shares: u64, share48: *const u8,
                                  share_ct: *const u32, share_pk: *const u32, ok: *mut u8, flags: u32) -> c_int;
    pub fn hbg_ct_verify(ctx: *mut hbg_ctx, n_ct: u32, u48: *const u8, v: *const u8, v_off: *const u64,
                         w96: *const u8, ok: *mut u8, flags: u32) -> c_int;
    pub fn hbg_tdec_combine(ctx: *mut hbg_ctx, t: u32, n_ct: u32, share48: *const u8, share_index: *const u32,
                            v: *const u8, v_off: *const u64, plaintext: *mut u8, status: *mut i32,
                            flags: u32) -> c_int;
    pub fn hbg_tdec_threshold_decrypt(ctx: *mut hbg_ctx, t: u32, n_nodes: u32, n_ct: u32, u48: *const u8,
                                      v: *const u8, v_off: *const u64, w96: *const u8, pk48: *const u8,
                                      share48: *const u8, arrival: *const u32, arrival_len: u32,
                                      plaintext: *mut u8, status: *mut i32, outcome: *mut u8,
                                      flags: u32) -> c_int;
    pub fn hbg_tdec_encrypt(ctx: *mut hbg_ctx, pk48: *const u8, n: u64, r32: *const u8, msg: *const u8,
                            msg_off: *const u64, u48: *mut u8, v: *mut u8, w96: *mut u8, flags: u32) -> c_int;
    pub fn hbg_tdec_decrypt_shares(ctx: *mut hbg_ctx, n_ct: u32, u48: *const u8, n_sk: u32, sk32: *const u8,
                                   n: u64, share_ct: *const u32, share_sk: *const u32, share48: *mut u8,
                                   status: *mut i32, flags: u32) -> c_int;
    pub fn hbg_bls_sign(ctx: *mut hbg_ctx, n_sk: u32, sk32: *const u8, n: u64, msg_sk: *const u32,
                        msg: *const u8, msg_off: *const u64, sig96: *mut u8, flags: u32) -> c_int;
    pub fn hbg_bls_verify(ctx: *mut hbg_ctx, n_pk: u32, pk48: *const u8, n: u64, msg_pk: *const u32,
                          msg: *const u8, msg_off: *const u64, sig96: *const u8, ok: *mut u8, flags: u32) -> c_int;
    pub fn hbg_sig_combine(ctx: *mut hbg_ctx, t: u32, n: u64, share96: *const u8, share_index: *const u32,
                           sig96: *mut u8, parity: *mut u8, status: *mut i32, flags: u32) -> c_int;
    pub fn hbg_sig_verify_shares(ctx: *mut hbg_ctx, n_doc: u32, doc: *const u8, doc_off: *const u64, n_pk: u32,
                                 pk48: *const u8, n: u64, share96: *const u8, share_doc: *const u32,
                                 share_pk: *const u32, ok: *mut u8, flags: u32) -> c_int;
    pub fn hbg_proof_digests(n: u32, index: u32) -> u32;
    pub fn hbg_proof_msg_len(n: u32, index: u32, value_len: u64) -> u64;
    pub fn hbg_rbc_write_proof_msgs(ctx: *mut hbg_ctx, n_nodes: u32, shard_len: u64, shards: *const u8,
                                    shard_stride: u64, levels: *const u8, n: u64, tag: u32, m: u64,
                                    inst: *const u64, index: *const u32, out: *mut u8, out_off: *const u64,
                                    flags: u32) -> c_int;
    pub fn hbg_rbc_read_msgs(ctx: *mut hbg_ctx, n_nodes: u32, shard_len: u64, msgs: *const u8,
                             msg_off: *const u64, m: u64, tag: *mut u32, values: *mut u8, value_stride: u64,
                             index: *mut u32, digests: *mut u8, ndigests: *mut u32, roots: *mut u8,
                             status: *mut i32, flags: u32) -> c_int;
    pub fn hbg_wire_frame_len(msg_len: u64) -> u64;
    pub fn hbg_wire_sign_frames(ctx: *mut hbg_ctx, n_sk: u32, sk32: *const u8, n: u64, msg_sk: *const u32,
                                msg: *const u8, msg_off: *const u64, frames: *mut u8, frame_off: *const u64,
                                flags: u32) -> c_int;
    pub fn hbg_wire_verify_frames(ctx: *mut hbg_ctx, n_pk: u32, pk48: *const u8, n: u64, frame_pk: *const u32,
                                  frames: *const u8, frame_off: *const u64, status: *mut i32, flags: u32) -> c_int;
    pub fn hbg_synth_bytes(ctx: *mut hbg_ctx, tag: u32, first_instance: u64, nbytes: u64, out: *mut u8,
                           out_stride: u64, n: u64, flags: u32) -> c_int;
}
