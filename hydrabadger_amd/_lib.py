"""ctypes binding of libhbgpu.so (include/hbgpu.h).

The product path has NO CPU fallback: if the HIP library is missing or no
device is present, every compute call raises.  Pure shape helpers
(``merkle_nodes``, ``coding_matrix`` …) are host functions of the same
library and work without a GPU.
"""
from __future__ import annotations

import ctypes as C
import os
import sys

import numpy as np

_PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("HBG_LIB_PATH") or os.path.join(_PKG, "libhbgpu.so")  # override: A/B experiments only

HBG_OK = 0
HBG_E_ARG = -1
HBG_E_DEVICE = -2
HBG_E_NOMEM = -3
HBG_E_TOO_FEW_DATA_SHARDS = -10
HBG_E_TOO_FEW_PARITY_SHARDS = -11
HBG_E_TOO_MANY_SHARDS = -12
HBG_E_TOO_FEW_SHARDS = -13
HBG_E_TOO_FEW_SHARDS_PRESENT = -14
HBG_E_EMPTY_SHARD = -15
HBG_E_INCORRECT_SHARD_SIZE = -16
HBG_E_SINGULAR_MATRIX = -17
HBG_E_NOT_ENOUGH_SHARES = -20
HBG_E_DUPLICATE_ENTRY = -21
HBG_E_INVALID_POINT = -22
HBG_E_INVALID_CIPHERTEXT = -23
HBG_E_WIRE_EOF = -30
HBG_E_WIRE_TAG = -31
HBG_E_WIRE_FRAME = -32
HBG_E_INVALID_SIGNATURE = -33
HBG_E_UNKNOWN_PEER = -34
HBG_E_WIRE_VALUE = -35
HBG_WIRE_KIND_MESSAGE, HBG_WIRE_KIND_KEYGEN, HBG_WIRE_KIND_MAX = 7, 9, 10

HBG_SHARE_NONE, HBG_SHARE_ACCEPTED, HBG_SHARE_FAULTY, HBG_SHARE_IGNORED, HBG_SHARE_REPEAT = 0, 1, 2, 3, 4
HBG_ARRIVAL_CIPHERTEXT = 0xFFFFFFFE
HBG_ARRIVAL_OWN = 0x80000000

HBG_MSG_VALUE, HBG_MSG_ECHO, HBG_MSG_READY, HBG_MSG_CAN_DECODE, HBG_MSG_ECHO_HASH = 0, 1, 2, 3, 4

HBG_DEVICE = 1
HBG_ASYNC = 2

HBG_DECODE_OK = 1
HBG_DECODE_NONE = 0

# hbg_set_share_verify: the batched small-exponent test (default; a 1 bit is
# the crate's except with probability <= 2^-127) or the crate's per-share
# equation for every share (deterministic)
HBG_VERIFY_BATCHED = 0
HBG_VERIFY_PER_SHARE = 1

# (name, restype, argtypes) for every symbol include/hbgpu.h declares.
_vp, _u8p, _u32, _u64, _i = C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint64, C.c_int
SIGNATURES = {
    "hbg_init": (_i, [C.POINTER(C.c_void_p), _i]),
    "hbg_free": (None, [_vp]),
    "hbg_ctx_device": (_i, [_vp]),
    "hbg_set_stream": (_i, [_vp, _vp]),
    "hbg_reset_stream": (_i, [_vp]),
    "hbg_sync": (_i, [_vp]),
    "hbg_strerror": (C.c_char_p, [_i]),
    "hbg_version": (C.c_char_p, []),
    "hbg_merkle_nodes": (_u32, [_u32]),
    "hbg_merkle_depth": (_u32, [_u32]),
    "hbg_num_faulty": (_u32, [_u32]),
    "hbg_shard_len": (_u64, [_u32, _u64]),
    "hbg_coding_matrix": (_i, [_u32, _u32, _u8p]),
    "hbg_rs_encode": (_i, [_vp, _u32, _u32, _u64, _u8p, _u64, _u64, _u32]),
    "hbg_rs_reconstruct": (_i, [_vp, _u32, _u32, _u64, _u8p, _u64, _u8p, _vp, _u64, _u32]),
    "hbg_merkle_build": (_i, [_vp, _u32, _u64, _u8p, _u64, _u8p, _u64, _u32]),
    "hbg_merkle_validate": (_i, [_vp, _u32, _u64, _u8p, _u64, _vp, _u8p, _vp, _u8p, _u8p, _u64, _u32]),
    "hbg_merkle_validate_views": (_i, [_vp, _u32, _u64, _u8p, _u64, _vp, _u8p, _vp, _u8p, _u8p, _u64, _u32, _u32]),
    "hbg_rbc_encode_merkle": (_i, [_vp, _u32, _u8p, _u64, _vp, _u64, _u8p, _u64, _u8p, _u64, _u32]),
    "hbg_rbc_decode": (_i, [_vp, _u32, _u64, _u8p, _u64, _u8p, _u8p, _u8p, _u64, _vp, _u8p, _u64, _u32]),
    "hbg_proof_digests": (_u32, [_u32, _u32]),
    "hbg_proof_msg_len": (_u64, [_u32, _u32, _u64]),
    "hbg_rbc_write_proof_msgs": (_i, [_vp, _u32, _u64, _u8p, _u64, _u8p, _u64, _u32, _u64, _vp, _vp, _u8p, _vp,
                                      _u32]),
    "hbg_rbc_read_msgs": (_i, [_vp, _u32, _u64, _u8p, _vp, _u64, _vp, _u8p, _u64, _vp, _u8p, _vp, _u8p, _vp, _u32]),
    "hbg_wire_frame_len": (_u64, [_u64]),
    "hbg_wire_sign_frames": (_i, [_vp, _u32, _u8p, _u64, _vp, _u8p, _vp, _u8p, _vp, _u32]),
    "hbg_wire_verify_frames": (_i, [_vp, _u32, _u8p, _u64, _vp, _u8p, _vp, _vp, _u32]),
    "hbg_synth_bytes": (_i, [_vp, _u32, _u64, _u64, _u8p, _u64, _u64, _u32]),
    "hbg_set_share_verify": (_i, [_vp, C.c_int]),
    "hbg_tdec_verify_shares": (_i, [_vp, _u32, _u8p, _u8p, _vp, _u8p, _u32, _u8p, _u64, _u8p, _vp, _vp, _u8p, _u32]),
    "hbg_ct_verify": (_i, [_vp, _u32, _u8p, _u8p, _vp, _u8p, _u8p, _u32]),
    "hbg_tdec_combine": (_i, [_vp, _u32, _u32, _u8p, _vp, _u8p, _vp, _u8p, _vp, _u32]),
    "hbg_tdec_threshold_decrypt": (_i, [_vp, _u32, _u32, _u32, _u8p, _u8p, _vp, _u8p, _u8p, _u8p, _vp, _u32, _u8p,
                                        _vp, _u8p, _u32]),
    "hbg_tdec_encrypt": (_i, [_vp, _u8p, _u64, _u8p, _u8p, _vp, _u8p, _u8p, _u8p, _u32]),
    "hbg_tdec_decrypt_shares": (_i, [_vp, _u32, _u8p, _u32, _u8p, _u64, _vp, _vp, _u8p, _vp, _u32]),
    "hbg_bls_sign": (_i, [_vp, _u32, _u8p, _u64, _vp, _u8p, _vp, _u8p, _u32]),
    "hbg_bls_verify": (_i, [_vp, _u32, _u8p, _u64, _vp, _u8p, _vp, _u8p, _u8p, _u32]),
    "hbg_sig_combine": (_i, [_vp, _u32, _u64, _u8p, _vp, _u8p, _u8p, _vp, _u32]),
    "hbg_sig_verify_shares": (_i, [_vp, _u32, _u8p, _vp, _u32, _u8p, _u64, _u8p, _vp, _vp, _u8p, _u32]),
    "hbg_test_bls": (_i, [_vp, C.c_int, _u32, _vp, _u32, _vp, _u32]),
    "hbg_test_set_tdec_batched": (_i, [_vp, C.c_int]),
    "hbg_test_set_rbc_fused": (_i, [_vp, C.c_int]),
    "hbg_test_set_rs_split": (_i, [_vp, C.c_int]),
    "hbg_test_set_rbc_decode_fused": (_i, [_vp, C.c_int]),
    "hbg_test_set_merkle_pairs": (_i, [_vp, C.c_int]),
    "hbg_test_set_clock_probe": (_i, [_vp, _vp, C.c_uint64]),
    "hbg_test_set_latency_lanes": (C.c_uint64, [C.c_uint64]),
}

_lib = None


class HbgError(RuntimeError):
    def __init__(self, code: int, what: str = ""):
        self.code = code
        name = lib().hbg_strerror(code).decode() if _lib is not None else str(code)
        super().__init__(f"{what}: {name} ({code})" if what else f"{name} ({code})")


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} not built: run `python -m hydrabadger_amd.build` (hipcc, gfx950). "
                "There is no CPU fallback.")
        l = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(l, name)
            f.restype = res
            f.argtypes = args
        _lib = l
    return _lib


def check(rc: int, what: str = "") -> None:
    if rc != HBG_OK:
        raise HbgError(rc, what)


def ptr(a) -> int:
    """Address of a contiguous numpy array or a torch tensor (host or device)."""
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        assert a.flags.c_contiguous, "array must be C-contiguous"
        return a.ctypes.data
    return a.data_ptr()  # torch.Tensor


class Context:
    """Owns an ``hbg_ctx`` (device, stream, scratch pools)."""

    def __init__(self, device: int = -1):
        h = C.c_void_p()
        check(lib().hbg_init(C.byref(h), device), "hbg_init")
        self.h = h
        self.device = lib().hbg_ctx_device(h)   # the device it binds (device -1: the current one)

    def close(self) -> None:
        if self.h:
            lib().hbg_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_stream(self, stream_handle: int | None) -> None:
        """Use a hipStream_t verbatim (0 / None = the HIP null stream)."""
        check(lib().hbg_set_stream(self.h, stream_handle or None), "hbg_set_stream")

    def reset_stream(self) -> None:
        check(lib().hbg_reset_stream(self.h), "hbg_reset_stream")

    def sync(self) -> None:
        check(lib().hbg_sync(self.h), "hbg_sync")

    def set_share_verify(self, mode: int) -> None:
        """HBG_VERIFY_BATCHED (default) or HBG_VERIFY_PER_SHARE (every
        share-validity bit from the crate's own per-share equation)."""
        check(lib().hbg_set_share_verify(self.h, mode), "hbg_set_share_verify")


_default: Context | None = None
_default_stream: int | None = None


def default_context() -> Context:
    """The process-wide context of the convenience wrappers.  Once torch has
    initialised the GPU it follows torch's current stream (hbg_set_stream
    orders the switch), so device tensors torch just wrote are ready for it
    and its results are ready for torch — no extra synchronisation."""
    global _default, _default_stream
    if _default is None:
        _default = Context()
    torch = sys.modules.get("torch")
    if torch is not None and torch.cuda.is_initialized():
        # the current stream of the context's device (not of torch's current device)
        h = torch.cuda.current_stream(_default.device).cuda_stream
        if h != _default_stream:
            _default.set_stream(h)
            _default_stream = h
    return _default


# ---- pure host helpers -------------------------------------------------------
def merkle_nodes(n: int) -> int:
    return lib().hbg_merkle_nodes(n)


def merkle_depth(n: int) -> int:
    return lib().hbg_merkle_depth(n)


def num_faulty(n: int) -> int:
    return lib().hbg_num_faulty(n)


def shard_len(n: int, payload_len: int) -> int:
    return lib().hbg_shard_len(n, payload_len)


def coding_matrix(data: int, parity: int) -> np.ndarray:
    out = np.zeros((data + parity, max(data, 1)), np.uint8)
    check(lib().hbg_coding_matrix(data, parity, ptr(out)), "hbg_coding_matrix")
    return out
