"""ctypes view of oracle/liborc_rbc.so (TEST INFRASTRUCTURE ONLY — see oracle/__init__.py).

The C restatement (oracle/c/rbc_oracle.c) is checked against the numpy oracle
and hashlib in tests/test_oracle_rbc.py, then used as the checker at large
sizes and as bench.py's cpu_baseline ("port").
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "liborc_rbc.so")
_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _SO


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        l = C.CDLL(_SO)
        u8p = C.POINTER(C.c_uint8)
        l.orc_rs_encode.argtypes = [C.c_uint32, C.c_uint32, C.c_uint64, u8p, C.c_uint64]
        l.orc_rs_reconstruct.argtypes = [C.c_uint32, C.c_uint32, C.c_uint64, u8p, C.c_uint64, u8p]
        l.orc_sha3_256.argtypes = [u8p, C.c_uint64, u8p]
        l.orc_sha3_256.restype = None
        l.orc_merkle_nodes.argtypes = [C.c_uint32]
        l.orc_merkle_nodes.restype = C.c_uint32
        l.orc_merkle_levels.argtypes = [C.c_uint32, C.c_uint64, u8p, C.c_uint64, u8p]
        l.orc_proof_validate.argtypes = [C.c_uint32, u8p, C.c_uint64, C.c_uint32, u8p, C.c_uint32, u8p]
        l.orc_synth_bytes.argtypes = [C.c_uint32, C.c_uint64, C.c_uint64, u8p]
        l.orc_synth_bytes.restype = None
        l.orc_shard_len.argtypes = [C.c_uint32, C.c_uint64]
        l.orc_shard_len.restype = C.c_uint64
        l.orc_rbc_encode_merkle.argtypes = [C.c_uint32, u8p, C.c_uint64, u8p, C.c_uint64, u8p]
        l.orc_rbc_decode.argtypes = [C.c_uint32, C.c_uint64, u8p, C.c_uint64, u8p, u8p, u8p,
                                     C.POINTER(C.c_uint64), u8p]
        l.orc_rbc_encode_merkle_batch.argtypes = [C.c_uint32, u8p, C.c_uint64, C.c_uint64, u8p,
                                                  C.c_uint64, u8p, C.c_int]
        l.orc_build_matrix.argtypes = [C.c_uint32, C.c_uint32, u8p]
        l.orc_simd_enabled.argtypes = []
        _lib = l
    return _lib


def _p(a: np.ndarray):
    assert a.dtype == np.uint8 and a.flags.c_contiguous
    return a.ctypes.data_as(C.POINTER(C.c_uint8))


def sha3(data: bytes) -> bytes:
    a = np.frombuffer(bytes(data), dtype=np.uint8).copy() if len(data) else np.zeros(1, np.uint8)
    out = np.zeros(32, np.uint8)
    lib().orc_sha3_256(_p(a), len(data), _p(out))
    return out.tobytes()


def build_matrix(D: int, Q: int) -> np.ndarray:
    m = np.zeros((D + Q, D), np.uint8)
    rc = lib().orc_build_matrix(D, Q, _p(m))
    assert rc == 0, rc
    return m


def rs_encode(D: int, Q: int, shards: np.ndarray) -> None:
    """shards: [N][stride] uint8, in place; L = stride."""
    rc = lib().orc_rs_encode(D, Q, shards.shape[1], _p(shards), shards.shape[1])
    assert rc == 0, rc


def rs_reconstruct(D: int, Q: int, shards: np.ndarray, present: np.ndarray) -> int:
    return lib().orc_rs_reconstruct(D, Q, shards.shape[1], _p(shards), shards.shape[1],
                                    _p(present.astype(np.uint8)))


def merkle_levels(shards: np.ndarray, L: int | None = None) -> np.ndarray:
    N, S = shards.shape
    L = S if L is None else L
    out = np.zeros((lib().orc_merkle_nodes(N), 32), np.uint8)
    lib().orc_merkle_levels(N, L, _p(shards), S, _p(out))
    return out


def synth_bytes(tag: int, instance: int, nbytes: int) -> np.ndarray:
    out = np.zeros(max(nbytes, 1), np.uint8)
    lib().orc_synth_bytes(tag, instance, nbytes, _p(out))
    return out[:nbytes]


def shard_len(N: int, P: int) -> int:
    return lib().orc_shard_len(N, P)


def rbc_encode_merkle(N: int, payload: np.ndarray, stride: int | None = None):
    P = payload.shape[0]
    L = shard_len(N, P)
    S = L if stride is None else stride
    shards = np.zeros((N, S), np.uint8)
    levels = np.zeros((lib().orc_merkle_nodes(N), 32), np.uint8)
    pl = payload if P else np.zeros(1, np.uint8)
    rc = lib().orc_rbc_encode_merkle(N, _p(pl), P, _p(shards), S, _p(levels))
    assert rc == 0, rc
    return shards, levels


def rbc_decode(N: int, L: int, shards: np.ndarray, present: np.ndarray, root: bytes):
    """Returns (status, payload bytes or None); shards modified in place."""
    out = np.zeros(max(shards.shape[0] * L, 4), np.uint8)
    ln = C.c_uint64(0)
    st = np.zeros(1, np.uint8)
    r = np.frombuffer(root, np.uint8).copy()
    rc = lib().orc_rbc_decode(N, L, _p(shards), shards.shape[1], _p(present.astype(np.uint8)), _p(r),
                              _p(out), C.byref(ln), _p(st))
    assert rc == 0, rc
    return (out[: ln.value].tobytes() if st[0] else None)


def rbc_encode_merkle_batch(N: int, payloads: np.ndarray, stride: int, threads: int):
    n, P = payloads.shape
    shards = np.zeros((n, N, stride), np.uint8)
    levels = np.zeros((n, lib().orc_merkle_nodes(N), 32), np.uint8)
    rc = lib().orc_rbc_encode_merkle_batch(N, _p(payloads), P, n, _p(shards), stride, _p(levels), threads)
    assert rc == 0, rc
    return shards, levels
