"""ctypes view of oracle/liborc_bls.so (TEST INFRASTRUCTURE ONLY — see oracle/__init__.py).

The C restatement of the ThresholdDecrypt path (oracle/c/bls_oracle.c) is
checked against the Python oracle and the committed fixtures in
tests/test_oracle_tdec.py, then used as a fast checker and as bench.py's TDec
cpu_baseline ("port": threshold_crypto's per-share algorithm — hash_g1_g2 and
two full pairings per verify_decryption_share — one contiguous block of shares
per host thread).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "liborc_bls.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            subprocess.run(["make", "-s", "-C", _HERE], check=True)
        l = C.CDLL(_SO)
        vp = C.c_void_p
        l.orb_verify_share.argtypes = [vp, vp, vp, vp, C.c_uint64, vp]
        l.orb_verify_share.restype = C.c_int
        l.orb_ct_verify.argtypes = [vp, vp, C.c_uint64, vp]
        l.orb_ct_verify.restype = C.c_int
        l.orb_decrypt.argtypes = [C.c_uint32, vp, vp, vp, C.c_uint64, vp]
        l.orb_decrypt.restype = C.c_int
        l.orb_verify_shares_batch.argtypes = [C.c_int, C.c_uint64, vp, vp, vp, vp, C.c_uint64, vp, C.c_uint64, vp, vp, vp,
                                              vp]
        l.orb_verify_shares_batch.restype = None
        l.orb_decrypt_batch.argtypes = [C.c_int, C.c_uint32, C.c_uint64, vp, vp, vp, vp, vp, vp]
        l.orb_decrypt_batch.restype = None
        _lib = l
    return _lib


def _p(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


def _ct_table(cts):
    """cts: [(U48, V, W96)] bytes -> (U, V, V_off, W) numpy arrays."""
    U = np.frombuffer(b"".join(bytes(c[0]) for c in cts), np.uint8).copy()
    W = np.frombuffer(b"".join(bytes(c[2]) for c in cts), np.uint8).copy()
    V = np.frombuffer(b"".join(bytes(c[1]) for c in cts) + b"\0", np.uint8).copy()
    off = np.zeros(len(cts) + 1, np.uint64)
    off[1:] = np.cumsum([len(c[1]) for c in cts])
    return U, V, off, W


def verify_shares(cts, pk48s, items, threads: int = 1) -> np.ndarray:
    """items: [(share48, ct_index, pk_index)] -> ok bits."""
    U, V, off, W = _ct_table(cts)
    pk = np.frombuffer(b"".join(bytes(p) for p in pk48s), np.uint8).copy()
    n = len(items)
    sh = np.frombuffer(b"".join(bytes(s) for s, _, _ in items), np.uint8).copy()
    sct = np.array([c for _, c, _ in items], np.uint32)
    spk = np.array([p for _, _, p in items], np.uint32)
    ok = np.zeros(n, np.uint8)
    lib().orb_verify_shares_batch(threads, len(cts), _p(U), _p(V), _p(off), _p(W), len(pk48s), _p(pk), n, _p(sh), _p(sct),
                                  _p(spk), _p(ok))
    return ok


def verify_shares_arrays(threads, U, V, off, W, pk, sh, sct, spk) -> np.ndarray:
    """Array form (all numpy, contiguous) for the bench baseline."""
    n = len(sct)
    ok = np.zeros(n, np.uint8)
    lib().orb_verify_shares_batch(threads, len(off) - 1, _p(U), _p(V), _p(off), _p(W), len(pk) // 48, _p(pk), n, _p(sh),
                                  _p(sct), _p(spk), _p(ok))
    return ok


def ct_verify(U48: bytes, V: bytes, W96: bytes) -> bool:
    u, w = np.frombuffer(U48, np.uint8).copy(), np.frombuffer(W96, np.uint8).copy()
    v = np.frombuffer(bytes(V) + b"\0", np.uint8).copy()
    return bool(lib().orb_ct_verify(_p(u), _p(v), len(V), _p(w)))


def decrypt_batch(t: int, cts, shares, threads: int = 1):
    """shares[k] = [(index, share48)] (first t+1 used) -> (plaintexts, status)."""
    n, m = len(cts), t + 1
    _, V, off, _ = _ct_table(cts)
    sh = np.frombuffer(b"".join(bytes(x) for s in shares for _, x in s[:m]), np.uint8).copy()
    ix = np.array([[i for i, _ in s[:m]] for s in shares], np.uint32).reshape(n, m)
    out = np.zeros(max(int(off[-1]), 1), np.uint8)
    st = np.zeros(n, np.int32)
    lib().orb_decrypt_batch(threads, t, n, _p(sh), _p(ix), _p(V), _p(off), _p(out), _p(st))
    return [out[int(off[k]):int(off[k + 1])].tobytes() for k in range(n)], st


def decrypt_arrays(threads, t, sh, ix, V, off) -> tuple:
    n = len(off) - 1
    out = np.zeros(max(int(off[-1]), 1), np.uint8)
    st = np.zeros(n, np.int32)
    lib().orb_decrypt_batch(threads, t, n, _p(sh), _p(ix), _p(V), _p(off), _p(out), _p(st))
    return out, st
