"""Drop-in mirror of threshold_crypto's ThresholdDecrypt surfaces over the gfx950 engine.

Same names, argument meaning and error behaviour as threshold_crypto [EXT]
as hbbft's ``ThresholdDecrypt`` uses it, reached from
``/root/reference/src/hydrabadger/state.rs:486-487``:

  Ciphertext(U, V, W).verify()                         -> hbg_ct_verify          (a12)
  PublicKeyShare.verify_decryption_share(share, ct)    -> hbg_tdec_verify_shares (a14)
  PublicKeySet.decrypt(shares, ct)                     -> hbg_tdec_combine       (a15, a16)
  ThresholdDecrypt (set_ciphertext, handle_message,
    try_output) for a whole epoch                      -> hbg_tdec_threshold_decrypt (a18)
  PublicKey.encrypt_with_r(msg, r)                     -> hbg_tdec_encrypt       (§8 f1)
  SecretKey.decrypt_share_no_verify(ct)                -> hbg_tdec_decrypt_shares (§8 f1)
  SecretKey.sign(msg) / PublicKey.verify(sig, msg)     -> hbg_bls_sign / hbg_bls_verify (§8 f2,
                                                          src/lib.rs:405-416, :434)
  PublicKeyShare.verify(sig_share, doc) (coin shares)  -> hbg_sig_verify_shares  (§8 f3 coin)
  combine_signatures(t, shares) (+ Signature::parity)  -> hbg_sig_combine        (§8 f3 coin)

Points are the crate's zcash-compressed bytes (G1 48 B, G2 96 B).  Every
computation runs in libhbgpu.so on the GPU; there is no CPU fallback.  The
``*_batch`` forms take whole epochs at once.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from . import _lib
from ._lib import HbgError, check, default_context, lib, ptr


class NotEnoughShares(HbgError):
    def __init__(self):
        RuntimeError.__init__(self, "NotEnoughShares")
        self.code = _lib.HBG_E_NOT_ENOUGH_SHARES


class DuplicateEntry(HbgError):
    pass


@dataclass
class Ciphertext:
    U: bytes  # G1, 48 B compressed
    V: bytes
    W: bytes  # G2, 96 B compressed

    def verify(self, ctx=None) -> bool:
        return bool(ct_verify_batch([self], ctx)[0])


def _ct_table(cts):
    n = len(cts)
    U = np.frombuffer(b"".join(bytes(c.U) for c in cts), np.uint8).copy().reshape(n, 48)
    W = np.frombuffer(b"".join(bytes(c.W) for c in cts), np.uint8).copy().reshape(n, 96)
    lens = [len(c.V) for c in cts]
    off = np.zeros(n + 1, np.uint64)
    off[1:] = np.cumsum(lens)
    V = np.frombuffer(b"".join(bytes(c.V) for c in cts) or b"\0", np.uint8).copy()
    return U, V, off, W


def ct_verify_batch(cts: list, ctx=None) -> np.ndarray:
    n = len(cts)
    if n == 0:
        return np.zeros(0, np.uint8)
    U, V, off, W = _ct_table(cts)
    ok = np.zeros(n, np.uint8)
    check(lib().hbg_ct_verify((ctx or default_context()).h, n, ptr(U), ptr(V), ptr(off), ptr(W), ptr(ok), 0),
          "Ciphertext::verify")
    return ok


def verify_shares_batch(cts: list, pk_shares: list, shares: list, ctx=None) -> np.ndarray:
    """shares: [(share48, ct_index, pk_index)] -> ok bits (one per share)."""
    n = len(shares)
    if n == 0:
        return np.zeros(0, np.uint8)
    U, V, off, W = _ct_table(cts)
    pk = np.frombuffer(b"".join(bytes(p) for p in pk_shares), np.uint8).copy().reshape(len(pk_shares), 48)
    sh = np.frombuffer(b"".join(bytes(s) for s, _, _ in shares), np.uint8).copy().reshape(n, 48)
    sct = np.array([c for _, c, _ in shares], np.uint32)
    spk = np.array([p for _, _, p in shares], np.uint32)
    ok = np.zeros(n, np.uint8)
    check(lib().hbg_tdec_verify_shares((ctx or default_context()).h, len(cts), ptr(U), ptr(V), ptr(off), ptr(W),
                                       len(pk_shares), ptr(pk), n, ptr(sh), ptr(sct), ptr(spk), ptr(ok), 0),
          "verify_decryption_share")
    return ok


@dataclass
class PublicKeyShare:
    pk: bytes  # 48 B compressed G1

    def verify_decryption_share(self, share: bytes, ct: Ciphertext, ctx=None) -> bool:
        return bool(verify_shares_batch([ct], [self.pk], [(share, 0, 0)], ctx)[0])


def combine_batch(t: int, cts: list, shares: list, ctx=None):
    """shares[k] = the first t+1 (index, share48) items for ciphertext k.
    Returns (plaintexts, status array)."""
    n = len(cts)
    m = t + 1
    for s in shares:
        if len(s) < m:
            raise NotEnoughShares()
    _, V, off, _ = _ct_table(cts)
    sh = np.frombuffer(b"".join(bytes(x) for s in shares for _, x in s[:m]), np.uint8).copy().reshape(n, m, 48)
    ix = np.array([[i for i, _ in s[:m]] for s in shares], np.uint32).reshape(n, m)
    out = np.zeros(max(int(off[-1]), 1), np.uint8)
    st = np.zeros(n, np.int32)
    check(lib().hbg_tdec_combine((ctx or default_context()).h, t, n, ptr(sh), ptr(ix), ptr(V), ptr(off), ptr(out),
                                 ptr(st), 0), "PublicKeySet::decrypt")
    return [out[int(off[k]):int(off[k + 1])].tobytes() for k in range(n)], st


@dataclass
class PublicKeySet:
    threshold: int

    def decrypt(self, shares, ct: Ciphertext, ctx=None) -> bytes:
        """shares: iterable of (node index, share48) in iterator order."""
        items = list(shares)
        if len(items) <= self.threshold:
            raise NotEnoughShares()
        pts, st = combine_batch(self.threshold, [ct], [items[: self.threshold + 1]], ctx)
        if st[0] == _lib.HBG_E_DUPLICATE_ENTRY:
            raise DuplicateEntry(int(st[0]), "PublicKeySet::decrypt")
        if st[0] != 0:
            raise HbgError(int(st[0]), "PublicKeySet::decrypt")
        return pts[0]


# --------------------------------------------------------------------------- a18: ThresholdDecrypt glue
SHARE_NONE, SHARE_ACCEPTED, SHARE_FAULTY, SHARE_IGNORED = (_lib.HBG_SHARE_NONE, _lib.HBG_SHARE_ACCEPTED,
                                                           _lib.HBG_SHARE_FAULTY, _lib.HBG_SHARE_IGNORED)
SHARE_REPEAT = _lib.HBG_SHARE_REPEAT  # flag: MultipleDecryptionShares
ARRIVAL_CIPHERTEXT = _lib.HBG_ARRIVAL_CIPHERTEXT  # arrival entry: set_ciphertext + start_decryption
ARRIVAL_OWN = _lib.HBG_ARRIVAL_OWN  # ARRIVAL_OWN | i: the same at validator node i (own share inserted)


def is_marker(s: int, n: int) -> bool:
    """An arrival entry at which set_ciphertext + start_decryption run."""
    return s == ARRIVAL_CIPHERTEXT or (s & ARRIVAL_OWN != 0 and (s & ~ARRIVAL_OWN) < n)


def threshold_decrypt_arrays(t: int, n_nodes: int, U, V, V_off, W, pk48, share48, arrival, plaintext, status,
                             outcome, ctx=None, device: bool = False, asynchronous: bool = False) -> None:
    """hbbft ThresholdDecrypt for a whole epoch (hbg_tdec_threshold_decrypt):
    U [n_ct][48], W [n_ct][96], V bytes at V_off [n_ct+1], pk48 [N][48],
    share48 [n_ct][N][48] (sender i's share of ct k at [k][i]), arrival
    [n_ct][A] u32 sender ids in arrival order (ARRIVAL_CIPHERTEXT marks the
    ciphertext's arrival; an entry >= N otherwise ends the list) or None
    (node order); outputs plaintext (V layout), status [n_ct] i32, outcome
    [n_ct][N] u8.  Host numpy arrays, or (device=True) CUDA tensors."""
    n_ct = U.shape[0]
    flags = (_lib.HBG_DEVICE if device else 0) | (_lib.HBG_ASYNC if asynchronous else 0)
    alen = 0 if arrival is None else int(arrival.shape[1])
    check(lib().hbg_tdec_threshold_decrypt((ctx or default_context()).h, t, n_nodes, n_ct, ptr(U), ptr(V),
                                           ptr(V_off), ptr(W), ptr(pk48), ptr(share48), ptr(arrival), alen,
                                           ptr(plaintext), ptr(status), ptr(outcome), flags), "ThresholdDecrypt")


def threshold_decrypt_batch(t: int, cts: list, pk_shares: list, shares: list, arrivals=None, ctx=None):
    """One node's ThresholdDecrypt instances for an epoch's ciphertexts:
    shares[k][i] = sender i's 48-B share of cts[k] (None: never sent);
    arrivals[k] = sender ids in arrival order, repeats allowed, with
    ARRIVAL_CIPHERTEXT where the ciphertext arrives at an observer or
    ARRIVAL_OWN | i where it arrives at validator node i (hbbft
    start_decryption inserts node i's own share before try_output) (None:
    every sender once in node order, after the ciphertext).  Returns (plaintexts (None where
    status != 0), status array, outcome [n_ct][N])."""
    n_ct, n = len(cts), len(pk_shares)
    if n_ct == 0:
        return [], np.zeros(0, np.int32), np.zeros((0, n), np.uint8)
    U, V, off, W = _ct_table(cts)
    pk = np.frombuffer(b"".join(bytes(p) for p in pk_shares), np.uint8).copy().reshape(n, 48)
    sh = np.zeros((n_ct, n, 48), np.uint8)
    sent = []
    for k in range(n_ct):
        order = list(range(n)) if arrivals is None or arrivals[k] is None else list(arrivals[k])
        end = next((j for j, i in enumerate(order) if i >= n and not is_marker(i, n)), len(order))
        sent.append([i for i in order[:end] if is_marker(i, n) or shares[k][i] is not None])  # >= n: the list's end
        for i in range(n):
            if shares[k][i] is not None:
                sh[k, i] = np.frombuffer(bytes(shares[k][i]), np.uint8)
    arr = None
    if arrivals is not None or any(x is None for row in shares for x in row):
        arr = np.full((n_ct, max(1, max(len(o) + 1 for o in sent))), 0xFFFFFFFF, np.uint32)
        for k, o in enumerate(sent):
            arr[k, :len(o)] = o
    pt = np.zeros(max(int(off[-1]), 1), np.uint8)
    st = np.zeros(n_ct, np.int32)
    oc = np.zeros((n_ct, n), np.uint8)
    threshold_decrypt_arrays(t, n, U, V, off, W, pk, sh, arr, pt, st, oc, ctx)
    pts = [pt[int(off[k]):int(off[k + 1])].tobytes() if st[k] == 0 else None for k in range(n_ct)]
    return pts, st, oc


def test_bls(op: int, inputs: np.ndarray, out_words: int, ctx=None) -> np.ndarray:
    """Unit-test hook (include/hbgpu_testing.h): inputs [n][in_words] u32."""
    inputs = np.ascontiguousarray(inputs, dtype=np.uint32)
    n, iw = inputs.shape
    out = np.zeros((n, out_words), np.uint32)
    check(lib().hbg_test_bls((ctx or default_context()).h, op, n, ptr(inputs), iw, ptr(out), out_words),
          "hbg_test_bls")
    return out


# --------------------------------------------------------------------------- SURVEY.md §8(f1), (f2)
def _scalar_bytes(k) -> bytes:
    """An Fr scalar as the C ABI's 32-byte little-endian integer (int or bytes)."""
    if isinstance(k, (bytes, bytearray)):
        if len(k) != 32:
            raise ValueError("scalar must be 32 bytes")
        return bytes(k)
    return int(k).to_bytes(32, "little")


def _msg_table(msgs):
    off = np.zeros(len(msgs) + 1, np.uint64)
    off[1:] = np.cumsum([len(m) for m in msgs])
    buf = np.frombuffer(b"".join(bytes(m) for m in msgs) or b"\0", np.uint8).copy()
    return buf, off


def encrypt_batch(pk48: bytes, msgs: list, rs: list, ctx=None) -> list:
    """PublicKey::encrypt_with_rng for each (msg, r) with the scalar r explicit
    (the crate draws it from the caller's RNG)."""
    n = len(msgs)
    if n == 0:
        return []
    buf, off = _msg_table(msgs)
    r = np.frombuffer(b"".join(_scalar_bytes(x) for x in rs), np.uint8).copy()
    pk = np.frombuffer(bytes(pk48), np.uint8).copy()
    U = np.zeros((n, 48), np.uint8)
    W = np.zeros((n, 96), np.uint8)
    V = np.zeros(max(int(off[-1]), 1), np.uint8)
    check(lib().hbg_tdec_encrypt((ctx or default_context()).h, ptr(pk), n, ptr(r), ptr(buf), ptr(off), ptr(U), ptr(V),
                                 ptr(W), 0), "PublicKey::encrypt_with_rng")
    return [Ciphertext(U[k].tobytes(), V[int(off[k]):int(off[k + 1])].tobytes(), W[k].tobytes()) for k in range(n)]


def decrypt_shares_batch(cts: list, sks: list, pairs: list, ctx=None):
    """SecretKeyShare::decrypt_share_no_verify for each (ct index, sk index):
    returns (share48 list, status array)."""
    n = len(pairs)
    if n == 0:
        return [], np.zeros(0, np.int32)
    U = np.frombuffer(b"".join(bytes(c.U) for c in cts), np.uint8).copy()
    sk = np.frombuffer(b"".join(_scalar_bytes(x) for x in sks), np.uint8).copy()
    sc = np.array([c for c, _ in pairs], np.uint32)
    ss = np.array([s for _, s in pairs], np.uint32)
    out = np.zeros((n, 48), np.uint8)
    st = np.zeros(n, np.int32)
    check(lib().hbg_tdec_decrypt_shares((ctx or default_context()).h, len(cts), ptr(U), len(sks), ptr(sk), n, ptr(sc),
                                        ptr(ss), ptr(out), ptr(st), 0), "decrypt_share_no_verify")
    return [out[k].tobytes() for k in range(n)], st


def sign_batch(sks: list, items: list, ctx=None) -> list:
    """SecretKey::sign: items = [(sk index, msg)] -> 96-B compressed signatures."""
    n = len(items)
    if n == 0:
        return []
    buf, off = _msg_table([m for _, m in items])
    sk = np.frombuffer(b"".join(_scalar_bytes(x) for x in sks), np.uint8).copy()
    ix = np.array([i for i, _ in items], np.uint32)
    sig = np.zeros((n, 96), np.uint8)
    check(lib().hbg_bls_sign((ctx or default_context()).h, len(sks), ptr(sk), n, ptr(ix), ptr(buf), ptr(off),
                             ptr(sig), 0), "SecretKey::sign")
    return [sig[k].tobytes() for k in range(n)]


def verify_sig_batch(pk48s: list, items: list, ctx=None) -> np.ndarray:
    """PublicKey::verify: items = [(pk index, msg, sig96)] -> ok bits."""
    n = len(items)
    if n == 0:
        return np.zeros(0, np.uint8)
    buf, off = _msg_table([m for _, m, _ in items])
    pk = np.frombuffer(b"".join(bytes(p) for p in pk48s), np.uint8).copy()
    ix = np.array([i for i, _, _ in items], np.uint32)
    sig = np.frombuffer(b"".join(bytes(s) for _, _, s in items), np.uint8).copy()
    ok = np.zeros(n, np.uint8)
    check(lib().hbg_bls_verify((ctx or default_context()).h, len(pk48s), ptr(pk), n, ptr(ix), ptr(buf), ptr(off),
                               ptr(sig), ptr(ok), 0), "PublicKey::verify")
    return ok


@dataclass
class SecretKey:
    """threshold_crypto SecretKey (also SecretKeyShare): an Fr scalar."""
    scalar: int

    def sign(self, msg: bytes, ctx=None) -> bytes:
        return sign_batch([self.scalar], [(0, msg)], ctx)[0]

    def decrypt_share_no_verify(self, ct: Ciphertext, ctx=None) -> bytes:
        shares, st = decrypt_shares_batch([ct], [self.scalar], [(0, 0)], ctx)
        if st[0] != 0:
            raise HbgError(int(st[0]), "decrypt_share_no_verify")
        return shares[0]


@dataclass
class PublicKey:
    pk: bytes  # G1, 48 B compressed

    def verify(self, sig: bytes, msg: bytes, ctx=None) -> bool:
        return bool(verify_sig_batch([self.pk], [(0, msg, sig)], ctx)[0])

    def encrypt_with_r(self, msg: bytes, r, ctx=None) -> Ciphertext:
        return encrypt_batch(self.pk, [msg], [r], ctx)[0]


# --------------------------------------------------------------------------- SURVEY.md §8(f3)
def verify_sig_shares_batch(pk48s: list, docs: list, items: list, ctx=None) -> np.ndarray:
    """PublicKeyShare::verify(sig_share, doc) for many signature shares:
    items = [(doc index, pk index, sig96)] -> ok bits (identical to
    verify_sig_batch on the same triples; hash_g2 once per document)."""
    n = len(items)
    if n == 0:
        return np.zeros(0, np.uint8)
    buf, off = _msg_table(docs)
    pk = np.frombuffer(b"".join(bytes(p) for p in pk48s), np.uint8).copy()
    sd = np.array([d for d, _, _ in items], np.uint32)
    sp = np.array([p for _, p, _ in items], np.uint32)
    sig = np.frombuffer(b"".join(bytes(s) for _, _, s in items), np.uint8).copy()
    ok = np.zeros(n, np.uint8)
    check(lib().hbg_sig_verify_shares((ctx or default_context()).h, len(docs), ptr(buf), ptr(off), len(pk48s), ptr(pk),
                                      n, ptr(sig), ptr(sd), ptr(sp), ptr(ok), 0), "PublicKeyShare::verify")
    return ok


def sig_combine_batch(t: int, shares: list, ctx=None):
    """PublicKeySet::combine_signatures + Signature::parity for many coins:
    shares[k] = the first t+1 (node index, 96-B signature share) items.
    Returns (signatures, parity bits, status array)."""
    n, m = len(shares), t + 1
    if n == 0:
        return [], np.zeros(0, np.uint8), np.zeros(0, np.int32)
    for s in shares:
        if len(s) < m:
            raise NotEnoughShares()
    sh = np.frombuffer(b"".join(bytes(x) for s in shares for _, x in s[:m]), np.uint8).copy()
    ix = np.array([[i for i, _ in s[:m]] for s in shares], np.uint32).reshape(n, m)
    sig = np.zeros((n, 96), np.uint8)
    par = np.zeros(n, np.uint8)
    st = np.zeros(n, np.int32)
    check(lib().hbg_sig_combine((ctx or default_context()).h, t, n, ptr(sh), ptr(ix), ptr(sig), ptr(par), ptr(st), 0),
          "PublicKeySet::combine_signatures")
    return [sig[k].tobytes() for k in range(n)], par, st


def combine_signatures(t: int, shares, ctx=None) -> tuple:
    """PublicKeySet::combine_signatures(shares) -> (signature96, parity)."""
    items = list(shares)
    if len(items) <= t:
        raise NotEnoughShares()
    sigs, par, st = sig_combine_batch(t, [items[: t + 1]], ctx)
    if st[0] == _lib.HBG_E_DUPLICATE_ENTRY:
        raise DuplicateEntry(int(st[0]), "PublicKeySet::combine_signatures")
    if st[0] != 0:
        raise HbgError(int(st[0]), "PublicKeySet::combine_signatures")
    return sigs[0], bool(par[0])
