"""threshold_crypto restatement (TEST INFRASTRUCTURE ONLY — see oracle/__init__.py).

Restates threshold_crypto [EXT, 0.3/0.4-era, unpinned] as hbbft's
ThresholdDecrypt uses it, reached from the
reference at /root/reference/src/hydrabadger/state.rs:486-487:

  Ciphertext(U: G1, V: bytes, W: G2); encrypt_with_rng; Ciphertext::verify;
  SecretKeyShare::decrypt_share_no_verify; PublicKeyShare::verify_decryption_share;
  PublicKeySet::decrypt -> interpolate(t, first t+1 shares) + xor_with_hash;
  hash_g2 / hash_g1_g2 (ChaChaRng-seeded try-and-increment G2 sampling).

``hash_g2`` is the version-dependent row: "parity unpinned" (DESIGN.md).
Randomness (r, polynomial coefficients) is an explicit argument here: the
reference draws it from an entropy-seeded StdRng (state.rs:480), so runs are
not reproducible there anyway; our harness seeds it.
"""
from __future__ import annotations

from dataclasses import dataclass

from . import bls12_381 as B
from .chacha import ChaChaRng
from .merkle import sha3

FQ_SHAVE_MASK = 0xFFFFFFFFFFFFFFFF >> 3


def _rand_fq(rng: ChaChaRng) -> int:
    """ff_derive ``Rand for Fq``: six next_u64 limbs (LE), top limb masked by
    3 shave bits, rejected unless < p, read as a MONTGOMERY representation."""
    while True:
        limbs = [rng.next_u64() for _ in range(6)]
        limbs[5] &= FQ_SHAVE_MASK
        repr_int = sum(l << (64 * i) for i, l in enumerate(limbs))
        if repr_int < B.P:
            return B.fq_from_mont_repr(repr_int)


def _rand_g2(rng: ChaChaRng):
    """pairing ``Rand for G2``: x = Fq2{c0, c1}, greatest = next_u32 & 1,
    get_point_from_x, scale_by_cofactor, retry on failure / identity."""
    while True:
        x = (_rand_fq(rng), _rand_fq(rng))
        greatest = (rng.next_u32() & 1) == 1
        p = B.g2_get_point_from_x(x, greatest)
        if p is not None:
            q = B.g2_scale_by_cofactor(p)
            if q is not None:
                return q


def hash_g2(msg: bytes):
    return _rand_g2(ChaChaRng(sha3(msg)))


def hash_g1_g2(g1, msg: bytes):
    m = sha3(msg) if len(msg) > 64 else bytes(msg)
    return hash_g2(m + B.g1_compress(g1))


def xor_with_hash(g1, data: bytes) -> bytes:
    rng = ChaChaRng(sha3(B.g1_compress(g1)))
    return bytes(b ^ (rng.next_u32() & 0xFF) for b in data)


@dataclass
class Ciphertext:
    U: tuple
    V: bytes
    W: tuple

    def verify(self) -> bool:
        h = hash_g1_g2(self.U, self.V)
        return B.pairing_check([(B.G1, self.W), (B.g1_neg(self.U), h)])


def encrypt(pk, msg: bytes, r: int) -> Ciphertext:
    """PublicKey::encrypt_with_rng with the scalar r given explicitly."""
    u = B.g1_mul(B.G1, r)
    v = xor_with_hash(B.g1_mul(pk, r), msg)
    w = B.g2_mul(hash_g1_g2(u, v), r)
    return Ciphertext(u, v, w)


def sign(sk: int, msg: bytes):
    """SecretKey::sign: hash_g2(msg) * sk (G2)."""
    return B.g2_mul(hash_g2(msg), sk)


def verify(pk, sig, msg: bytes) -> bool:
    """PublicKey::verify: e(pk, hash_g2(msg)) == e(G1, sig)."""
    return B.pairing_check([(pk, hash_g2(msg)), (B.g1_neg(B.G1), sig)])


def decrypt_share(sk_share: int, ct: Ciphertext):
    """SecretKeyShare::decrypt_share_no_verify: U * sk_i."""
    return B.g1_mul(ct.U, sk_share)


def verify_decryption_share(pk_share, share, ct: Ciphertext, h=None) -> bool:
    """PublicKeyShare::verify_decryption_share: e(share, H) == e(pk_i, W)."""
    h = hash_g1_g2(ct.U, ct.V) if h is None else h
    return B.pairing_check([(share, h), (B.g1_neg(pk_share), ct.W)])


class NotEnoughShares(Exception):
    pass


class DuplicateEntry(Exception):
    pass


def interpolate(t: int, items: list):
    """threshold_crypto ``interpolate``: first t+1 (index, G1) items, x = index+1,
    value at 0 of the Lagrange polynomial through them."""
    samples = [(i + 1, s) for i, s in items[: t + 1]]
    if len(samples) <= t:
        raise NotEnoughShares()
    xs = [x for x, _ in samples]
    if len(set(xs)) != len(xs):
        raise DuplicateEntry()
    if t == 0:
        return samples[0][1]
    acc = None
    for x, s in samples:
        num, den = 1, 1
        for x0 in xs:
            if x0 != x:
                num = num * x0 % B.R
                den = den * (x0 - x) % B.R
        lam = num * pow(den, -1, B.R) % B.R
        acc = B.g1_add(acc, B.g1_mul(s, lam))
    return acc


def interpolate_g2(t: int, items: list):
    """``interpolate`` over G2 samples (PublicKeySet::combine_signatures):
    first t+1 (index, G2) items, x = index+1, value at 0."""
    samples = [(i + 1, s) for i, s in items[: t + 1]]
    if len(samples) <= t:
        raise NotEnoughShares()
    xs = [x for x, _ in samples]
    if len(set(xs)) != len(xs):
        raise DuplicateEntry()
    if t == 0:
        return samples[0][1]
    acc = None
    for x, s in samples:
        num, den = 1, 1
        for x0 in xs:
            if x0 != x:
                num = num * x0 % B.R
                den = den * (x0 - x) % B.R
        acc = B.g2_add(acc, B.g2_mul(s, num * pow(den, -1, B.R) % B.R))
    return acc


def combine_signatures(t: int, shares: list):
    """PublicKeySet::combine_signatures(shares): shares = [(index, G2 sig share)]."""
    return interpolate_g2(t, shares)


def g2_uncompressed(pt) -> bytes:
    """zcash uncompressed G2 (192 B): x.c1 || x.c0 || y.c1 || y.c0 big-endian,
    flag bit 6 for the identity (bit 7, 'compressed', clear)."""
    if pt is None:
        out = bytearray(192)
        out[0] = 0x40
        return bytes(out)
    (x0, x1), (y0, y1) = pt
    return b"".join(v.to_bytes(48, "big") for v in (x1, x0, y1, y0))


def sig_parity(sig) -> bool:
    """Signature::parity (threshold_crypto [EXT], version-dependent — parity
    unpinned): XOR of all bytes of the uncompressed encoding, then the parity
    of that byte's number of ones — the hbbft common-coin bit."""
    x = 0
    for b in g2_uncompressed(sig):
        x ^= b
    return bin(x).count("1") % 2 == 1


def decrypt(t: int, shares: list, ct: Ciphertext) -> bytes:
    """PublicKeySet::decrypt(shares, ct): shares = [(index, G1)] in iterator order."""
    g = interpolate(t, shares)
    return xor_with_hash(g, ct.V)


class SecretKeySet:
    """Polynomial of degree t over Fr with explicit coefficients."""

    def __init__(self, coeffs: list):
        self.coeffs = [c % B.R for c in coeffs]

    @property
    def threshold(self) -> int:
        return len(self.coeffs) - 1

    def secret_key_share(self, i: int) -> int:
        x, acc = i + 1, 0
        for c in reversed(self.coeffs):
            acc = (acc * x + c) % B.R
        return acc

    def public_key(self):
        return B.g1_mul(B.G1, self.coeffs[0])

    def commitment(self) -> list:
        return [B.g1_mul(B.G1, c) for c in self.coeffs]


def public_key_share(commitment: list, i: int):
    """PublicKeySet::public_key_share(i) = commitment evaluated at i+1."""
    x = i + 1
    acc = None
    for c in reversed(commitment):
        acc = B.g1_add(B.g1_mul(acc, x) if acc is not None else None, c)
    return acc


# ----------------------------------------------------------------------------- a18: ThresholdDecrypt glue
SHARE_NONE, SHARE_ACCEPTED, SHARE_FAULTY, SHARE_IGNORED = 0, 1, 2, 3
SHARE_REPEAT = 4  # flag: FaultKind::MultipleDecryptionShares logged for the sender
ARRIVAL_CIPHERTEXT = 0xFFFFFFFE  # arrival entry: set_ciphertext + start_decryption happen here
ARRIVAL_OWN = 0x80000000  # ARRIVAL_OWN | i: the same at validator node i, which inserts its own share
E_NOT_ENOUGH_SHARES, E_INVALID_CIPHERTEXT = -20, -23


def threshold_decrypt(t: int, ct: Ciphertext, pk_shares: list, shares: list, arrival=None, cache=None):
    """One node's hbbft ThresholdDecrypt instance [EXT, hbbft
    src/threshold_decrypt.rs, recalled from upstream: parity unpinned],
    restated.

    arrival: sender ids in arrival order (None: 0..N-1 after the ciphertext);
    the list ends at the first entry >= N other than a marker.  The marker is
    the point at which HoneyBadger calls set_ciphertext + start_decryption (no
    marker: before the first arrival): ARRIVAL_CIPHERTEXT for an observer,
    ARRIVAL_OWN | i for validator node i, whose start_decryption inserts its
    own share (decrypt_share_no_verify: trusted, never verified) into the
    held map AFTER dropping the invalid held shares and BEFORE try_output.
      * handle_message before the ciphertext: the share is held unverified;
        a sender already held is replaced (same bytes here) and faulted
        (MultipleDecryptionShares -> SHARE_REPEAT flag);
      * set_ciphertext: an invalid ciphertext (Ciphertext::verify false) ends
        the instance (E_INVALID_CIPHERTEXT); start_decryption then removes
        the held shares that fail verify_decryption_share (node-id order,
        UnverifiedDecryptionShareSender -> SHARE_FAULTY; the others
        SHARE_ACCEPTED) and try_output fires if more than t are held;
      * handle_message after the ciphertext: an invalid share is a fault
        (SHARE_FAULTY); a valid one is held (SHARE_ACCEPTED), or, if the
        sender is already held, faulted as a repeat (SHARE_REPEAT flag);
        try_output fires when t+1 are held;
      * try_output terminates the instance and decrypts with the first t+1
        held shares in node-id order (BTreeMap); later arrivals are ignored
        unchecked (SHARE_IGNORED); fewer than t+1 valid shares:
        E_NOT_ENOUGH_SHARES.
    shares[i]: sender i's share (G1 point or None).  Returns (status,
    plaintext or None, outcome per sender).  cache: a dict shared by the
    instances of ONE ciphertext with the same shares (every node's own
    ThresholdDecrypt of it, oracle/epoch.py): verdicts and combinations are
    computed once (a memo of pure functions, not a change of semantics)."""
    if cache is None:
        cache = {}
    n = len(pk_shares)
    order = list(range(n)) if arrival is None else list(arrival)

    def is_marker(s):
        return s == ARRIVAL_CIPHERTEXT or (s & ARRIVAL_OWN and (s & ~ARRIVAL_OWN) < n)
    for j, s in enumerate(order):
        if s >= n and not is_marker(s):
            order = order[:j]
            break
    outcome = [SHARE_NONE] * n
    if "ct_ok" not in cache:
        cache["ct_ok"] = ct.verify()
        cache["h"] = hash_g1_g2(ct.U, ct.V) if cache["ct_ok"] else None
    ct_ok, h = cache["ct_ok"], cache["h"]

    def valid(s):
        if ("v", s) not in cache:
            cache[("v", s)] = shares[s] is not None and verify_decryption_share(pk_shares[s], shares[s], ct, h)
        return cache[("v", s)]

    ct_set = not any(is_marker(s) for s in order)
    if ct_set and not ct_ok:
        return E_INVALID_CIPHERTEXT, None, outcome
    pending, held, term = set(), set(), False
    for s in order:
        if is_marker(s):
            if ct_set:
                continue
            ct_set = True
            if not ct_ok:
                return E_INVALID_CIPHERTEXT, None, outcome
            for p in sorted(pending):
                if valid(p):
                    outcome[p] |= SHARE_ACCEPTED
                    held.add(p)
                else:
                    outcome[p] |= SHARE_FAULTY
            pending.clear()
            if s != ARRIVAL_CIPHERTEXT:  # our own share: inserted unverified (replacing a held one)
                own = s & ~ARRIVAL_OWN
                outcome[own] = (outcome[own] & SHARE_REPEAT) | SHARE_ACCEPTED
                held.add(own)
            term = len(held) >= t + 1
            continue
        if not ct_set:
            if s in pending:
                outcome[s] |= SHARE_REPEAT
            pending.add(s)
            continue
        base = outcome[s] & 3
        if term:
            if base == SHARE_NONE:
                outcome[s] |= SHARE_IGNORED
            continue
        if not valid(s):
            outcome[s] = (outcome[s] & SHARE_REPEAT) | SHARE_FAULTY
            continue
        if s in held:
            outcome[s] |= SHARE_REPEAT
            continue
        held.add(s)
        outcome[s] = (outcome[s] & SHARE_REPEAT) | SHARE_ACCEPTED
        term = len(held) == t + 1
    if not term:
        return E_NOT_ENOUGH_SHARES, None, outcome
    sel = tuple(sorted(held)[: t + 1])
    if ("d", sel) not in cache:
        cache[("d", sel)] = decrypt(t, [(i, shares[i]) for i in sel], ct)
    return 0, cache[("d", sel)], outcome
