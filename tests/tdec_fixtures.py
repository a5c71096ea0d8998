"""Seeded ThresholdDecrypt scenarios built with the oracle (test helper).

The reference draws keys and encryption randomness from an entropy-seeded
StdRng (/root/reference/src/hydrabadger/state.rs:480, key_gen.rs:193-200), so
no run of it is reproducible; our scenarios derive every scalar from the
SplitMix64 streams of SURVEY.md §8(d) (tag TAG_TDEC).
"""
from __future__ import annotations

from functools import lru_cache

from oracle import bls12_381 as B
from oracle import synth
from oracle import tcrypto as T


def _scalar(rng: synth.SplitMix64) -> int:
    v = 0
    for _ in range(4):
        v = (v << 64) | rng.next()
    return v % B.R


def limbs(v: int, n: int = 12) -> list:
    return [(v >> (32 * i)) & 0xFFFFFFFF for i in range(n)]


def from_limbs(ws) -> int:
    return sum(int(w) << (32 * i) for i, w in enumerate(ws))


@lru_cache(maxsize=None)
def scenario(n_nodes: int = 7, n_ct: int = 3, msg_len: int = 40, seed: int = 1):
    """Returns dict with keyset, public key shares, ciphertexts and all shares."""
    f = (n_nodes - 1) // 3
    rng = synth.SplitMix64(synth.TAG_TDEC, seed)
    ks = T.SecretKeySet([_scalar(rng) for _ in range(f + 1)])
    pk = ks.public_key()
    com = ks.commitment()
    pk_shares = [T.public_key_share(com, i) for i in range(n_nodes)]
    cts, msgs, shares = [], [], []
    for c in range(n_ct):
        msg = synth.synth_bytes(synth.TAG_TDEC, seed * 1000 + c, msg_len + 17 * c)
        ct = T.encrypt(pk, msg, _scalar(rng))
        cts.append(ct)
        msgs.append(msg)
        shares.append([T.decrypt_share(ks.secret_key_share(i), ct) for i in range(n_nodes)])
    return {"t": f, "ks": ks, "pk_shares": pk_shares, "cts": cts, "msgs": msgs, "shares": shares}
