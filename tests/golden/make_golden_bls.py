"""Regenerates tests/golden/bls_ops.json from the oracle (SURVEY.md §8(f1),
(f2)): SecretKey::sign / PublicKey::verify vectors for wire-message
signatures, PublicKey::encrypt_with_rng with explicit r, and
SecretKeyShare::decrypt_share_no_verify.  python tests/golden/make_golden_bls.py

No reference fixtures exist for these surfaces; these
pin the oracle's outputs (oracle/bls12_381.py, oracle/tcrypto.py) so the GPU
tests compare against fixed bytes.  Scalars are stored as 32-byte little-endian
hex (the C ABI's encoding)."""
import json
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import bls12_381 as B  # noqa: E402
from oracle import tcrypto as T  # noqa: E402


def le(k: int) -> str:
    return k.to_bytes(32, "little").hex()


def main():
    rng = random.Random(0x5167)
    sks = [rng.randrange(1, B.R) for _ in range(2)]
    msgs = [b"", b"hydrabadger wire message", bytes(rng.randrange(256) for _ in range(300))]
    sign = {"sk": [le(k) for k in sks], "pk": [B.g1_compress(B.g1_mul(B.G1, k)).hex() for k in sks],
            "items": [{"sk": i % 2, "msg": m.hex(), "sig": B.g2_compress(T.sign(sks[i % 2], m)).hex()}
                      for i, m in enumerate(msgs)]}
    pk_sk = rng.randrange(1, B.R)
    pk = B.g1_mul(B.G1, pk_sk)
    enc = {"pk": B.g1_compress(pk).hex(), "sk": le(pk_sk), "items": []}
    for m in (b"", bytes(rng.randrange(256) for _ in range(40)), bytes(rng.randrange(256) for _ in range(100))):
        r = rng.randrange(1, B.R)
        ct = T.encrypt(pk, m, r)
        enc["items"].append({"r": le(r), "msg": m.hex(), "U": B.g1_compress(ct.U).hex(), "V": ct.V.hex(),
                             "W": B.g2_compress(ct.W).hex(),
                             "share": B.g1_compress(T.decrypt_share(pk_sk, ct)).hex()})
    # §8(f3) common coin at N=7 t=2: signature shares of a nonce, their
    # combination (== the master key's signature) and its parity
    from tests.tdec_fixtures import scenario
    s = scenario()
    ks, t, n = s["ks"], s["t"], len(s["pk_shares"])
    coins = []
    for nonce in (b"coin epoch 0 round 0", b"coin epoch 7 round 3"):
        shares = [T.sign(ks.secret_key_share(i), nonce) for i in range(n)]
        sig = T.combine_signatures(t, [(i, shares[i]) for i in range(n)][1:1 + t + 1])
        assert sig == T.sign(ks.coeffs[0], nonce)
        coins.append({"doc": nonce.hex(), "shares": [B.g2_compress(x).hex() for x in shares],
                      "sig": B.g2_compress(sig).hex(), "parity": T.sig_parity(sig)})
    coin = {"t": t, "pk": B.g1_compress(ks.public_key()).hex(),
            "pk_shares": [B.g1_compress(p).hex() for p in s["pk_shares"]], "coins": coins}
    out = {"generator": "tests/golden/make_golden_bls.py", "sign": sign, "encrypt": enc, "coin": coin}
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "bls_ops.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
